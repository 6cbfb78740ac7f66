"""Algorithmic FP32 FLOP model of one humanoid step (mjx.step), for bench.py's roofline.

Counts the arithmetic the algorithm needs (an FMA is 2 FLOPs), not what the kernel issues: the
kernel runs one env per 64-lane wave and most of its VALU instructions have few active lanes, so
issued lane-FLOPs are many times this. Each term follows the stage of the reference pipeline it
models (mujoco/mjx/_src: smooth.py, collision_driver.py, constraint.py, solver.py, forward.py);
DESIGN.md lists the derivation. Sizes come from the compiled model, the solver statistics (active
contacts, rows, Newton iterations) from a forward pass over the benchmarked states.
"""
from __future__ import annotations


def cholesky(n: int) -> float:
    """Dense LL^T factor (n^3/3 FMAs) + forward and back substitution (2 n^2 FMAs)."""
    return 2.0 * (n ** 3 / 3.0 + 2.0 * n * n)


def step_flops(m, ncon: float, nefc: float, iters: float, ls_evals: float = 3.0, nact=None) -> dict:
    """FP32 FLOPs of one env-step, by stage. `m` is a CompiledModel (sizes only). `nact`: mean
    active rows per Newton Hessian (stats[3]); the Hessian counts only those rows, as the kernel
    computes only those (MJX's dense J'DJ multiplies the inactive rows by D = 0)."""
    nv, nb, nj, npair = m.nv, m.nbody, m.njnt, m.npair
    nh = nefc if nact is None else nact
    f = {}
    # kinematics: per joint local quaternion (sincos, qmul, 2 quat->mat, 2 mat-vec),
    # per body compose with the parent (qmul, quat->mat, 2 mat-vec), geom and site frames
    f["kinematics"] = 2.0 * (nj * 70 + nb * 60 + m.ngeom * 18 + m.nsite * 36)
    # com_pos / crb: cinert (two 3x3 products + parallel axis), cdof, subtree crb, M columns
    depth = 0.5 * nv  # mean ancestor-chain length of a dof (humanoid: 6 free + limb chains)
    f["crb_M"] = 2.0 * (nb * 70 + nv * 9 + nb * 10 * 4 + nv * (36 + 6 * depth))
    # rne (cvel, cacc by levels; body forces; subtree sums; dof projection), passive, actuation
    f["rne"] = 2.0 * (nb * (2 * 18 + 2 * 36 + 18 + 6 * 4) + nv * 8)
    # collision: every candidate pair (capsule-capsule dominates: ~120 FMAs)
    f["collision"] = 2.0 * npair * 120
    # constraint rows: contact Jacobians (4 pyramid rows x nv) + impedance + reference accel
    f["rows"] = 2.0 * (ncon * nv * 20 + nefc * (nv + 30))
    # smooth acceleration M^-1 qfrc_smooth and the implicit-integration solve
    f["factor_M"] = cholesky(nv)
    f["integrate"] = cholesky(nv) + 2.0 * nv * 4
    # Newton solver: warm-start costs (M q, J q for two candidates), then per iteration:
    # Hessian J'DJ (full nv x nv over the active rows), factor + solve, line search (M s, J s,
    # ls_evals evaluations of the rows), update (J'f, gradient)
    per_it = (2.0 * nv * nv * nh + cholesky(nv) + 2.0 * (nv * nv + nv * nefc + ls_evals * 4 * nefc)
              + 2.0 * (nv * nefc + 4 * nv))
    f["solver"] = 2.0 * 2 * (nv * nv + nv * nefc) + iters * per_it
    f["total"] = sum(f.values())
    return f


def env_post_flops(m) -> float:
    """single_step's reward / termination / observation (src/envs.py:347-492): rpy from the pelvis
    quaternion, the torso velocity rotated into the pelvis frame, distances, energy over the nu
    actuated dofs, the target features; ~500 FMAs."""
    return 2.0 * (60 + 2 * 9 + 30 + 4 * m.nu + 40 + 10 * 4 + m.nq + m.nv)


def env_step_flops(m, ncon: float, nefc: float, iters: float, nact=None, reset_frac: float = 0.0) -> dict:
    """FP32 FLOPs of one fused PPO env step (mjl_env_step, auto_reset = 1): the physics step at the
    rollout's own solver statistics, the env's reward / obs, and for the fraction `reset_frac` of envs
    that finish in a step, single_reset's forward pass (envs.py:108-113: a full forward without
    integration, from a standing pose; counted with the same statistics)."""
    f = dict(step_flops(m, ncon, nefc, iters, nact=nact))
    phys = f.pop("total")
    f["env_post"] = env_post_flops(m)
    fwd = phys - f["integrate"]
    f["auto_reset"] = reset_frac * (fwd + env_post_flops(m))
    f["total"] = phys + f["env_post"] + f["auto_reset"]
    return f


def vjp_replay_flops(m, ncon: float, nefc: float, iters: float, nact=None, unrolled: bool = False) -> dict:
    """FP32 FLOPs of one env-step VJP replayed from the tape (mjl_env_step_vjp_replay: reverse passes
    only, the forward's workspace and factors read back). Reverse mode of a bilinear operation costs
    two FMAs per forward FMA (a' += c' b, b' += c' a), so each smooth stage, the collision of the
    active contacts, the row construction and the integrator's solve count twice their forward
    (step_flops). The constraint solve: implicit, one solve with the taped factor of the converged
    Hessian (2 substitutions) plus the cotangents of M (an nv x nv outer product), J (nact x nv), D and
    aref, and the J^T products; unrolled (jax.grad through the iterations), twice each taped
    iteration's forward arithmetic."""
    nv = m.nv
    fw = step_flops(m, ncon, nefc, iters, nact=nact)
    nh = nefc if nact is None else nact
    f = {k: 2.0 * fw[k] for k in ("kinematics", "crb_M", "rne", "rows", "integrate")}
    f["collision"] = 2.0 * 2.0 * max(ncon, 1.0) * 120  # only active contacts carry cotangents
    f["factor_M"] = 2.0 * (2.0 * nv * nv) + 2.0 * nv * nv  # M^-1 solve reverse + M' outer product
    if unrolled:
        f["solver"] = 2.0 * fw["solver"]
    else:
        f["solver"] = 2.0 * (2.0 * nv * nv) + 2.0 * (nv * nv + 3 * nh * nv + 4 * nefc)
    f["env_post"] = 2.0 * env_post_flops(m)
    f["total"] = sum(f.values())
    return f


def mlp_dims(in_dim: int, layer_specs, out_dim: int):
    """[(K, N, activated)] of an MLP (src/networks.py:22-61): hidden (features, act) layers + a linear
    output layer of out_dim units."""
    dims, k = [], in_dim
    for feat, act in layer_specs:
        dims.append((k, int(feat), str(act).lower() not in ("linear", "none")))
        k = int(feat)
    dims.append((k, out_dim, False))
    return dims


def mlp_forward_flops(dims, out_tanh: bool = False) -> float:
    """FLOPs per row of one forward pass: 2 K N per Dense + bias N + tanh (counted as 1 FLOP per
    element: the algorithmic count, not the transcendental's instruction sequence)."""
    f = 0.0
    for i, (k, n, act) in enumerate(dims):
        f += 2.0 * k * n + n + (n if act or (out_tanh and i == len(dims) - 1) else 0)
    return f


def mlp_train_flops(dims, out_tanh: bool = False) -> float:
    """FLOPs per row of forward + backward (train_ppo.py value_and_grad through the MLP): the forward,
    then per layer dZ = dH (1 - H^2) (3 per element when activated), the weight gradient dZᵀ X (2 K N),
    the bias gradient (N) and dX = dZ W (2 K N, not for the first layer: the observations need none)."""
    f = mlp_forward_flops(dims, out_tanh)
    for i, (k, n, act) in enumerate(dims):
        tanh_here = act or (out_tanh and i == len(dims) - 1)
        f += (3.0 * n if tanh_here else 0.0) + 2.0 * k * n + n + (2.0 * k * n if i > 0 else 0.0)
    return f


def ppo_update_flops(obs_dim: int, act_dim: int, policy_specs, value_specs) -> dict:
    """Per minibatch row: both nets' forward + backward (train_ppo.py:204-252), the losses (log-prob,
    ratio, clip, entropy: ~12 FLOPs per action dimension; MSE 3) and Adam is per parameter, not per row
    (left out: 151K parameters x 2 nets x ~12 FLOPs per minibatch is < 0.1 % at 8,192 rows)."""
    pd = mlp_dims(obs_dim, policy_specs, act_dim)
    vd = mlp_dims(obs_dim, value_specs, 1)
    f = {"policy": mlp_train_flops(pd, out_tanh=True), "value": mlp_train_flops(vd), "losses": 12.0 * act_dim + 3.0}
    f["total"] = sum(f.values())
    return f


def policy_rollout_flops(obs_dim: int, act_dim: int, policy_specs) -> dict:
    """Per env per rollout step (the fused policy launch, mjl_policy_fwd): observation normalisation
    (3 per input), the MLP forward with the mean's tanh, and the Gaussian head (sample, log-prob: ~8
    per action dimension)."""
    d = mlp_dims(obs_dim, policy_specs, act_dim)
    f = {"normalise": 3.0 * obs_dim, "mlp": mlp_forward_flops(d, out_tanh=True), "head": 8.0 * act_dim}
    f["total"] = sum(f.values())
    return f

"""Step adjoint (APG backward; reference train_apg.py:161-209 differentiates through mjx.step).

Reference derivative: the exact Jacobian of the fp64 oracle step by forward-mode dual numbers
(oracle/dual.hpp), itself pinned against central finite differences (CPU test below). MJX's own
gradients are unavailable here (no jax): parity unpinned against MJX.

HIP VJP vs the dual-number Jacobian: for random output cotangents u, the HIP result g = u' J must
match within |g - g_ref| <= tol * (|g_ref| + |u| |J| 1e-3) per input group, tol 2e-3 (fp32 kernel,
solver differentiated at its converged active set vs differentiated Newton iterates in fp64).
"""
import numpy as np
import pytest

import mjx_amd
from mjx_amd import abi
from mjx_amd.config import reference_ppo_config
from mjx_amd.envs import obs_size, resolve_ids
from oracle import Oracle, state_arrays

MODELS = ["humanoid_mjx", "humanoid"]


def _states(m, n, seed):
    """fp32-representable states with contacts / limits active: random poses near qpos0, a few
    oracle steps so the feet touch, plus random ctrl."""
    rng = np.random.default_rng(seed)
    o = Oracle(m)
    out = []
    for i in range(n):
        q = m.qpos0.copy()
        q[7:] += rng.uniform(-0.25, 0.25, m.nq - 7)
        q[2] += rng.uniform(-0.12, 0.0)
        s = o.new_state(q, rng.uniform(-0.5, 0.5, m.nv), ctrl=rng.uniform(-1, 1, m.nu))
        o.rollout(s, rng.uniform(-1, 1, (int(rng.integers(1, 15)), m.nu)))
        a = state_arrays(m, s)
        out.append(tuple(np.float32(x).astype(np.float64)
                         for x in (a["qpos"], a["qvel"], a["qacc_warmstart"], rng.uniform(-1, 1, m.nu))))
    return out


@pytest.mark.parametrize("name", MODELS)
def test_dual_jacobian_matches_central_differences(name):
    m = mjx_amd.load_model(name)
    o = Oracle(m)
    nq, nv, nu = m.nq, m.nv, m.nu
    for q, v, w, c in _states(m, 2, 1):
        J = o.step_jacobian(o.new_state(q, v, w, c))

        def F(x):
            a = state_arrays(m, o.step(o.new_state(x[:nq], x[nq:nq + nv], w, x[nq + nv:])))
            return np.concatenate([a["qpos"], a["qvel"]])

        x0 = np.concatenate([q, v, c])
        eps = 1e-6
        Jfd = np.stack([(F(x0 + eps * e) - F(x0 - eps * e)) / (2 * eps) for e in np.eye(len(x0))], 1)
        assert np.abs(J - Jfd).max() <= 1e-5 * (1 + np.abs(Jfd).max())


def _rel_err(g, ref, scale):
    return np.abs(g - ref).max() / (np.abs(ref).max() + scale)


@pytest.mark.gpu
@pytest.mark.parametrize("name", MODELS)
def test_step_vjp_matches_dual_jacobian(name):
    import torch
    from mjx_amd import mjx
    m = mjx_amd.load_model(name)
    o = Oracle(m)
    sts = _states(m, 12, 2)
    B, nq, nv, nu = len(sts), m.nq, m.nv, m.nu
    sys_ = mjx.put_model(m)
    d = mjx.make_data(sys_, B)
    t = lambda i: torch.tensor(np.array([s[i] for s in sts]), dtype=torch.float32)  # noqa: E731
    for k, i in (("qpos", 0), ("qvel", 1), ("qacc_warmstart", 2), ("ctrl", 3)):
        d.set(k, t(i))
    rng = np.random.default_rng(3)
    gq = rng.normal(size=(B, nq)).astype(np.float32)
    gv = rng.normal(size=(B, nv)).astype(np.float32)
    oq, ov, oc = (x.cpu().numpy() for x in mjx.step_vjp(sys_, d, torch.tensor(gq), torch.tensor(gv)))
    errs = []
    for i, (q, v, w, c) in enumerate(sts):
        J = o.step_jacobian(o.new_state(q, v, w, c))
        u = np.concatenate([gq[i], gv[i]]).astype(np.float64)
        ref = u @ J
        scale = 1e-3 * np.abs(u).max() * np.abs(J).max()
        e = [_rel_err(oq[i], ref[:nq], scale), _rel_err(ov[i], ref[nq:nq + nv], scale),
             _rel_err(oc[i], ref[nq + nv:], scale)]
        errs.append(e)
    errs = np.array(errs)
    assert errs.max() <= 2e-3, f"relative VJP errors (qpos, qvel, ctrl) per state:\n{errs}"


@pytest.mark.gpu
def test_env_step_vjp_matches_dual_jacobian():
    import torch
    from mjx_amd import mjx
    from mjx_amd.envs import HumanoidEnv
    m = mjx_amd.load_model("humanoid_mjx")
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    cfg_c = abi.env_config_c(cfg, m, obs_size(m.nq, m.nv))
    o = Oracle(m)
    B, nq, nv, nu, na = 10, m.nq, m.nv, m.nu, abi.AUX_DIM
    rng = np.random.default_rng(4)
    env = HumanoidEnv(mjx.put_model(m), cfg, B, seed=5)
    nd = nq - 7 + nv + 2
    noise = rng.uniform(0, 1, (B, nd)).astype(np.float32)
    env.reset(noise=torch.tensor(noise))
    for _ in range(3):  # a few steps so contacts, stance state and the potential are non-trivial
        env.step(torch.tensor(rng.uniform(-1, 1, (B, nu)).astype(np.float32)), auto_reset=False)
    qpos, qvel = env.data.get("qpos").cpu().numpy(), env.data.get("qvel").cpu().numpy()
    qws, aux = env.data.get("qacc_warmstart").cpu().numpy(), env.aux.cpu().numpy()
    tm = env.data.get("time").cpu().numpy()
    act = rng.uniform(-1.2, 1.2, (B, nu)).astype(np.float32)
    gq, gv = rng.normal(size=(B, nq)).astype(np.float32), rng.normal(size=(B, nv)).astype(np.float32)
    gr = rng.normal(size=B).astype(np.float32)
    ga = rng.normal(size=(B, na)).astype(np.float32)
    oq, ov, oa, oaux = (x.cpu().numpy() for x in env.step_vjp(torch.tensor(act), torch.tensor(gq), torch.tensor(gv),
                                                              torch.tensor(gr), torch.tensor(ga)))
    errs = []
    for i in range(B):
        s = o.new_state(qpos[i].astype(np.float64), qvel[i].astype(np.float64), qws[i].astype(np.float64),
                        time=float(tm[i]))
        J = o.env_step_jacobian(cfg_c, s, aux[i].astype(np.float64), act[i].astype(np.float64))
        u = np.concatenate([gq[i], gv[i], [gr[i]], ga[i]]).astype(np.float64)
        ref = u @ J
        scale = 1e-3 * np.abs(u).max() * np.abs(J).max()
        errs.append([_rel_err(oq[i], ref[:nq], scale), _rel_err(ov[i], ref[nq:nq + nv], scale),
                     _rel_err(oa[i], ref[nq + nv:nq + nv + nu], scale), _rel_err(oaux[i], ref[nq + nv + nu:], scale)])
    errs = np.array(errs)
    assert errs.max() <= 2e-3, f"relative VJP errors (qpos, qvel, action, aux) per state:\n{errs}"


def _truncated(name, solver, it, ls):
    from mjx_amd import mjcf
    m = mjx_amd.load_model(name)
    m.solver = mjcf.SOLVER_CG if solver == "cg" else mjcf.SOLVER_NEWTON
    m.iterations, m.ls_iterations = it, ls
    return m


def _step_vjp_errors(m, sts, unrolled, seed=3):
    import torch
    from mjx_amd import mjx
    o = Oracle(m)
    B, nq, nv = len(sts), m.nq, m.nv
    sys_ = mjx.put_model(m)
    d = mjx.make_data(sys_, B)
    d.set_option(abi.OPT_VJP_UNROLLED, int(unrolled))
    t = lambda i: torch.tensor(np.array([s[i] for s in sts]), dtype=torch.float32)  # noqa: E731
    for k, i in (("qpos", 0), ("qvel", 1), ("qacc_warmstart", 2), ("ctrl", 3)):
        d.set(k, t(i))
    rng = np.random.default_rng(seed)
    gq = rng.normal(size=(B, nq)).astype(np.float32)
    gv = rng.normal(size=(B, nv)).astype(np.float32)
    oq, ov, oc = (x.cpu().numpy() for x in mjx.step_vjp(sys_, d, torch.tensor(gq), torch.tensor(gv)))
    errs = []
    for i, (q, v, w, c) in enumerate(sts):
        J = o.step_jacobian(o.new_state(q, v, w, c))
        u = np.concatenate([gq[i], gv[i]]).astype(np.float64)
        ref = u @ J
        scale = 1e-3 * np.abs(u).max() * np.abs(J).max()
        errs.append(max(_rel_err(oq[i], ref[:nq], scale), _rel_err(ov[i], ref[nq:nq + nv], scale),
                        _rel_err(oc[i], ref[nq + nv:], scale)))
    return np.array(errs)


@pytest.mark.gpu
@pytest.mark.parametrize("solver,it,ls", [("cg", 4, 4), ("newton", 1, 4)])
def test_unrolled_step_vjp_matches_dual_jacobian_of_truncated_step(solver, it, ls):
    """MJL_OPT_VJP_UNROLLED under train_apg.py's CG 4/4 (and Newton 1/4): the VJP equals u' J with
    J the dual-number Jacobian of the oracle's truncated step (the derivative jax.grad takes through
    MJX's fixed-count iterations), where the implicit mode (converged-set derivative) does not."""
    m = _truncated("humanoid_mjx", solver, it, ls)
    sts = _states(mjx_amd.load_model("humanoid_mjx"), 16, 5)  # states from converged rollouts
    unr = _step_vjp_errors(m, sts, True)
    imp = _step_vjp_errors(m, sts, False)
    print(f"\n{solver} {it}/{ls} unrolled:", np.round(unr, 5), "\nimplicit:", np.round(imp, 5))
    assert np.median(unr) <= 1e-3 and unr.max() <= 2e-2, unr
    assert np.median(imp) > 10 * np.median(unr), (unr, imp)  # the implicit derivative is not this one


@pytest.mark.gpu
@pytest.mark.parametrize("solver,it,ls", [("cg", 4, 4), ("newton", 1, 4)])
def test_unrolled_step_vjp_full_matches_dual_jacobian_with_warm_start(solver, it, ls):
    """mjl_step_vjp_full: with the carried warm start as state (input and output), the unrolled VJP
    equals u' J_ws, J_ws the dual-number Jacobian of (qpos', qvel', qacc_warmstart') in (qpos, qvel,
    qacc_warmstart, ctrl) of the oracle's truncated step."""
    import torch
    from mjx_amd import mjx
    m = _truncated("humanoid_mjx", solver, it, ls)
    sts = _states(mjx_amd.load_model("humanoid_mjx"), 12, 6)
    o = Oracle(m)
    B, nq, nv = len(sts), m.nq, m.nv
    sys_ = mjx.put_model(m)
    d = mjx.make_data(sys_, B)
    d.set_option(abi.OPT_VJP_UNROLLED, 1)
    t = lambda i: torch.tensor(np.array([s[i] for s in sts]), dtype=torch.float32)  # noqa: E731
    for k, i in (("qpos", 0), ("qvel", 1), ("qacc_warmstart", 2), ("ctrl", 3)):
        d.set(k, t(i))
    rng = np.random.default_rng(9)
    gq, gv, gw = (rng.normal(size=(B, n)).astype(np.float32) for n in (nq, nv, nv))
    oq, ov, ow, oc = (x.cpu().numpy() for x in mjx.step_vjp_full(sys_, d, torch.tensor(gq), torch.tensor(gv),
                                                                 torch.tensor(gw)))
    errs = []
    for i, (q, v, w, c) in enumerate(sts):
        J = o.step_jacobian_ws(o.new_state(q, v, w, c))
        u = np.concatenate([gq[i], gv[i], gw[i]]).astype(np.float64)
        ref = u @ J
        scale = 1e-3 * np.abs(u).max() * np.abs(J).max()
        errs.append(max(_rel_err(oq[i], ref[:nq], scale), _rel_err(ov[i], ref[nq:nq + nv], scale),
                        _rel_err(ow[i], ref[nq + nv:nq + 2 * nv], scale), _rel_err(oc[i], ref[nq + 2 * nv:], scale)))
    errs = np.array(errs)
    print(f"\n{solver} {it}/{ls} unrolled, with warm start:", np.round(errs, 5))
    assert np.median(errs) <= 1e-3 and errs.max() <= 2e-2, errs


@pytest.mark.gpu
def test_unrolled_env_step_vjp_matches_dual_jacobian_cg44():
    """The env step (reward, aux, obs-relevant state) under CG 4/4 with the unrolled VJP, against the
    oracle env step's dual-number Jacobian (states from a converged rollout of the same env)."""
    import torch
    from mjx_amd import mjx
    from mjx_amd.envs import HumanoidEnv
    m0 = mjx_amd.load_model("humanoid_mjx")
    m = _truncated("humanoid_mjx", "cg", 4, 4)
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    cfg_c = abi.env_config_c(cfg, m, obs_size(m.nq, m.nv))
    o = Oracle(m)
    B, nq, nv, nu, na = 12, m.nq, m.nv, m.nu, abi.AUX_DIM
    rng = np.random.default_rng(14)
    env0 = HumanoidEnv(mjx.put_model(m0), cfg, B, seed=5)
    env0.reset(noise=torch.tensor(rng.uniform(0, 1, (B, nq - 7 + nv + 2)).astype(np.float32)))
    for _ in range(3):
        env0.step(torch.tensor(rng.uniform(-1, 1, (B, nu)).astype(np.float32)), auto_reset=False)
    env = HumanoidEnv(mjx.put_model(m), cfg, B, seed=5)
    env.set_state(env0.get_state())
    env.data.set_option(abi.OPT_VJP_UNROLLED, 1)
    qpos, qvel = env.data.get("qpos").cpu().numpy(), env.data.get("qvel").cpu().numpy()
    qws, aux = env.data.get("qacc_warmstart").cpu().numpy(), env.aux.cpu().numpy()
    tm = env.data.get("time").cpu().numpy()
    act = rng.uniform(-1.2, 1.2, (B, nu)).astype(np.float32)
    gq, gv = rng.normal(size=(B, nq)).astype(np.float32), rng.normal(size=(B, nv)).astype(np.float32)
    gr = rng.normal(size=B).astype(np.float32)
    ga = rng.normal(size=(B, na)).astype(np.float32)
    oq, ov, oa, oaux = (x.cpu().numpy() for x in env.step_vjp(torch.tensor(act), torch.tensor(gq), torch.tensor(gv),
                                                              torch.tensor(gr), torch.tensor(ga)))
    errs = []
    for i in range(B):
        s = o.new_state(qpos[i].astype(np.float64), qvel[i].astype(np.float64), qws[i].astype(np.float64),
                        time=float(tm[i]))
        J = o.env_step_jacobian(cfg_c, s, aux[i].astype(np.float64), act[i].astype(np.float64))
        u = np.concatenate([gq[i], gv[i], [gr[i]], ga[i]]).astype(np.float64)
        ref = u @ J
        scale = 1e-3 * np.abs(u).max() * np.abs(J).max()
        errs.append(max(_rel_err(oq[i], ref[:nq], scale), _rel_err(ov[i], ref[nq:nq + nv], scale),
                        _rel_err(oa[i], ref[nq + nv:nq + nv + nu], scale), _rel_err(oaux[i], ref[nq + nv + nu:], scale)))
    errs = np.array(errs)
    print("\nunrolled env-step VJP errors:", np.round(errs, 5))
    assert np.median(errs) <= 1e-3 and errs.max() <= 2e-2, errs


@pytest.mark.gpu
def test_unrolled_vjp_refused_beyond_tape_capacity():
    """the unrolled solve's tape holds 64 line-search points per search (a zoom search
    creates up to 1 + 2 ls_iterations); a model with more (humanoid.xml: Newton 100/50) is refused at
    mjl_batch_set_option instead of overwriting tape entries (a silently wrong gradient)."""
    from mjx_amd import mjx
    from mjx_amd._lib import MjlError
    m = mjx_amd.load_model("humanoid")
    assert m.ls_iterations > 31
    d = mjx.make_data(mjx.put_model(m), 4)
    with pytest.raises(MjlError, match="ls_iterations"):
        d.set_option(abi.OPT_VJP_UNROLLED, 1)
    d.set_option(abi.OPT_VJP_UNROLLED, 0)  # the implicit VJP stays available
    m2 = _truncated("humanoid", "cg", 4, 31)
    mjx.make_data(mjx.put_model(m2), 4).set_option(abi.OPT_VJP_UNROLLED, 1)  # 63 points fit

"""APG trainer (mjx_amd/apg.py): the tape + reverse-sweep gradient equals autograd through the whole
rollout (CPU, differentiable stand-in env); data-parallel ranks stay identical (gloo, world size 2);
on the GPU, the gradient of the real humanoid rollout loss matches fp64 oracle finite differences."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

from mjx_amd import apg
from mjx_amd.config import APGConfig


class DiffPointEnv:
    """Differentiable stand-in with the HumanoidAPGEnv interface: qpos (3), qvel (3), action (2);
    reward = -|qpos|^2 - 0.1 |a|^2; terminates when |qpos_z| > 1.5."""

    def __init__(self, num_envs, seed=0):
        self.num_envs, self.act_dim, self.nq, self.nv = num_envs, 2, 3, 3
        self.g = torch.Generator().manual_seed(seed)
        self.q = torch.zeros(num_envs, 3, dtype=torch.float64)
        self.v = torch.zeros(num_envs, 3, dtype=torch.float64)

    @staticmethod
    def f(q, v, a):
        acc = torch.stack([a[:, 0], a[:, 1], -0.5 * a[:, 0] * a[:, 1]], 1) - 0.3 * v - torch.sin(q)
        v2 = v + 0.1 * acc
        q2 = q + 0.1 * v2
        r = -(q * q).sum(1) - 0.1 * (a * a).sum(1)
        return q2, v2, r

    def reset(self):
        self.q = torch.rand((self.num_envs, 3), generator=self.g, dtype=torch.float64) - 0.5
        self.v = torch.zeros(self.num_envs, 3, dtype=torch.float64)

    def step(self, act, auto_reset=False):
        self.q, self.v, r = self.f(self.q, self.v, act.double())
        term = (self.q[:, 2].abs() > 1.5).double()
        return None, r, term, torch.zeros_like(term)

    def qpos_qvel(self):
        return torch.cat([self.q, self.v], 1)

    def get_state(self):
        return (self.q.clone(), self.v.clone())

    def set_state(self, st, warm_from=None):
        self.q, self.v = st[0].clone(), st[1].clone()

    def step_vjp(self, act, gq, gv, grew, gaux, nonfinite=None):
        q = self.q.clone().requires_grad_(True)
        v = self.v.clone().requires_grad_(True)
        a = act.double().clone().requires_grad_(True)
        q2, v2, r = self.f(q, v, a)
        torch.autograd.backward([q2, v2, r], [gq.double(), gv.double(), grew.double()])
        return q.grad, v.grad, a.grad, None


def _cfg(**kw):
    c = APGConfig()
    c.batch_size, c.horizon, c.hidden_size, c.hidden_depth = 8, 6, 16, 2
    c.obs_warmup_steps, c.rms_update_every, c.lr = 1, 1, 1e-3
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_reverse_sweep_equals_autograd_through_rollout():
    cfg = _cfg()
    env = DiffPointEnv(cfg.batch_size, 0)
    tr = apg.APGTrainer(cfg, env, device="cpu")
    tr.policy.double()
    tr.rms.mean = torch.randn(6, dtype=torch.float64) * 0.1
    tr.rms.var = torch.rand(6, dtype=torch.float64) + 0.5
    loss, _, _, _ = tr.loss_and_grad(use_norm=True)
    g_sweep = [p.grad.clone() for p in tr.policy.parameters()]
    # the same loss built as one autograd graph
    env2 = DiffPointEnv(cfg.batch_size, 0)
    env2.reset()
    tr.policy.zero_grad()
    q, v = env2.q, env2.v
    disc = torch.ones(cfg.batch_size, dtype=torch.float64)
    ret = torch.zeros(cfg.batch_size, dtype=torch.float64)
    for _ in range(cfg.horizon):
        a = tr.policy(apg.apg_normalize(tr.rms, torch.cat([q, v], 1)))
        q, v, r = DiffPointEnv.f(q, v, a)
        ret = ret + disc * r
        disc = disc * cfg.gamma * (1.0 - (q[:, 2].abs() > 1.5).double())
    (-ret.mean()).backward()
    assert float(loss) == pytest.approx(float(-ret.mean()), rel=1e-12)
    for a, b in zip(g_sweep, [p.grad for p in tr.policy.parameters()]):
        torch.testing.assert_close(a, b, rtol=1e-9, atol=1e-12)


def test_update_clips_global_norm():
    cfg = _cfg(grad_clip=1e-3, lr=1.0)
    tr = apg.APGTrainer(cfg, DiffPointEnv(cfg.batch_size, 1), device="cpu")
    tr.policy.double()
    before = [p.detach().clone() for p in tr.policy.parameters()]
    m = tr.update(0)
    assert m["grad_norm"] > 1e-3 and np.isfinite(m["loss"])
    # Adam's first step moves each coordinate by ~lr regardless of scale; the clipped gradient is what
    # the optimiser saw: check its norm
    g = torch.cat([p.grad.reshape(-1) for p in tr.policy.parameters()])
    assert float(g.norm()) == pytest.approx(1e-3, rel=1e-6)
    assert any(not torch.equal(a, b) for a, b in zip(before, tr.policy.parameters()))


class _WideStartEnv(DiffPointEnv):
    """DiffPointEnv whose resets start some envs past the termination bound (|q_z| > 1.5)."""

    def reset(self):
        super().reset()
        self.q = self.q * 6.0


@pytest.mark.parametrize("in_loss_only", [True, False])
def test_obs_statistics_from_in_loss_observations(in_loss_only):
    """cfg.rms_in_loss_only: the running observation statistics take only the observations of envs
    still in the loss at that step; a terminated env's later (here: diverged) observations stay out."""
    from mjx_amd.ppo import RunningMeanStd
    cfg = _cfg(rms_in_loss_only=in_loss_only)
    tr = apg.APGTrainer(cfg, _WideStartEnv(cfg.batch_size, 2), device="cpu")
    tr.policy.double()
    out = tr.loss_and_grad(use_norm=False)
    obs, mask = out[2]
    assert obs.shape == (cfg.horizon, cfg.batch_size, 6) and mask.shape == (cfg.horizon, cfg.batch_size)
    assert bool(mask[0].all()) and 0 < int(mask.sum()) < mask.numel()
    obs = obs.clone()
    obs[~mask.bool()] = 1e12  # a fallen env diverging after it left the loss
    tr.loss_and_grad = lambda use_norm, per_step_param_grad=False: (out[0], out[1], (obs, mask), out[3])
    tr.update(0)
    keep = mask.reshape(-1).bool() if in_loss_only else torch.ones(mask.numel(), dtype=torch.bool)
    ref = RunningMeanStd(6, torch.device("cpu"))
    ref.update(obs.reshape(-1, 6)[keep])
    torch.testing.assert_close(tr.rms.mean, ref.mean)
    torch.testing.assert_close(tr.rms.var, ref.var)
    assert (float(tr.rms.var.max()) < 1e3) == in_loss_only


def test_obs_statistics_freeze_after():
    """cfg.rms_freeze_after = N (opt-in): the observation statistics update every rms_update_every
    updates up to update N and never after."""
    cfg = _cfg(rms_update_every=1, rms_freeze_after=1)
    tr = apg.APGTrainer(cfg, DiffPointEnv(cfg.batch_size, 3), device="cpu")
    tr.policy.double()
    counts = []
    for step in range(4):
        tr.update(step)
        counts.append(float(tr.rms.count))
    assert counts[1] > counts[0] and counts[2] == counts[1] and counts[3] == counts[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=2)
    cfg = _cfg()
    tr = apg.APGTrainer(cfg, DiffPointEnv(cfg.batch_size, 10 + rank), device="cpu", dist=tdist)
    tr.policy.double()
    tr.train(3, verbose=False)
    torch.save(torch.cat([p.detach().reshape(-1) for p in tr.policy.parameters()]), out[rank])
    tdist.destroy_process_group()


def test_data_parallel_ranks_stay_identical(tmp_path):
    out = [str(tmp_path / "r0.pt"), str(tmp_path / "r1.pt")]
    mp.spawn(_dp_worker, args=(_port(), out), nprocs=2, join=True)
    a, b = torch.load(out[0], weights_only=True), torch.load(out[1], weights_only=True)
    torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("solver,vjp", [("model", "implicit"), ("cg44", "unrolled")])
def test_humanoid_apg_gradient_matches_oracle_finite_differences(solver, vjp):
    """d loss / d theta along a random direction: GPU tape + VJP sweep vs central differences of the
    same rollout on the fp64 oracle (same reset draws, policy in float64). With train_apg.py's CG
    4/4 the unrolled VJP is the derivative of the truncated rollout the finite differences see."""
    import mjx_amd
    from mjx_amd import abi, mjcf, mjx
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, obs_size, resolve_ids
    from oracle import Oracle, state_arrays
    m = mjx_amd.load_model("humanoid_mjx")
    if solver == "cg44":
        m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
    ecfg = resolve_ids(m, reference_ppo_config().env_config)
    # truncated CG amplifies fp32 rounding step over step (the fp32 and fp64 oracles part within a
    # few steps, tools/cg_parity_probe.py), so its rollout is kept shorter and the bounds looser
    cfg = _cfg(batch_size=4, horizon=5 if solver == "model" else 3, hidden_size=16)
    tol_loss, tol_grad = (1e-3, 2e-2) if solver == "model" else (5e-3, 5e-2)
    B, H = cfg.batch_size, cfg.horizon
    nd = m.nq - 7 + m.nv + 2
    noise = np.random.default_rng(7).uniform(0, 1, (B, nd)).astype(np.float32)
    henv = HumanoidEnv(mjx.put_model(m), ecfg, B, seed=3)

    class FixedReset(apg.HumanoidAPGEnv):
        def reset(self):
            return self.env.reset(noise=torch.tensor(noise))

    tr = apg.APGTrainer(cfg, FixedReset(henv, vjp), device="cuda")
    loss_gpu, _, _, _ = tr.loss_and_grad(use_norm=False)
    params = list(tr.policy.parameters())
    grad = torch.cat([p.grad.reshape(-1) for p in params]).double().cpu()
    d = torch.randn(grad.numel(), generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    pol64 = [p.detach().double().cpu() for p in params]
    cfg_c = abi.env_config_c(ecfg, m, obs_size(m.nq, m.nv))
    o = Oracle(m)

    def loss64(theta):
        ws, o_ = [], 0
        for p in pol64:
            ws.append(theta[o_:o_ + p.numel()].view_as(p))
            o_ += p.numel()
        total = 0.0
        for i in range(B):
            s, aux, _ = o.env_reset(cfg_c, noise[i].astype(np.float64))
            disc, ret = 1.0, 0.0
            for _ in range(H):
                a_ = state_arrays(m, s)
                x = torch.tensor(np.concatenate([a_["qpos"], a_["qvel"]]), dtype=torch.float64)
                for k in range(0, len(ws) - 2, 2):
                    x = torch.tanh(x @ ws[k].T + ws[k + 1])
                act = torch.tanh(x @ ws[-2].T + ws[-1]).numpy()
                s, aux, _, r, te, tu = o.env_step(cfg_c, s, aux, act)
                ret += disc * r
                disc *= cfg.gamma * (1.0 - max(te, tu))
            total += ret
        return -total / B

    def dloss64(theta, dvec):
        """Directional derivative of loss64 by forward mode along the rollout: the oracle env step's
        dual-number Jacobian (its branch decisions fixed, as jax.grad has them) chained with the
        float64 policy's JVP. Finite differences cannot resolve it for a truncated solve: a line-search
        or activity decision flips within +-eps somewhere in the rollout."""
        nq, nv, na = m.nq, m.nv, abi.AUX_DIM

        def pol(th, x):
            ws_, o_ = [], 0
            for p in pol64:
                ws_.append(th[o_:o_ + p.numel()].view_as(p))
                o_ += p.numel()
            for k in range(0, len(ws_) - 2, 2):
                x = torch.tanh(x @ ws_[k].T + ws_[k + 1])
            return torch.tanh(x @ ws_[-2].T + ws_[-1])

        total = 0.0
        for i in range(B):
            s, aux, _ = o.env_reset(cfg_c, noise[i].astype(np.float64))
            # the reset does not depend on theta; the carried warm start is state too (Data carry)
            tx, tws, taux = np.zeros(nq + nv), np.zeros(nv), np.zeros(na)
            disc, dret = 1.0, 0.0
            for _ in range(H):
                a_ = state_arrays(m, s)
                x = torch.tensor(np.concatenate([a_["qpos"], a_["qvel"]]), dtype=torch.float64)
                act, dact = torch.func.jvp(pol, (theta, x), (dvec, torch.tensor(tx)))
                act, dact = act.numpy(), dact.numpy()
                J = o.env_step_jacobian_ws(cfg_c, s, aux, act)
                s, aux, _, r, te, tu = o.env_step(cfg_c, s, aux, act)
                dout = J @ np.concatenate([tx, tws, dact, taux])
                tx, tws = dout[:nq + nv], dout[nq + nv:nq + 2 * nv]
                dr, taux = dout[nq + 2 * nv], dout[nq + 2 * nv + 1:]
                dret += disc * dr
                disc *= cfg.gamma * (1.0 - max(te, tu))
            total += dret
        return -total / B

    theta = torch.cat([p.reshape(-1) for p in pol64])
    an = float(grad @ d)
    assert abs(float(loss_gpu) - loss64(theta)) <= tol_loss * (1 + abs(loss64(theta)))
    if solver == "model":
        eps = 1e-5
        ref = (loss64(theta + eps * d) - loss64(theta - eps * d)) / (2 * eps)
    else:
        ref = dloss64(theta, d)
    assert an == pytest.approx(ref, rel=tol_grad, abs=1e-3)


@pytest.mark.gpu
def test_packed_state_roundtrip_and_guarded_vjp():
    """mjl_get_state / mjl_set_state restore every persistent field (with the warm-start override);
    the guarded VJP zeroes and counts exactly the env whose cotangents are non-finite and leaves the
    others equal to the unguarded VJP."""
    import mjx_amd
    from mjx_amd import mjx
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    m = mjx_amd.load_model("humanoid_mjx")
    B = 8
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, reference_ppo_config().env_config), B, seed=2)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(5):
        env.step(torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1, auto_reset=False)
    st = env.get_state().clone()
    fields = {f: env.data.get(f).clone() for f in ("qpos", "qvel", "qacc_warmstart", "aux", "time")}
    assert st.shape == (B, m.nq + 2 * m.nv + 9 + 1)
    env.step(torch.zeros((B, m.nu), device="cuda"), auto_reset=False)
    other = env.get_state().clone()
    env.set_state(st)
    for f, v in fields.items():
        assert torch.equal(env.data.get(f), v), f
    env.set_state(st, other)
    assert torch.equal(env.data.get("qacc_warmstart"), other[:, m.nq + m.nv:m.nq + 2 * m.nv])
    env.set_state(st)
    act = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
    gq, gv, gr = torch.randn((B, m.nq), device="cuda"), torch.randn((B, m.nv), device="cuda"), torch.randn(B, device="cuda")
    ref = env.step_vjp(act, gq, gv, gr)
    gq2 = gq.clone()
    gq2[3, 0] = float("nan")
    cnt = torch.zeros(1, device="cuda")
    out = env.step_vjp(act, gq2, gv, gr, None, cnt)
    assert float(cnt) == 1.0
    keep = torch.arange(B, device="cuda") != 3
    for a, b in zip(out, ref):
        assert torch.all(a[3] == 0) and torch.equal(a[keep], b[keep])


@pytest.mark.gpu
@pytest.mark.parametrize("solver,vjp", [("model", "implicit"), ("cg44", "unrolled")])
def test_apg_graph_replay_bit_identical_to_eager(solver, vjp):
    """The hipGraph replay of the APG rollout + reverse sweep (APGTrainer use_graph) gives the eager
    call's loss, gradient and parameters bit for bit, update after update, through both
    observation-normalisation graphs (warm-up call, capture, replays) and the per-update reset draws
    (device counter base)."""
    import mjx_amd
    from mjx_amd import mjcf, mjx
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    m = mjx_amd.load_model("humanoid_mjx")
    if solver == "cg44":
        m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
    ecfg = resolve_ids(m, reference_ppo_config().env_config)
    cfg = _cfg(batch_size=64, horizon=8, hidden_size=32)
    trs = [apg.APGTrainer(cfg, apg.HumanoidAPGEnv(HumanoidEnv(mjx.put_model(m), ecfg, cfg.batch_size, seed=3), vjp),
                          device="cuda", use_graph=g) for g in (False, True)]
    for step in range(6):
        ms = [tr.update(step) for tr in trs]
        for k in ("loss", "grad_norm", "mean_reward", "nonfinite_envs"):
            assert ms[0][k] == ms[1][k] or (ms[0][k] != ms[0][k] and ms[1][k] != ms[1][k]), f"update {step}: {k}"
        for p, q in zip(trs[0].policy.parameters(), trs[1].policy.parameters()):
            assert torch.equal(p, q), f"update {step}: parameters"
        assert torch.equal(trs[0].rms.mean, trs[1].rms.mean)
    assert set(trs[1]._graphs) == {True} and trs[0]._graphs == {}


@pytest.mark.gpu
@pytest.mark.parametrize("solver,vjp", [("model", "implicit"), ("cg44", "unrolled")])
def test_apg_native_bookkeeping_matches_torch_ops(solver, vjp):
    """The native per-step bookkeeping (mjl_apg_obs / mjl_apg_post / mjl_apg_obs_vjp) gives the same
    loss, gradient, dropped-env count and parameters as the torch-op restatement of the same sweep
    (_loss_and_grad_torch), with and without observation normalisation."""
    import mjx_amd
    from mjx_amd import mjcf, mjx
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    m = mjx_amd.load_model("humanoid_mjx")
    if solver == "cg44":
        m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
    ecfg = resolve_ids(m, reference_ppo_config().env_config)
    cfg = _cfg(batch_size=64, horizon=8, hidden_size=32)
    envs = [apg.HumanoidAPGEnv(HumanoidEnv(mjx.put_model(m), ecfg, cfg.batch_size, seed=3), vjp) for _ in range(2)]
    envs[1].native_apg = False
    # both recompute the step in the VJP (the tape's replay is pinned against that in test_vjp_tape.py;
    # the implicit recompute here starts from the forward's solution, so it differs from it by ~1e-4)
    trs = [apg.APGTrainer(cfg, e, device="cuda", use_graph=False, vjp_tape=False) for e in envs]
    for step in range(3):
        ms = [tr.update(step) for tr in trs]
        assert ms[0]["nonfinite_envs"] == ms[1]["nonfinite_envs"]
        for k in ("loss", "grad_norm", "mean_reward"):
            assert ms[0][k] == pytest.approx(ms[1][k], rel=1e-5, abs=1e-6), f"update {step}: {k}"
        for p, q in zip(trs[0].policy.parameters(), trs[1].policy.parameters()):
            torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_apg_native_sweep_matches_pure_torch_restatement():
    """The native sweep (native bookkeeping + the native policy's per-step passes, mjl_small_mlp_fwd /
    mjl_small_mlp_bwd_input) against the torch restatement with the policy in torch too (native_policy =
    None: torch GEMMs, autograd for the input cotangent), so the native policy is checked independently.
    Newton 10/20 (converged solves, implicit VJP), 64 envs x 8 steps, 3 updates: the two policies round
    their GEMMs differently, so loss / gradient norm / parameters agree to 1e-4, not bit for bit."""
    import mjx_amd
    from mjx_amd import mjx
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    m = mjx_amd.load_model("humanoid_mjx")
    ecfg = resolve_ids(m, reference_ppo_config().env_config)
    cfg = _cfg(batch_size=64, horizon=8, hidden_size=32)
    envs = [apg.HumanoidAPGEnv(HumanoidEnv(mjx.put_model(m), ecfg, cfg.batch_size, seed=3), "implicit")
            for _ in range(2)]
    envs[1].native_apg = False
    trs = [apg.APGTrainer(cfg, e, device="cuda", use_graph=False, vjp_tape=False) for e in envs]
    assert trs[0].native_policy is not None
    trs[1].native_policy = None
    for step in range(3):
        ms = [tr.update(step) for tr in trs]
        assert ms[0]["nonfinite_envs"] == ms[1]["nonfinite_envs"]
        for k in ("loss", "grad_norm", "mean_reward"):
            assert ms[0][k] == pytest.approx(ms[1][k], rel=1e-4, abs=1e-5), f"update {step}: {k}"
        for p, q in zip(trs[0].policy.parameters(), trs[1].policy.parameters()):
            torch.testing.assert_close(p, q, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_apg_fused_obs_policy_launches_bit_identical(monkeypatch, graph):
    """The fused per-step launches (mjl_apg_obs_policy_fwd, mjl_apg_policy_bwd_obs_vjp) against the pairs
    they replace (MJL_APG_FUSED_OBS=0): loss, gradient, returns and parameters bit for bit over 4 updates
    on the taped sweep (the first without observation normalisation, the rest with it), eager and under
    the update's hipGraph."""
    import mjx_amd
    from mjx_amd import mjx
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    m = mjx_amd.load_model("humanoid_mjx")
    ecfg = resolve_ids(m, reference_ppo_config().env_config)
    cfg = _cfg(batch_size=100, horizon=8, hidden_size=32)
    envs = [apg.HumanoidAPGEnv(HumanoidEnv(mjx.put_model(m), ecfg, cfg.batch_size, seed=5), "implicit")
            for _ in range(2)]
    trs = [apg.APGTrainer(cfg, e, device="cuda", use_graph=graph) for e in envs]
    assert all(tr.native_policy is not None for tr in trs)
    for step in range(4):
        ms = []
        for tr, fused in zip(trs, ("1", "0")):
            monkeypatch.setenv("MJL_APG_FUSED_OBS", fused)
            ms.append(tr.update(step))
        for k in ("loss", "grad_norm", "mean_reward", "return", "nonfinite_envs"):
            assert ms[0][k] == ms[1][k], f"update {step}: {k}"
        for p, q in zip(trs[0].policy.parameters(), trs[1].policy.parameters()):
            assert torch.equal(p, q), f"update {step}"


@pytest.mark.gpu
@pytest.mark.parametrize("nxt", ["1", "0"])
@pytest.mark.parametrize("solver,vjp", [("cg44", "implicit"), ("model", "implicit"), ("cg44", "unrolled")])
@pytest.mark.parametrize("graph", [False, True])
def test_apg_fused_record_post_bit_identical(monkeypatch, graph, solver, vjp, nxt):
    """The record + post-step update as one launch (mjl_env_step_record_apg), with (nxt = "1") the next
    step's observation + policy forward in it too (mjl_env_step_record_apg_next) and the policy +
    observation backward in the replay (mjl_env_step_vjp_replay_apg), against the record, mjl_apg_post,
    mjl_apg_obs_policy_fwd and mjl_apg_policy_bwd_obs_vjp as separate launches (MJL_APG_FUSED_POST=0 and
    MJL_APG_FUSED_BWD=0 on the second trainer): loss, gradient,
    returns, cut envs and parameters bit for bit over 4 updates (the first without observation
    normalisation), eager and under the update's hipGraph; with a divergence bound low enough that some
    envs are cut by it."""
    monkeypatch.setenv("MJL_APG_FUSED_NEXT", nxt)
    import mjx_amd
    from mjx_amd import mjcf, mjx
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    m = mjx_amd.load_model("humanoid_mjx")
    if solver == "cg44":
        m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
    ecfg = resolve_ids(m, reference_ppo_config().env_config)
    cfg = _cfg(batch_size=100, horizon=8, hidden_size=32)
    cfg.diverge_qvel = 5.0
    envs = [apg.HumanoidAPGEnv(HumanoidEnv(mjx.put_model(m), ecfg, cfg.batch_size, seed=5), vjp)
            for _ in range(2)]
    trs = [apg.APGTrainer(cfg, e, device="cuda", use_graph=graph) for e in envs]
    cut = 0.0
    for step in range(4):
        ms = []
        for tr, fused in zip(trs, ("1", "0")):
            monkeypatch.setenv("MJL_APG_FUSED_POST", fused)
            monkeypatch.setenv("MJL_APG_FUSED_BWD", nxt if fused == "1" else "0")
            ms.append(tr.update(step))
        for k in ("loss", "grad_norm", "mean_reward", "return", "nonfinite_envs"):
            assert ms[0][k] == ms[1][k], f"update {step}: {k}"
        cut += float(ms[0]["nonfinite_envs"])
        for p, q in zip(trs[0].policy.parameters(), trs[1].policy.parameters()):
            assert torch.equal(p, q), f"update {step}"
    assert cut > 0, "the divergence bound should cut some envs"


@pytest.mark.gpu
@pytest.mark.parametrize("k0,hidden,depth,act_dim,B", [(55, 32, 2, 21, 2048), (55, 64, 3, 21, 1000), (7, 16, 1, 3, 5)])
def test_native_apg_policy_matches_torch(k0, hidden, depth, act_dim, B):
    """mjl_small_mlp_fwd / mjl_small_mlp_bwd_input against the APGPolicy's torch forward and the
    autograd input cotangent (float64 reference): outputs to 2e-6, input cotangent to 1e-5 of its scale."""
    from mjx_amd.ppo import APGPolicy
    pol = APGPolicy(k0, act_dim, hidden, depth, None, torch.Generator().manual_seed(k0 + B)).cuda()
    assert apg.NativeAPGPolicy.eligible(pol, "cuda")
    nat = apg.NativeAPGPolicy(pol)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn((B, k0), generator=g, device="cuda") * 2
    ga = torch.randn((B, act_dim), generator=g, device="cuda")
    ys = [torch.empty((B, n), device="cuda") for n in nat.widths]
    a = nat.forward(x, ys)
    gx = nat.backward_input(ga, ys)
    pol64 = APGPolicy(k0, act_dim, hidden, depth).cuda().double()
    pol64.load_state_dict({k: v.double() for k, v in pol.state_dict().items()})
    x64 = x.double().requires_grad_(True)
    a64 = pol64(x64)
    gx64, = torch.autograd.grad(a64, x64, grad_outputs=ga.double())
    torch.testing.assert_close(a.double(), a64, rtol=0, atol=2e-6)
    torch.testing.assert_close(gx.double(), gx64, rtol=0, atol=1e-5 * float(gx64.abs().max()))
    ys2 = [torch.empty_like(y) for y in ys]
    assert torch.equal(nat.forward(x, ys2), a) and torch.equal(nat.backward_input(ga, ys2), gx)  # deterministic

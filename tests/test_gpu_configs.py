"""BASELINE configs run at their own sizes on the MI355X (VERDICT r1 "configs not exercised"), plus
the reference-shaped env functions, evaluation and the qpos-history dump.

* C3: PPOTrainer iterations at src/config.json values with 1024 envs x 256 steps x 4 epochs x
  minibatch 65,536 (train_ppo.py:320-441): finite metrics, metrics.jsonl keys, and the captured
  rollout graph replays the eager rollout bit for bit at that size, and its first 25 steps of six
  envs that do not finish match the oracle env (rewards, done flags, observations) from the state
  each env entered the rollout with, under the rollout's sampled actions.
* C4: one APG update at 2048 envs x 128 steps with train_apg.py's CG 4/4 override and the unrolled
  VJP (jax.grad semantics): finite loss and gradient (diverging envs leave the loss, DESIGN.md
  "Truncated solves"); the batched parameter gradient equals the per-step accumulation.
* A17: evaluate() at 32 envs x 500 deterministic steps with the reference's key chain, against the
  same loop run here step by step, and its first steps against the oracle env.
"""
import json
import os

import numpy as np
import pytest
import torch

import mjx_amd
from mjx_amd import abi, mjcf, mjx
from mjx_amd._lib import MjlError
from mjx_amd.config import APGConfig, EnvConfig, reference_ppo_config
from mjx_amd.envs import HumanoidEnv, create_env_functions, obs_size, resolve_ids
from oracle import Oracle, state_arrays

pytestmark = pytest.mark.gpu


def _humanoid():
    m = mjx_amd.load_model("humanoid_mjx")
    return m, mjx.put_model(m)


def test_create_env_functions_reference_shape():
    """(single_reset, single_step, v_reset, v_step) with the reference's arguments: v_reset(keys)
    equals the oracle env reset from the same jax.random draws; v_step equals the oracle env step."""
    from mjx_amd import jaxrng
    from rng_ref import jax_reset_noise
    m, sys_ = _humanoid()
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    single_reset, single_step, v_reset, v_step = create_env_functions(sys_, cfg, m.qpos0, m.nq, m.nv)
    B = 4
    keys = jaxrng.split(jaxrng.prng_key(5), B)
    state, obs = v_reset(keys)
    assert obs.shape == (B, obs_size(m.nq, m.nv)) and state.aux.shape == (B, abi.AUX_DIM)
    noise = jax_reset_noise(keys.cpu().numpy().view(np.uint32), m.nq - 7, m.nv, jaxrng.PARTITIONABLE)
    cfg_c = abi.env_config_c(cfg, m, obs_size(m.nq, m.nv))
    o = Oracle(m)
    ost = [list(o.env_reset(cfg_c, noise[i].astype(np.float64))[:2]) for i in range(B)]
    for i in range(B):
        assert np.abs(state.data.get("qpos").cpu().numpy()[i] - state_arrays(m, ost[i][0])["qpos"]).max() < 1e-6
    rng = np.random.default_rng(1)
    for _ in range(3):
        act = rng.uniform(-1, 1, (B, m.nu)).astype(np.float32)
        state, obs, rew, term, trunc = v_step(state, torch.tensor(act, device="cuda"))
        for i in range(B):
            s, oa, oo, r, te, tr = o.env_step(cfg_c, ost[i][0], ost[i][1], act[i].astype(np.float64))
            ost[i][1] = oa
            assert float(rew[i]) == pytest.approx(r, abs=5e-3 * (1 + abs(r)))
            np.testing.assert_allclose(obs[i].cpu().numpy(), oo, atol=5e-3 * (1 + np.abs(oo).max()))
            assert (float(term[i]), float(trunc[i])) == (te, tr)
    st1, ob1 = single_reset(keys[0])
    assert ob1.shape == (obs_size(m.nq, m.nv),)
    _, ob2, r2, _, _ = single_step(st1, torch.zeros(m.nu, device="cuda"))
    assert ob2.shape == ob1.shape and r2.dim() == 0
    with pytest.raises(MjlError):
        create_env_functions(sys_, cfg, m.qpos0, m.nq + 1, m.nv)


def test_ppo_c3_iterations_at_full_size(tmp_path):
    from mjx_amd import ppo
    m, sys_ = _humanoid()
    cfg = reference_ppo_config()
    cfg.num_envs, cfg.rollout_length = 1024, 256
    assert (cfg.epochs, cfg.minibatch_size, cfg.gamma, cfg.lam) == (4, 65536, 0.99, 0.95)
    ecfg = resolve_ids(m, cfg.env_config)
    env = HumanoidEnv(sys_, ecfg, cfg.num_envs, seed=11)
    tr = ppo.PPOTrainer(cfg, env, None, device="cuda", out_dir=str(tmp_path / "run"))
    for it in range(3):  # eager rollout, the capturing rollout, a replay
        met = tr.iteration(it)
        tr.log(it, met)
        assert all(np.isfinite(v) for v in met.values()), met
        assert met["env_steps_per_sec"] > 1e5
    for p in list(tr.policy.parameters()) + list(tr.value.parameters()):
        assert torch.isfinite(p).all()
    lines = [json.loads(x) for x in open(tmp_path / "run" / "logs" / "metrics.jsonl")]
    assert [x["step"] for x in lines] == [0, 1, 2]
    for k in ("train_return_avg", "train_return_max", "train_eplen_avg", "env_steps_per_sec", "total_env_steps",
              "elapsed_time"):
        assert k in lines[-1]
    assert lines[-1]["total_env_steps"] == 3 * 1024 * 256
    assert json.load(open(tmp_path / "run" / "config.json"))["minibatch_size"] == 65536
    # graph replay == eager loop at C3 size: same state, RNG and noise in both
    env2 = HumanoidEnv(sys_, ecfg, cfg.num_envs, seed=11)
    tr2 = ppo.PPOTrainer(cfg, env2, None, device="cuda", use_graph=False)
    for a in ("policy", "value"):
        getattr(tr2, a).load_state_dict(getattr(tr, a).state_dict())
    tr2.rms.load_state_dict(tr.rms.state_dict())
    env2.set_state(env.get_state())
    env2.counter = env.counter
    tr2.obs = tr.obs.clone()
    tr2.gen.set_state(tr.gen.get_state())
    tr2._pool_n.copy_(tr._pool_n)  # the reset pool's size adapts per rollout
    st = env.get_state().cpu().numpy().astype(np.float64)
    a = [x.clone() for x in tr.collect_rollout()]
    b = tr2.collect_rollout()
    assert tr._graph is not None and tr2._graph is None
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    # the replayed rollout against the oracle env: envs that run 25 steps without finishing, from
    # the state they entered the rollout with, under the rollout's own (unclipped) actions
    obs_b, act_b, _, rew_b, te_b, tr_b = (x.cpu().numpy().astype(np.float64) for x in a)
    cfg_c = abi.env_config_c(ecfg, m, obs_size(m.nq, m.nv))
    nq, nv, S = m.nq, m.nv, 25
    alive = np.nonzero((np.maximum(te_b[:S], tr_b[:S]) < 0.5).all(0))[0]
    assert len(alive) >= 4
    o = Oracle(m)
    for i in alive[:: max(1, len(alive) // 6)][:6]:
        row = st[i]
        s_ = o.new_state(row[:nq], row[nq:nq + nv], row[nq + nv:nq + 2 * nv], time=row[-1])
        aux = row[nq + 2 * nv:nq + 2 * nv + abi.AUX_DIM]
        for t in range(S):
            s_, aux, oo, ro, te, trn = o.env_step(cfg_c, s_, aux, act_b[t, i])
            assert rew_b[t, i] == pytest.approx(ro, abs=5e-3 * (1 + abs(ro))), (i, t)
            assert (te_b[t, i], tr_b[t, i]) == (te, trn)
            if t + 1 < S:
                np.testing.assert_allclose(obs_b[t + 1, i], oo[:obs_b.shape[2]], atol=5e-3 * (1 + np.abs(oo).max()))


def _apg_trainer(B, H, seed=0, vjp="unrolled"):
    from mjx_amd import apg
    m = mjx_amd.load_model("humanoid_mjx")
    m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4  # train_apg.py:101-105
    cfg = APGConfig()
    cfg.batch_size, cfg.horizon, cfg.seed = B, H, seed
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), B, seed=seed * 7919)
    return cfg, env, apg.APGTrainer(cfg, apg.HumanoidAPGEnv(env, vjp), device="cuda")


@pytest.mark.parametrize("vjp", ["implicit", "unrolled"])
def test_apg_c4_update_at_full_size(vjp):
    """C4 (2048 x 128, CG 4/4), two updates (the second a graph replay). Implicit VJP: no env's
    cotangents overflow (reverse_nonfinite_envs == 0). Unrolled VJP (jax.grad through the truncated
    solve): the chained per-step Jacobians grow x2.3 per reverse step and overflow fp32 for part of the
    batch (measured 700-770 of 2048 in updates 0-1), which the guard cuts; bounded here at
    800 (a regression that raised the overflow rate would show). Either
    way a few envs' forward states diverge under the truncated solve (forward_dropped_envs, the same
    in both modes: the forward is identical)."""
    cfg, env, tr = _apg_trainer(2048, 128, vjp=vjp)
    for it in range(2):
        met = tr.update(it)
        assert np.isfinite(met["loss"]) and np.isfinite(met["grad_norm"]) and met["grad_norm"] > 0
        for p in tr.policy.parameters():
            assert torch.isfinite(p).all()
        if vjp == "implicit":
            assert met["reverse_nonfinite_envs"] == 0, met
        else:
            assert met["reverse_nonfinite_envs"] <= 800, met
        assert met["forward_dropped_envs"] <= 2048 // 20, met


def test_apg_batched_param_grad_equals_per_step_accumulation():
    cfg, env, tr = _apg_trainer(256, 16, seed=3)
    c0 = env.counter
    tr.loss_and_grad(use_norm=False)
    g_batched = [p.grad.clone() for p in tr.policy.parameters()]
    env.counter = c0  # the same resets
    tr.loss_and_grad(use_norm=False, per_step_param_grad=True)
    for a, b in zip(g_batched, [p.grad for p in tr.policy.parameters()]):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-6 * (1 + float(b.abs().max())))


def test_evaluate_32x500_against_stepwise_loop_and_oracle():
    from mjx_amd import jaxrng, ppo
    from rng_ref import jax_reset_noise
    m, sys_ = _humanoid()
    cfg = reference_ppo_config()
    cfg.num_envs, cfg.rollout_length = 64, 8
    ecfg = resolve_ids(m, cfg.env_config)
    env = HumanoidEnv(sys_, ecfg, 64, seed=1)
    ev = HumanoidEnv(sys_, ecfg, 32, seed=2)
    tr = ppo.PPOTrainer(cfg, env, ev, device="cuda", jax_keys=True)
    tr.iteration(0)  # non-trivial obs statistics
    it = 7
    score = tr.evaluate(it)
    # the same loop, step by step, keeping every step's keys, actions, rewards and done flags
    jr = jaxrng
    sp = jr.split(jr.prng_key(int(cfg.seed) + 10000 + it))
    rng, keys = sp[0].clone(), jr.split(sp[1], 32).contiguous()
    ev.set_reset_keys(keys, jr.PARTITIONABLE)
    init_keys = keys.clone()
    obs = ev.reset().clone()
    acc = torch.zeros(32, device="cuda")
    rec = []
    for _ in range(500):
        sp = jr.split(rng)
        rng.copy_(sp[0])
        keys.copy_(jr.split(sp[1], 32))
        with torch.no_grad():
            mean, _ = tr.policy(tr.rms.normalize(obs))
        o, r, te, trn = ev.step(mean)
        rec.append((keys.clone(), mean.clone(), r.clone(), torch.maximum(te, trn).clone()))
        obs = o
        acc += r
    ev.set_reset_keys(None)
    assert score == pytest.approx(float(acc.mean()), rel=1e-6, abs=1e-6)
    # first 40 steps of 4 envs on the oracle env: same resets (jax draws), same actions
    cfg_c = abi.env_config_c(ecfg, m, obs_size(m.nq, m.nv))
    o_ = Oracle(m)
    nj, nv = m.nq - 7, m.nv
    noise0 = jax_reset_noise(init_keys.cpu().numpy().view(np.uint32), nj, nv, jr.PARTITIONABLE)
    for i in range(4):
        s, aux, _ = o_.env_reset(cfg_c, noise0[i].astype(np.float64))
        for t in range(40):
            k, a, r, d = (x[i].cpu().numpy() for x in rec[t])
            s, aux, _, ro, te, trn = o_.env_step(cfg_c, s, aux, a.astype(np.float64))
            assert float(r) == pytest.approx(ro, abs=5e-3 * (1 + abs(ro))), (i, t)
            assert float(d) == max(te, trn)
            if d > 0.5:  # the merge: reset from this step's key
                nz = jax_reset_noise(k.view(np.uint32)[None], nj, nv, jr.PARTITIONABLE)[0]
                s, aux, _ = o_.env_reset(cfg_c, nz.astype(np.float64))


def test_qpos_history_dump(tmp_path):
    """rendering.py: post-step qpos and the clipped actions; replaying the actions from the same
    (jax-keyed) initial state through the oracle env reproduces the history's first steps."""
    from mjx_amd import jaxrng, rendering
    from rng_ref import jax_reset_noise
    m, sys_ = _humanoid()
    ecfg = resolve_ids(m, reference_ppo_config().env_config)
    env = HumanoidEnv(sys_, ecfg, 1, seed=4)
    g = torch.Generator(device="cuda").manual_seed(0)
    pol = lambda o: torch.rand((1, m.nu), generator=g, device="cuda") * 2.4 - 1.2  # noqa: E731
    keys = jaxrng.split(jaxrng.prng_key(9), 1)
    qpos, act = rendering.rollout_qpos_history(env, pol, 0.5, reset_keys=keys)
    assert qpos.shape == (100, 1, m.nq) and act.shape == (100, 1, m.nu) and np.abs(act).max() <= 1.0
    path = rendering.save_qpos_history(str(tmp_path / "videos" / "iter_000001.npz"), qpos[:, 0], act[:, 0],
                                       m.timestep, 60, "humanoid_mjx.xml")
    d = rendering.load_qpos_history(path)
    assert d["qpos"].shape == (100, m.nq) and int(d["stride"]) == 3 and float(d["dt"]) == pytest.approx(m.timestep)
    assert np.isfinite(d["qpos"]).all()
    cfg_c = abi.env_config_c(ecfg, m, obs_size(m.nq, m.nv))
    o = Oracle(m)
    nz = jax_reset_noise(keys.cpu().numpy().view(np.uint32), m.nq - 7, m.nv, jaxrng.PARTITIONABLE)[0]
    s, aux, _ = o.env_reset(cfg_c, nz.astype(np.float64))
    for t in range(10):
        s, aux, *_ = o.env_step(cfg_c, s, aux, d["act"][t].astype(np.float64))
        np.testing.assert_allclose(d["qpos"][t], state_arrays(m, s)["qpos"], atol=1e-3)


def test_apg_c4_step_descends_after_normalisation():
    """the C4 update's direction at full size (2048 x 128, CG 4/4, implicit VJP), probed
    at the first post-normalisation update (100, train_apg.py:256,262). On that update's own resets,
    with the observation statistics held at their pre-update values, the clipped Adam step lowers the
    loss at 1 and 10 learning-rate steps: loss(theta0 + eps (theta1 - theta0)) < loss(theta0) for eps
    in {1, 10}. Statistics from the observations in the loss (--rms-in-loss-only: under the reference's
    rule, every rollout observation, the statistics collapse at this update and the gradient is not
    finite, DESIGN.md "APG at C4"). Deterministic: the same run gives the same losses (measured round
    4, tools/apg_direction_probe.py: 101.11 -> 99.94 / 99.46)."""
    from mjx_amd import apg
    from train_apg import apg_model
    cfg = APGConfig()
    cfg.batch_size, cfg.horizon = 2048, 128
    cfg.rms_in_loss_only = True
    m = apg_model(cfg, solver="cg")
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), cfg.batch_size, seed=cfg.seed)
    tr = apg.APGTrainer(cfg, apg.HumanoidAPGEnv(env, "implicit"), device="cuda", use_graph=False)
    for it in range(100):
        tr.update(it)
    params = list(tr.policy.parameters())
    c0 = env.counter
    rms0 = (tr.rms.mean.clone(), tr.rms.var.clone(),
            tr.rms.count.clone() if torch.is_tensor(tr.rms.count) else float(tr.rms.count))
    th0 = [p.detach().clone() for p in params]
    met = tr.update(100)
    assert np.isfinite(met["grad_norm"]) and met["reverse_nonfinite_envs"] == 0, met
    th1 = [p.detach().clone() for p in params]
    tr.rms.mean, tr.rms.var, tr.rms.count = rms0
    losses = {}
    with torch.no_grad():
        for eps in (0.0, 1.0, 10.0):
            for p, x0, x1 in zip(params, th0, th1):
                p.copy_(x0 + eps * (x1 - x0))
            env.counter = c0
            with torch.enable_grad():
                losses[eps] = float(tr.loss_and_grad(True)[0])
    print("APG C4 update 100 losses at eps 0 / 1 / 10:", losses)
    assert losses[0.0] == pytest.approx(met["loss"], rel=1e-5)
    assert losses[1.0] < losses[0.0] and losses[10.0] < losses[0.0]

"""VJP tape (mjl_env_step_record / mjl_env_step_vjp_replay): the recorded step is the env step, and
the replayed VJP is the recomputing one (train_apg.py:187-189's jax.grad through the step)."""
import pytest
import torch

import mjx_amd
from mjx_amd import abi, apg, mjcf, mjx
from mjx_amd.config import reference_ppo_config
from mjx_amd.envs import HumanoidEnv, resolve_ids

pytestmark = pytest.mark.gpu

STATE = ("qpos", "qvel", "qacc_warmstart", "ctrl", "time", "aux")


def _pair(solver, vjp, B=64, model="humanoid_mjx"):
    m = mjx_amd.load_model(model)
    if solver == "cg44":
        m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
    ecfg = resolve_ids(m, reference_ppo_config().env_config)
    return m, [apg.HumanoidAPGEnv(HumanoidEnv(mjx.put_model(m), ecfg, B, seed=9), vjp) for _ in range(2)]


@pytest.mark.parametrize("model,solver,vjp", [("humanoid_mjx", "model", "implicit"), ("humanoid_mjx", "cg44", "unrolled"),
                                              ("humanoid_mjx", "cg44", "implicit"),
                                              ("humanoid", "model", "implicit"), ("humanoid", "cg44", "unrolled")])
def test_record_and_replay_equal_step_and_recompute(model, solver, vjp):
    """Over 12 steps of random actions (humanoid_mjx: implicitfast; humanoid.xml: Euler with
    eulerdamp): the recorded step's outputs and state are the env step's;
    the replayed VJP's cotangents (state, warm start, action, aux) are those of the VJP that restores
    the pre-step state and recomputes (same warm start), bit for bit."""
    m, (plain, taped) = _pair(solver, vjp, model=model)
    B, H = plain.num_envs, 12
    taped.enable_vjp_tape(H)
    for e in (plain, taped):
        e.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    acts, pre = [], []
    for t in range(H):
        a = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
        acts.append(a)
        pre.append(plain.get_state())
        o1 = [x.clone() for x in plain.step(a)]
        o2 = [x.clone() for x in taped.step_record(t, a)]
        for x, y, k in zip(o1, o2, ("obs", "rew", "term", "trunc")):
            assert torch.equal(x, y), f"step {t}: {k}"
        for f in STATE:
            assert torch.equal(plain.env.data.get(f), taped.env.data.get(f)), f"step {t}: {f}"
    gws_on = vjp == "unrolled"
    for t in range(H - 1, -1, -1):
        gq = torch.randn((B, m.nq), generator=g, device="cuda")
        gv = torch.randn((B, m.nv), generator=g, device="cuda")
        gw = torch.randn((B, m.nv), generator=g, device="cuda") if gws_on else None
        gr = torch.randn(B, generator=g, device="cuda")
        gx = torch.randn((B, abi.AUX_DIM), generator=g, device="cuda")
        plain.env.set_state(pre[t])  # the forward's own warm start
        if gws_on:
            r1 = plain.step_vjp_full(acts[t], gq, gv, gw, gr, gx)
        else:
            oq, ov, oa, ox = plain.step_vjp(acts[t], gq, gv, gr, gx)
            r1 = (oq, ov, None, oa, ox)
        r2 = taped.step_vjp_replay(t, acts[t], gq, gv, gw, gr, gx)
        for x, y, k in zip(r1, r2, ("qpos", "qvel", "ws", "act", "aux")):
            if x is None:
                assert y is None
                continue
            assert torch.equal(x, y), f"step {t}: {k} cotangent ({(x - y).abs().max().item():.3g})"


def test_tape_slot_bounds():
    m, (env, _) = _pair("model", "implicit", B=4)
    a = torch.zeros((4, m.nu), device="cuda")
    with pytest.raises(Exception, match="slot"):
        env.step_record(0, a)
    env.enable_vjp_tape(2)
    env.step_record(1, a)
    with pytest.raises(Exception, match="slot"):
        env.step_record(2, a)


@pytest.mark.parametrize("solver,vjp", [("cg44", "implicit"), ("model", "implicit"), ("cg44", "unrolled")])
def test_lds_row_record_equals_global_row_record(solver, vjp):
    """The implicit record keeps its constraint rows in LDS (vjp_record_kernel) and writes the tape
    slot vjp_kernel's global-row record writes (MJL_OPT_FORCE_GLOBAL_ROWS selects that one): over 8
    steps, with env 0 posed past every hinge limit and into the floor (more rows than the LDS holds:
    the record's global fallback), the step outputs, the state and every replayed cotangent agree
    bit for bit (CG 4/4 drives that pose to NaN within a few steps in both: NaN equals NaN here)."""
    same = lambda x, y: torch.testing.assert_close(x, y, rtol=0, atol=0, equal_nan=True) is None
    m, (lds, glb) = _pair(solver, vjp, B=32)
    glb.env.data.set_option(abi.OPT_FORCE_GLOBAL_ROWS, 1)
    B, H = lds.num_envs, 8
    q = m.key_qpos[m.names["key"].index("supine")].copy()
    for j in range(1, m.njnt):
        q[m.jnt_qposadr[j]] = m.jnt_range[j][1] + 0.05
    for e in (lds, glb):
        e.enable_vjp_tape(H)
        e.reset()
    st = lds.get_state()
    st[0, :m.nq] = torch.tensor(q, dtype=torch.float32, device="cuda")
    st[0, m.nq:m.nq + 2 * m.nv] = 0.0
    for e in (lds, glb):
        e.env.set_state(st)
    d = mjx.make_data(lds.env.sys, 1)  # env 0's pose overflows the LDS rows (the fallback runs)
    d.set("qpos", st[:1, :m.nq].cpu())
    mjx.forward(lds.env.sys, d)
    assert d.get("stats")[0, 1].item() > 48
    g = torch.Generator(device="cuda").manual_seed(3)
    acts = []
    for t in range(H):
        a = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
        acts.append(a)
        o1 = [x.clone() for x in lds.step_record(t, a)]
        o2 = [x.clone() for x in glb.step_record(t, a)]
        for x, y, k in zip(o1, o2, ("obs", "rew", "term", "trunc")):
            assert same(x, y), f"step {t}: {k}"
        for f in STATE:
            assert same(lds.env.data.get(f), glb.env.data.get(f)), f"step {t}: {f}"
        assert torch.isfinite(lds.env.data.get("qpos")[1:]).all()
    for t in range(H - 1, -1, -1):
        gq = torch.randn((B, m.nq), generator=g, device="cuda")
        gv = torch.randn((B, m.nv), generator=g, device="cuda")
        gr = torch.randn(B, generator=g, device="cuda")
        gx = torch.randn((B, abi.AUX_DIM), generator=g, device="cuda")
        gw = torch.randn((B, m.nv), generator=g, device="cuda") if vjp == "unrolled" else None
        r1 = lds.step_vjp_replay(t, acts[t], gq, gv, gw, gr, gx)
        r2 = glb.step_vjp_replay(t, acts[t], gq, gv, gw, gr, gx)
        for x, y, k in zip(r1, r2, ("qpos", "qvel", "ws", "act", "aux")):
            if x is None:
                assert y is None
                continue
            assert same(x, y), f"step {t}: {k} cotangent"

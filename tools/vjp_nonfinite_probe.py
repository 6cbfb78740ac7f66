"""Unrolled-VJP overflow probe (CG 4/4): roll 2048 envs forward with smooth random actions, run
the env-step VJP (unit cotangents) at every step, count non-finite outputs, and for the first few
offending (env, step) pairs compare the magnitude with the oracle's dual-number Jacobian.
    python tools/vjp_nonfinite_probe.py [unrolled|implicit] [B H]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mujoco-mjx-lab_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import abi, mjcf, mjx  # noqa: E402
from mjx_amd.config import EnvConfig  # noqa: E402
from mjx_amd.envs import HumanoidEnv, obs_size, resolve_ids  # noqa: E402
from oracle import Oracle  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "unrolled"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
H = int(sys.argv[3]) if len(sys.argv) > 3 else 64
m = mjx_amd.load_model("humanoid_mjx")
m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
ecfg = resolve_ids(m, EnvConfig())
env = HumanoidEnv(mjx.put_model(m), ecfg, B, seed=3)
env.data.set_option(abi.OPT_VJP_UNROLLED, int(mode == "unrolled"))
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
u = torch.zeros((B, m.nu), device="cuda")
o = Oracle(m)
cfg_c = abi.env_config_c(ecfg, m, obs_size(m.nq, m.nv))
shown = 0
tot_bad = 0
for t in range(H):
    u = 0.9 * u + 0.2 * (torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1)
    act = u.clamp(-1, 1)
    st = env.get_state().clone()
    qv = env.data.get("qvel")
    ok_state = torch.isfinite(qv).all(1) & (qv.abs().amax(1) < 1e3)
    gq = torch.ones((B, m.nq), device="cuda")
    gv = torch.ones((B, m.nv), device="cuda")
    gr = torch.ones(B, device="cuda")
    oq, ov, oa, oaux = env.step_vjp(act, gq, gv, gr)
    mag = torch.stack([x.abs().amax(1) for x in (oq, ov, oa)], 1).amax(1)
    bad = (~torch.isfinite(mag) | (mag > 1e8)) & ok_state
    nb = int(bad.sum())
    tot_bad += nb
    if nb:
        print(f"t {t}: {nb} envs with |vjp| > 1e8 or non-finite (of {int(ok_state.sum())} sane states); "
              f"median |vjp| {float(mag[ok_state & ~bad].median()):.3g}", flush=True)
        for i in bad.nonzero()[:, 0].tolist()[:2]:
            if shown >= 6:
                break
            shown += 1
            row = st[i].cpu().numpy().astype(np.float64)
            nq, nv = m.nq, m.nv
            s = o.new_state(row[:nq], row[nq:nq + nv], row[nq + nv:nq + 2 * nv], time=float(row[-1]))
            aux = row[nq + 2 * nv:nq + 2 * nv + abi.AUX_DIM]
            J = o.env_step_jacobian(cfg_c, s, aux, act[i].cpu().numpy().astype(np.float64))
            ref = np.ones(J.shape[0]) @ J
            print(f"   env {i}: gpu |vjp| {float(mag[i]):.3g}; oracle dual |u'J| {np.abs(ref).max():.3g} "
                  f"finite {np.isfinite(ref).all()}", flush=True)
    env.set_state(st)
    env.step(act, auto_reset=False)
print(f"total flagged (env, step) pairs: {tot_bad}")

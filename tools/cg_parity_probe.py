"""Truncated-solve parity probe: B seeded env resets, T steps with fixed small actions under CG 4/4
(or another solver override), GPU env step vs the fp64 / fp32 oracle; prints per-step max |qvel|
differences and rewards per env.   python tools/cg_parity_probe.py [cg|newton] IT LS [B T]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mujoco-mjx-lab_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import abi, mjcf, mjx  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402
from mjx_amd.envs import HumanoidEnv, obs_size, resolve_ids  # noqa: E402
from oracle import Oracle, state_arrays  # noqa: E402

solver, it, ls = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
B = int(sys.argv[4]) if len(sys.argv) > 4 else 4
T = int(sys.argv[5]) if len(sys.argv) > 5 else 5
m = mjx_amd.load_model("humanoid_mjx")
m.solver = mjcf.SOLVER_CG if solver == "cg" else mjcf.SOLVER_NEWTON
m.iterations, m.ls_iterations = it, ls
ecfg = resolve_ids(m, reference_ppo_config().env_config)
c = abi.env_config_c(ecfg, m, obs_size(m.nq, m.nv))
nd = m.nq - 7 + m.nv + 2
noise = np.random.default_rng(7).uniform(0, 1, (B, nd)).astype(np.float32)
acts = np.random.default_rng(1).uniform(-0.3, 0.3, (T, B, m.nu)).astype(np.float32)
env = HumanoidEnv(mjx.put_model(m), ecfg, B, seed=3, store_derived=True)
env.reset(noise=torch.tensor(noise))
orcs = [Oracle(m), Oracle(m, use_float=True)]
ost = [[list(o.env_reset(c, noise[i].astype(np.float64))[:2]) for i in range(B)] for o in orcs]
g = {f: env.data.get(f).cpu().numpy() for f in ("qpos", "qvel", "qacc_warmstart")}
for i in range(B):
    a = state_arrays(m, ost[0][i][0])
    print(f"reset env{i}: " + " ".join(f"d{f} {np.abs(a[f] - g[f][i]).max():.2e}" for f in g), flush=True)
for t in range(T):
    _, r, _, _ = env.step(torch.tensor(acts[t], device="cuda"), auto_reset=False)
    v = env.data.get("qvel").cpu().numpy()
    qa = env.data.get("qacc").cpu().numpy()
    fc = env.data.get("qfrc_constraint").cpu().numpy()
    st = env.data.get("stats").cpu().numpy()
    r = r.cpu().numpy()
    for i in range(B):
        line = f"t{t} env{i} gpu r {r[i]:+.4f} ncon/nefc/iter {st[i, :3]}"
        for k, o in enumerate(orcs):
            s, aux, _, ro, _, _ = o.env_step(c, ost[k][i][0], ost[k][i][1], acts[t, i].astype(np.float64))
            ost[k][i][1] = aux
            a = state_arrays(m, s)
            line += (f" | {'f64' if k == 0 else 'f32'} r {ro:+.4f} dv {np.abs(a['qvel'] - v[i]).max():.2e} "
                     f"dqacc {np.abs(a['qacc'] - qa[i]).max():.2e} dfc {np.abs(a['qfrc_constraint'] - fc[i]).max():.2e} "
                     f"niter {a['niter']} nefc {a['nefc']}")
        print(line, flush=True)

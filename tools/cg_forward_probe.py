"""One forward pass from seeded reset states with qacc_warmstart = 0 under a solver override: GPU
qacc vs the fp64 / fp32 oracle (the truncated solve's result depends on every rule of the loop).
    python tools/cg_forward_probe.py [cg|newton] IT LS [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mujoco-mjx-lab_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import abi, mjcf, mjx  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402
from mjx_amd.envs import obs_size, resolve_ids  # noqa: E402
from oracle import Oracle, state_arrays  # noqa: E402

solver, it, ls = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
B = int(sys.argv[4]) if len(sys.argv) > 4 else 8
m = mjx_amd.load_model("humanoid_mjx")
m.solver = mjcf.SOLVER_CG if solver == "cg" else mjcf.SOLVER_NEWTON
m.iterations, m.ls_iterations = it, ls
ecfg = resolve_ids(m, reference_ppo_config().env_config)
c = abi.env_config_c(ecfg, m, obs_size(m.nq, m.nv))
nd = m.nq - 7 + m.nv + 2
noise = np.random.default_rng(7).uniform(0, 1, (B, nd))
o64, o32 = Oracle(m), Oracle(m, use_float=True)
Q, V = [], []
for i in range(B):
    a = state_arrays(m, o64.env_reset(c, noise[i])[0])
    Q.append(np.float32(a["qpos"]))
    V.append(np.float32(a["qvel"]))
d = mjx.make_data(mjx.put_model(m), B)
d.set("qpos", torch.tensor(np.array(Q)))
d.set("qvel", torch.tensor(np.array(V)))
mjx.forward(mjx.put_model(m), d)
qa = d.get("qacc").cpu().numpy()
st = d.get("stats").cpu().numpy()
for i in range(B):
    line = f"env{i} gpu ncon/nefc/iter {st[i, :3]}"
    for name, o in (("f64", o64), ("f32", o32)):
        a = state_arrays(m, o.forward(o.new_state(Q[i].astype(np.float64), V[i].astype(np.float64))))
        line += f" | {name} dqacc {np.abs(a['qacc'] - qa[i]).max():.3e} (|qacc| {np.abs(a['qacc']).max():.3g}) niter {a['niter']} nefc {a['nefc']}"
    print(line, flush=True)

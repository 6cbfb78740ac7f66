"""Roll the CG-solver humanoid (train_apg.py solver options) with random actions; report envs whose
state blows up and dump the first offending pre-step state for CPU reproduction."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch
import mjx_amd
from mjx_amd import mjx, mjcf
from mjx_amd.config import EnvConfig
from mjx_amd.envs import HumanoidEnv, resolve_ids

B, H = 2048, 128
for solver in ("cg", "newton"):
    m = mjx_amd.load_model("humanoid_mjx")
    if solver == "cg":
        m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), B, seed=5)
    g = torch.Generator(device="cuda").manual_seed(0)
    for rep in range(2):
        env.reset()
        dumped = False
        traj, acts = [], []
        for t in range(H):
            st = {k: env.data.get(k).clone() for k in ("qpos", "qvel", "qacc_warmstart", "aux", "time")}
            act = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
            traj.append(st); acts.append(act)
            _, r, te, tu = env.step(act, auto_reset=False)
            v = env.data.get("qvel")
            bad = ~torch.isfinite(v).all(1) | (v.abs().max(1).values > 1e3)
            if bad.any():
                idx = bad.nonzero().flatten()
                print(solver, rep, "t", t, "bad envs", idx[:10].tolist(), "count", int(bad.sum()), flush=True)
                if not dumped:
                    i = int(idx[0])
                    torch.save({"solver": solver, "state": {k: x[i].cpu() for k, x in st.items()}, "act": act[i].cpu(),
                                "traj": [{k: x[i].cpu() for k, x in s_.items()} for s_ in traj],
                                "acts": [a_[i].cpu() for a_ in acts],
                                "qvel_after": v[i].cpu(), "qpos_after": env.data.get("qpos")[i].cpu()},
                               f"gpurun_out/cg_bad_{solver}_{rep}.pt")
                    dumped = True
                break
        else:
            print(solver, rep, "no blowup; final max|qvel|", float(env.data.get("qvel").abs().max()), flush=True)

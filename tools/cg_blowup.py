"""Blow-up census: 2048 humanoid envs x 128 steps under smooth random controls (an AR(1) process,
closer to a policy's than white noise), for several solver settings: how many envs end non-finite
or with max|qvel| > 1e3. Also dumps the first offending env's trajectory for CPU reproduction."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch
import mjx_amd
from mjx_amd import mjx, mjcf
from mjx_amd.config import EnvConfig
from mjx_amd.envs import HumanoidEnv, resolve_ids

B, H = 2048, 128
for solver, it, ls in (("cg", 4, 4), ("cg", 4, 20), ("cg", 10, 20), ("cg", 30, 20), ("newton", 10, 20), ("newton", 1, 4)):
    m = mjx_amd.load_model("humanoid_mjx")
    m.solver = mjcf.SOLVER_CG if solver == "cg" else mjcf.SOLVER_NEWTON
    m.iterations, m.ls_iterations = it, ls
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), B, seed=5)
    g = torch.Generator(device="cuda").manual_seed(0)
    env.reset()
    u = torch.zeros((B, m.nu), device="cuda")
    first = None
    traj, acts = [], []
    for t in range(H):
        st = {k: env.data.get(k).clone() for k in ("qpos", "qvel", "qacc_warmstart", "aux", "time")}
        u = 0.9 * u + 0.45 * (torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1)
        act = u.clamp(-1, 1)
        traj.append(st); acts.append(act)
        env.step(act, auto_reset=False)
        v = env.data.get("qvel")
        bad = ~torch.isfinite(v).all(1) | (v.abs().max(1).values > 1e3)
        if first is None and bad.any():
            first = (t, int(bad.nonzero()[0]))
    v = env.data.get("qvel")
    nonfin = int((~torch.isfinite(v).all(1)).sum())
    big = int((torch.isfinite(v).all(1) & (v.abs().max(1).values > 1e3)).sum())
    print(f"{solver} {it}/{ls}: non-finite {nonfin}, |qvel|>1e3 {big}, first bad {first}", flush=True)
    if first is not None and solver == "cg" and it == 4 and ls == 4:
        t, i = first
        torch.save({"traj": [{k: x[i].cpu() for k, x in s_.items()} for s_ in traj[:t + 1]],
                    "acts": [a_[i].cpu() for a_ in acts[:t + 1]]}, "gpurun_out/cg_bad.pt")

"""Diagnostic: per-phase cycle shares of the env-step VJP kernel from the MJL_TIMING build (run with
MJX355_LIB pointing at it). Slots: 0 start, 1 forward recompute done, 2..13 after each reverse pass."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import _lib, mjx  # noqa: E402
from mjx_amd.config import EnvConfig  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402

names = ["forward recompute", "adj env + integrate", "adj solver rows", "adj contact jac", "adj collision",
         "adj geom frames", "adj forces", "adj rne", "adj mass", "adj crb", "adj cinert", "adj cdof", "adj kinematics"]
L = _lib.lib()
L.mjl_debug_set_stamps.argtypes = [C.c_void_p]
m = mjx_amd.load_model("humanoid_mjx")
if os.environ.get("SOLVER") == "cg44":  # train_apg.py's override
    from mjx_amd import mjcf
    m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
B = 2048
env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), B, seed=3)
if os.environ.get("VJP") == "unrolled":
    from mjx_amd import abi
    env.data.set_option(abi.OPT_VJP_UNROLLED, 1)
buf = torch.zeros((B, 16), dtype=torch.int64, device="cuda")
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
for _ in range(20):
    env.step(torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1, auto_reset=False)
act = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
gq, gv, gr = torch.randn((B, m.nq), device="cuda"), torch.randn((B, m.nv), device="cuda"), torch.randn(B, device="cuda")
for _ in range(2):
    env.step_vjp(act, gq, gv, gr)
torch.cuda.synchronize()
L.mjl_debug_set_stamps(C.c_void_p(buf.data_ptr()))
env.step_vjp(act, gq, gv, gr)
torch.cuda.synchronize()
L.mjl_debug_set_stamps(C.c_void_p(0))
s = buf.cpu().numpy().astype(np.float64)
d = np.diff(s[:, :14], axis=1)
tot = d.sum(1)
print(f"VJP: mean cycles/env {tot.mean():.0f}; p50 / max {np.percentile(tot, 50):.0f} / {tot.max():.0f}")
for i, n in enumerate(names):
    print(f"   {n:22s} {d[:, i].mean():9.0f}  {100 * d[:, i].mean() / tot.mean():5.1f}%")

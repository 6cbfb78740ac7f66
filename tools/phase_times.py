"""Diagnostic: per-phase cycle shares from the MJL_TIMING build (s_memtime stamps, lane 0).
Run with MJX355_LIB pointing at a library built with -DMJL_TIMING. Read the shares, not the
absolute time (the stamps perturb what they measure)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mjx_amd  # noqa: E402
import mjx_amd.abi  # noqa: E402
from mjx_amd import _lib, mjx  # noqa: E402

names = ["kinematics", "com_pos+crb+M", "velocity(rne,passive,act)", "factor M + qacc_smooth", "collision+rows",
         "solver", "sensors", "integrate"]
L = _lib.lib()
L.mjl_debug_set_stamps.argtypes = [C.c_void_p]
m = mjx_amd.load_model("humanoid_mjx")
sys_ = mjx.put_model(m)
B = 2048
buf = torch.zeros((B, 48), dtype=torch.int64, device="cuda")
L.mjl_debug_set_stamps(C.c_void_p(buf.data_ptr()))
for mode in ("speedtest", "trajectory"):
    d = mjx.make_data(sys_, B)
    d.set_option(mjx_amd.abi.OPT_STORE_DERIVED, 1)
    if mode == "speedtest":
        vel = torch.linspace(0, 1, B, device="cuda")
        for _ in range(2):
            mjx.speedtest_step(sys_, d, vel)
        torch.cuda.synchronize()
        buf.zero_()
        mjx.speedtest_step(sys_, d, vel)
    else:
        g = torch.Generator(device="cuda").manual_seed(0)
        for _ in range(29):
            mjx.step(sys_, d, torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1)
        torch.cuda.synchronize()
        buf.zero_()
        mjx.step(sys_, d, torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    st = d.get("stats").cpu().numpy()
    s = buf.cpu().numpy().astype(np.float64)
    ok = s[:, 8] > 0
    d8 = np.diff(s[ok][:, [0, 1, 2, 3, 4, 5, 6, 7, 8]], axis=1)
    tot = d8.sum(1).mean()
    print(f"{mode}: envs with LDS rows {ok.mean():.2f}; mean cycles/env-step {tot:.0f}; "
          f"p50 / p99 / max {np.percentile(d8.sum(1), 50):.0f} / {np.percentile(d8.sum(1), 99):.0f} / {d8.sum(1).max():.0f}")
    for i, n in enumerate(names):
        print(f"   {n:28s} {d8[:, i].mean():9.0f}  {100 * d8[:, i].mean() / tot:5.1f}%")
    it = st[:, 2].mean()
    print(f"   solver: mean ncon {st[:, 0].mean():.2f} nefc {st[:, 1].mean():.2f} iterations {it:.2f}")
    for i, n in zip(range(9, 14), ["warm start", "line search (+step)", "update + convergence", "hessian J'DJ",
                                   "cholesky factor+solve"]):
        v = s[ok][:, i].mean()
        print(f"      {n:26s} {v:9.0f}  per iteration {v / max(it, 1e-9):8.0f}")
    subs = {16: "kin: record loads", 17: "kin: local transforms", 18: "kin: level compose", 19: "kin: joints/geoms/sites",
            20: "rows: limits", 21: "rows: collision pass", 22: "rows: contact Jacobians",
            23: "crb: cinert+cdof", 24: "crb: subtree crb", 25: "vel: joint terms", 26: "vel: level pass",
            27: "vel: forces + subtree sums", 28: "ls: M s, J s", 29: "ls: |s|, c1, c2, p0",
            30: "ls: segment test + q", 31: "ls: 3-point loop", 32: "chol(all): load rows",
            33: "chol(all): factor", 34: "chol(all): store + reload", 35: "chol(all): back subst"}
    for i, n in subs.items():
        print(f"      {n:26s} {s[ok][:, i].mean():9.0f}")
    ls_calls = s[ok][:, 15].mean()
    if ls_calls > 0:
        print(f"      line searches per env-step {ls_calls:.2f}; "
              f"3-point iterations per line search {s[ok][:, 14].mean() / ls_calls:.2f}; "
              f"per env-step p99 / max {np.percentile(s[ok][:, 14], 99):.0f} / {s[ok][:, 14].max():.0f}")
    buf.zero_()

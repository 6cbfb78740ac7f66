"""Diagnostic: the speed-test launch's tail (MJL_TIMING build: MJX355_LIB=<timing lib>). Per env the
absolute s_memtime at the kernel's first and last stamp: when envs finish relative to the launch's
span, and how per-env cost (cycles, solver iterations) varies with the env index (vel = linspace).
python tools/tail_probe.py [B]"""
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
L = _lib.lib()
L.mjl_debug_set_stamps.argtypes = [C.c_void_p]
m = mjx_amd.load_model("humanoid_mjx")
sys_ = mjx.put_model(m)
buf = torch.zeros((B, 48), dtype=torch.int64, device="cuda")
L.mjl_debug_set_stamps(C.c_void_p(buf.data_ptr()))
d = mjx.make_data(sys_, B)
d.set_option(mjx_amd.abi.OPT_STORE_DERIVED, 1)
vel = torch.linspace(0, 1, B, device="cuda")
for _ in range(3):
    mjx.speedtest_step(sys_, d, vel)
torch.cuda.synchronize()
buf.zero_()
mjx.speedtest_step(sys_, d, vel)
torch.cuda.synchronize()
s = buf.cpu().numpy().astype(np.float64)
st = d.get("stats").cpu().numpy()
t0, t1 = s[:, 0], s[:, 8]
span = t1.max() - t0.min()
tot = t1 - t0
print(f"B {B}: span {span:.0f} cycles; start spread {t0.max() - t0.min():.0f}; per-env cycles mean {tot.mean():.0f} "
      f"p50 {np.percentile(tot, 50):.0f} p90 {np.percentile(tot, 90):.0f} p99 {np.percentile(tot, 99):.0f} max {tot.max():.0f}")
fin = (t1 - t0.min()) / span
for q in (0.5, 0.7, 0.8, 0.9, 0.95):
    print(f"  envs finished by {q:.0%} of the span: {(fin <= q).mean():.3f}")
nb = 16
print("  env-index bins: mean cycles / mean iterations / mean nefc / max cycles")
for b in range(nb):
    sl = slice(b * B // nb, (b + 1) * B // nb)
    print(f"   {b:2d} {tot[sl].mean():8.0f} {st[sl, 2].mean():6.2f} {st[sl, 1].mean():6.1f} {tot[sl].max():8.0f}")
it = st[:, 2]
print("  cycles by solver iterations:", {int(k): (int((it == k).sum()), round(float(tot[it == k].mean()))) for k in np.unique(it)})
order = np.argsort(-tot)[:12]
print("  slowest envs (index, cycles, iterations, nefc, ncon):", [(int(i), int(tot[i]), int(st[i, 2]), int(st[i, 1]), int(st[i, 0])) for i in order])
ph = np.diff(s[:, :9], axis=1)
names = ["kin", "crb+M", "vel", "factM", "rows", "solver", "sensors", "integ"]
sub = {9: "warm", 10: "ls", 11: "update", 12: "hess", 13: "chol", 14: "ls iters", 15: "line searches"}
for lab, idx in (("slowest", np.argsort(-tot)[:8]), ("median", np.argsort(np.abs(tot - np.median(tot)))[:8]),
                 ("fastest", np.argsort(tot)[:8])):
    print(f"  {lab} envs: phases " + " ".join(f"{n} {ph[idx, i].mean():.0f}" for i, n in enumerate(names)))
    print("      solver sub: " + " ".join(f"{n} {s[idx, k].mean():.1f}" for k, n in sub.items()))

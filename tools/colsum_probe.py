"""Diagnostic: column sums x[n, d].sum(0) at the PPO update's shapes — torch's reduction, BLAS
(mv / mm with a ones vector) and the native mjl_colsum kernel. Not product code."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

from mjx_amd import ppo  # noqa: E402


def bench(f, reps=200):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.time() - t) / reps * 1e6


for n, d in ((65536, 256), (65536, 21), (65536, 1), (32, 65536), (32, 5376)):
    x = torch.randn(n, d, device="cuda")
    ones = torch.ones(n, device="cuda")
    o2 = torch.ones(1, n, device="cuda")
    r0 = x.double().sum(0)
    print(n, d, "sum0 %.1f us" % bench(lambda: x.sum(0)),
          "mv %.1f us" % bench(lambda: torch.mv(x.t(), ones)),
          "mm %.1f us" % bench(lambda: o2 @ x),
          "native %.1f us" % bench(lambda: ppo.colsum_native(x)),
          "maxdiff sum0 %.2e native %.2e" % ((x.sum(0).double() - r0).abs().max(),
                                             (ppo.colsum_native(x).double() - r0).abs().max()), flush=True)

# the split-K weight-gradient sum over the splits, as the 3-D tensor the batched GEMM returns
for shp in ((32, 256, 256), (32, 256, 54), (32, 21, 256), (32, 1, 256)):
    g3 = torch.randn(shp, device="cuda")
    print(shp, "sum0(3d) %.1f us" % bench(lambda: g3.sum(0)),
          "sum0(2d) %.1f us" % bench(lambda: g3.view(shp[0], -1).sum(0)),
          "native %.1f us" % bench(lambda: ppo.colsum_native(g3.view(shp[0], -1))), flush=True)

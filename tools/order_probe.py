"""Diagnostic: does the speed-test kernel time depend on which workgroup gets which env state?
Same 2048 speed-test states (qvel[0] = linspace(0, 1, B)) fed in the bench's order, reversed, and
randomly permuted; plus the per-env Newton iteration counts along the index (mjx.forward stats)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjx  # noqa: E402

B = 2048
m = mjx_amd.load_model("humanoid_mjx")
s = mjx.put_model(m)
d = mjx.make_data(s, B)
base = torch.linspace(0.0, 1.0, B, device="cuda")
out = torch.empty_like(base)
g = torch.Generator(device="cpu").manual_seed(0)
orders = {"bench": base, "reversed": base.flip(0), "random": base[torch.randperm(B, generator=g).cuda()]}


def kern_us(vel, n=200):
    for _ in range(10):
        mjx.speedtest_step(s, d, vel, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        mjx.speedtest_step(s, d, vel, out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for r in range(3):
    print("round", r, {k: round(kern_us(v), 2) for k, v in orders.items()}, flush=True)
ds = mjx.make_data(s, B)
qv = torch.zeros((B, s.nv), device="cuda")
qv[:, 0] = base
ds.set("qvel", qv)
mjx.forward(s, ds)
it = ds.get("stats")[:, 2].cpu().numpy()
print("iterations by index eighth:", [round(float(x), 2) for x in it.reshape(8, -1).mean(1)])
print("max iterations", it.max(), "at indices", np.nonzero(it == it.max())[0][:20].tolist())
print("histogram", np.bincount(it.astype(int)).tolist())

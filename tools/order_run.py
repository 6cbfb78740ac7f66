"""Diagnostic: 50 speed-test launches with the 2048 states in the bench order or a random
permutation (argv[1] = bench | random), for counter passes (rocprofv3 --pmc)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjx  # noqa: E402

B = 2048
s = mjx.put_model(mjx_amd.load_model("humanoid_mjx"))
d = mjx.make_data(s, B)
vel = torch.linspace(0.0, 1.0, B, device="cuda")
if sys.argv[1] == "random":
    vel = vel[torch.randperm(B, generator=torch.Generator().manual_seed(0)).cuda()]
out = torch.empty_like(vel)
for _ in range(50):
    mjx.speedtest_step(s, d, vel, out)
torch.cuda.synchronize()
print("done", sys.argv[1])

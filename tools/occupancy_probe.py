"""Speed-test kernel time vs batch size: B = 256..8192 at a fixed per-env workload. At B <= 1024
each SIMD holds <= 1 wave, at 2048 two: the ratio tells whether the kernel is issue-bound (time
scales with waves per SIMD) or latency-bound (time flat)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch
import mjx_amd
from mjx_amd import mjx

m = mjx_amd.load_model("humanoid_mjx")
sys_ = mjx.put_model(m)
for B, mode in [(b, "same") for b in (1, 64, 256, 512, 1024, 1536, 2048, 3072, 4096, 8192)] + \
               [(b, "linspace") for b in (1024, 2048, 4096)]:
    d = mjx.make_data(sys_, B)
    d.set_option(mjx_amd.abi.OPT_STORE_DERIVED, 0)
    # identical work in every env, or the speed test's own vel = linspace(0, 1, B)
    vel = torch.full((B,), 0.5, device="cuda") if mode == "same" else torch.linspace(0, 1, B, device="cuda")
    out = torch.empty(B, device="cuda")
    for _ in range(5):
        mjx.speedtest_step(sys_, d, vel, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        mjx.speedtest_step(sys_, d, vel, out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 50
    print(f"{mode:8s} B {B:5d}: {ms * 1000:8.1f} us/launch  {B / ms / 1e3:8.2f} M env-steps/s", flush=True)

"""Diagnostic: speed-test kernel time at B = 2048 (vel = linspace) with the Newton iteration cap
overridden (0 = smooth dynamics + collision + rows only, no solve), to price one solver iteration
in the real two-waves-per-SIMD setting. Not a parity configuration."""
import copy, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch
import mjx_amd
from mjx_amd import mjx

base = mjx_amd.load_model("humanoid_mjx")
B = 2048
for its in [int(x) for x in os.environ.get("ITERS", "0,1,2,3,4,10").split(",")]:
    m = copy.deepcopy(base)
    m.iterations = its
    sys_ = mjx.put_model(m)
    d = mjx.make_data(sys_, B)
    d.set_option(mjx_amd.abi.OPT_STORE_DERIVED, 0)
    vel = torch.linspace(0, 1, B, device="cuda")
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
    print(f"iterations {its:2d}: {e0.elapsed_time(e1) / 50 * 1000:7.1f} us/launch", flush=True)

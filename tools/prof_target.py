"""Minimal launch loop for rocprofv3 counter collection: speed-test (or env-step) kernel only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjx  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "speedtest"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
m = mjx_amd.load_model("humanoid_mjx")
sys_ = mjx.put_model(m)
if mode == "speedtest":
    d = mjx.make_data(sys_, B)
    vel = torch.linspace(0, 1, B, device="cuda")
    out = torch.empty_like(vel)
    for _ in range(n):
        mjx.speedtest_step(sys_, d, vel, out)
else:
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    env = HumanoidEnv(sys_, cfg, B, seed=1)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    act = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
    for _ in range(n):
        env.step(act)
torch.cuda.synchronize()
print("done", mode, B, n)

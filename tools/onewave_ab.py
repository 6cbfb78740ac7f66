"""A/B of the one-wave-per-SIMD step-kernel instantiation (MJL_ONE_WAVE=1, launches of <= 4 x CUs envs)
against the two-wave one (MJL_ONE_WAVE=0): speed test and pooled env step at 1024 envs (one wave per
SIMD: the instantiation applies) and 2048 (control: two waves per SIMD, never applies). HIP events on
the launch stream, 100 launches after 10. One JSON line; run once per setting, interleaved."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjx  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402


def timed(fn, n=100, w=10):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us


m = mjx_amd.load_model("humanoid_mjx")
sys_ = mjx.put_model(m)
res = {"one_wave": os.environ.get("MJL_ONE_WAVE", "1")}
for B in (1024, 2048):
    d = mjx.make_data(sys_, B)
    d.set_option(mjx_amd.abi.OPT_STORE_DERIVED, 0)
    vel = torch.linspace(0, 1, B, device="cuda")
    out = torch.empty_like(vel)
    res[f"speedtest_{B}_us"] = timed(lambda: mjx.speedtest_step(sys_, d, vel, out))
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    env = HumanoidEnv(sys_, cfg, B, seed=1)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    act = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
    for _ in range(50):
        env.step(act)
    env.enable_reset_pool(16)
    npool = torch.tensor([16], dtype=torch.int32, device="cuda")
    env.fill_reset_pool(npool)
    res[f"envstep_pool_{B}_us"] = timed(lambda: env.step(act), n=60)
    env.enable_reset_pool(0)
    res[f"envstep_inplace_{B}_us"] = timed(lambda: env.step(act), n=60)
    del env, d
print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)

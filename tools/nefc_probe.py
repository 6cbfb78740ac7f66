"""Diagnostic: constraint-row counts (nefc) the PPO env step meets: 2048 envs, random actions with
auto-reset for 400 steps; fraction of envs above the 48 LDS rows per step and the maximum."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjx  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402

m = mjx_amd.load_model("humanoid_mjx")
cfg = resolve_ids(m, reference_ppo_config().env_config)
B = 2048
env = HumanoidEnv(mjx.put_model(m), cfg, B, seed=1, store_derived=True)
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
over, mx, it_mx, ncon_mx = [], 0, 0, 0
for t in range(400):
    env.step(torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1)
    st = env.data.get("stats")
    nefc = st[:, 1]
    over.append(float((nefc > 48).float().mean()))
    mx = max(mx, int(nefc.max()))
    it_mx = max(it_mx, int(st[:, 2].max()))
    ncon_mx = max(ncon_mx, int(st[:, 0].max()))
    if t % 50 == 0:
        print(f"step {t}: nefc mean {float(nefc.mean()):.1f} max {int(nefc.max())}, >48 {over[-1]:.4f}, "
              f"iters mean {float(st[:, 2].mean()):.2f} max {int(st[:, 2].max())}, ncon max {int(st[:, 0].max())}", flush=True)
print(f"overall: envs above 48 rows {sum(over) / len(over):.4f} per step; max nefc {mx}, max iterations {it_mx}, max ncon {ncon_mx}")

"""Cotangent growth along the APG reverse sweep (CG 4/4): one loss_and_grad at B x H, recording per
reverse step the median and max |state cotangent| over the envs still in the gradient and the
number cut as non-finite so far.  python tools/vjp_chain_probe.py [unrolled|implicit] [B H]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mujoco-mjx-lab_amd")]
import torch  # noqa: E402

from mjx_amd import apg, mjx  # noqa: E402
from mjx_amd.config import APGConfig, EnvConfig  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402
from train_apg import apg_model  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "unrolled"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
H = int(sys.argv[3]) if len(sys.argv) > 3 else 128
cfg = APGConfig()
cfg.batch_size, cfg.horizon = B, H
m = apg_model(cfg)
env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), B, seed=cfg.seed)


class Rec(apg.HumanoidAPGEnv):
    log = []

    def step_vjp(self, act, gq, gv, grew, gaux, nonfinite=None):
        out = super().step_vjp(act, gq, gv, grew, gaux, nonfinite)
        n = torch.cat([out[0], out[1]], 1).abs().amax(1)
        live = n > 0
        self.log.append((float(n[live].median()) if live.any() else 0.0, float(n.max()),
                         float(nonfinite[0]) if nonfinite is not None else 0.0, int(live.sum())))
        return out


tr = apg.APGTrainer(cfg, Rec(env, mode), device="cuda")
loss, _, _, dropped = tr.loss_and_grad(use_norm=False)
print(f"{mode}: loss {float(loss):.4g}, dropped {float(dropped):.0f}")
for k, (med, mx, nf, live) in enumerate(Rec.log):
    if k % 8 == 0 or k == len(Rec.log) - 1:
        print(f"reverse step {k:3d} (t={H - 1 - k:3d}): live {live:5d} median |g| {med:.3g} max {mx:.3g} cut so far {nf:.0f}")

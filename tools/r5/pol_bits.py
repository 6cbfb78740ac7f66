"""Round 5: the rollout policy kernel's outputs on fixed inputs (reference-size policy, 1024 and 37 envs),
saved for a bit-for-bit comparison between two builds (MJX355_LIB).  python tools/r5/pol_bits.py OUT.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

from mjx_amd import ppo  # noqa: E402

out = {}
for B in (1024, 37):
    g = torch.Generator().manual_seed(4)
    pol = ppo.GaussianPolicy(54, 21, [(256, "tanh")] * 3, 0.0, g)
    with torch.no_grad():
        for lin in pol.mlp.layers:
            lin.bias.normal_(0.0, 0.3, generator=g)
    pol = pol.cuda()
    gd = torch.Generator(device="cuda").manual_seed(B)
    x = torch.randn((B, 54), generator=gd, device="cuda") * 3
    rms = ppo.RunningMeanStd(54, "cuda")
    rms.mean.copy_(torch.randn(54, generator=gd, device="cuda"))
    rms.var.copy_(torch.rand(54, generator=gd, device="cuda") + 0.5)
    eps = torch.randn((B, 21), generator=gd, device="cuda")
    act, lp = torch.empty((B, 21), device="cuda"), torch.empty(B, device="cuda")
    ppo.policy_fwd_native(x, rms.mean, rms.var, 10.0, ppo.pack_policy_params(pol), ppo.policy_fused_dims(pol),
                          pol.log_std, eps, act, lp)
    out[B] = (act.cpu(), lp.cpu())
torch.save(out, sys.argv[1])
print("saved", sys.argv[1])

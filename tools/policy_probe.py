"""Times mjl_policy_fwd (the rollout step's fused policy forward) at the trainer's batch sizes with
the reference's policy (obs 54, 3 x 256 tanh, act 21); MJL_POLICY_MFMA=1 selects the 16-env MFMA
kernel, the default the R-env vector kernel. Prints one JSON line per batch size."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
from mjx_amd import ppo  # noqa: E402


def main():
    g = torch.Generator().manual_seed(4)
    gd = torch.Generator(device="cuda").manual_seed(4)
    pol = ppo.GaussianPolicy(54, 21, [(256, "tanh")] * 3, 0.0, g).cuda()
    dims = ppo.policy_fused_dims(pol)
    params = ppo.pack_policy_params(pol)
    rms = ppo.RunningMeanStd(54, "cuda")
    for B in (1024, 2048, 4096):
        x = torch.randn((B, 54), generator=gd, device="cuda")
        eps = torch.randn((B, 21), generator=gd, device="cuda")
        act, lp = torch.empty((B, 21), device="cuda"), torch.empty(B, device="cuda")
        for _ in range(20):
            ppo.policy_fwd_native(x, rms.mean, rms.var, 10.0, params, dims, pol.log_std, eps, act, lp)
        n = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(n):
            ppo.policy_fwd_native(x, rms.mean, rms.var, 10.0, params, dims, pol.log_std, eps, act, lp)
        e1.record()
        torch.cuda.synchronize()
        xn = torch.empty_like(x)
        ppo.obs_normalize_native(x, rms.mean, rms.var, 10.0, xn)
        with torch.no_grad():
            z = pol.mlp(xn)
        a_ref, l_ref = torch.empty_like(act), torch.empty_like(lp)
        ppo.policy_head_native(z, pol.log_std, eps, a_ref, l_ref)
        print(json.dumps({"B": B, "mfma": os.environ.get("MJL_POLICY_MFMA", "0"),
                          "us_per_call": e0.elapsed_time(e1) * 1e3 / n,
                          "max_abs_act_diff": float((act - a_ref).abs().max()),
                          "max_abs_logp_diff": float((lp - l_ref).abs().max())}), flush=True)


if __name__ == "__main__":
    main()

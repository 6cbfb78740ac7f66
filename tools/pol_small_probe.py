import json, os, sys, torch
sys.path.insert(0, os.path.join(os.getcwd(), "mujoco-mjx-lab_amd"))
from mjx_amd import ppo
for hid in ([16], [256], [256, 256], [256, 256, 256]):
    g = torch.Generator().manual_seed(4)
    gd = torch.Generator(device="cuda").manual_seed(4)
    pol = ppo.GaussianPolicy(54, 21, [(h, "tanh") for h in hid], 0.0, g).cuda()
    dims = ppo.policy_fused_dims(pol); params = ppo.pack_policy_params(pol)
    rms = ppo.RunningMeanStd(54, "cuda")
    B = 1024
    x = torch.randn((B, 54), generator=gd, device="cuda"); eps = torch.randn((B, 21), generator=gd, device="cuda")
    act, lp = torch.empty((B, 21), device="cuda"), torch.empty(B, device="cuda")
    for _ in range(20):
        ppo.policy_fwd_native(x, rms.mean, rms.var, 10.0, params, dims, pol.log_std, eps, act, lp)
    # graph of 50 launches: no host cost between kernels
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for _ in range(50):
                ppo.policy_fwd_native(x, rms.mean, rms.var, 10.0, params, dims, pol.log_std, eps, act, lp)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); 
    for _ in range(4): gr.replay()
    e1.record(); torch.cuda.synchronize()
    n = 200
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(n):
        ppo.policy_fwd_native(x, rms.mean, rms.var, 10.0, params, dims, pol.log_std, eps, act, lp)
    t1.record(); torch.cuda.synchronize()
    print(json.dumps({"hidden": hid, "us_graph": e0.elapsed_time(e1) * 1e3 / 200, "us_eager": t0.elapsed_time(t1) * 1e3 / n}), flush=True)

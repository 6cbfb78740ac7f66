"""Rollout as S independent env shards on S streams (each shard its own HumanoidEnv of B / S envs,
its own 256-step hipGraph of fused policy + env step) against one B-env rollout. A launch lasts as
long as its slowest env; a shard's step waits only for the slowest of its own envs, so the shards'
chains drift apart instead of every step paying the whole batch's slowest env. Prints one JSON line
per S: ms per 256-step rollout (median of 5 replays after 3) and mean env-step kernel time."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import mjx_amd  # noqa: E402
from mjx_amd import mjx, ppo  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402


def run(B: int, S: int, T: int = 256, reps: int = 5):
    cfg = reference_ppo_config()
    m = mjx_amd.load_model("humanoid_mjx")
    sys_ = mjx.put_model(m)
    ecfg = resolve_ids(m, cfg.env_config)
    n = B // S
    envs = [HumanoidEnv(sys_, ecfg, n, device=0, seed=42 * 7919 + s) for s in range(S)]
    g = torch.Generator().manual_seed(42)
    pol = ppo.GaussianPolicy(envs[0].obs_dim, envs[0].act_dim, cfg.policy_hidden_layer_specs, 0.0, g).cuda()
    dims, params = ppo.policy_fused_dims(pol), ppo.pack_policy_params(pol)
    rms = ppo.RunningMeanStd(envs[0].obs_dim, "cuda")
    obs = torch.empty((T + 1, B, envs[0].obs_dim), device="cuda")
    act = torch.empty((T, B, envs[0].act_dim), device="cuda")
    eps = torch.randn((T, B, envs[0].act_dim), device="cuda") * 0.5
    logp, rew, term, trunc = (torch.empty((T, B), device="cuda") for _ in range(4))
    pool_n = []
    for s, e in enumerate(envs):
        e.enable_reset_pool(16)
        pool_n.append(torch.full((1,), 4, dtype=torch.int32, device="cuda"))
        obs[0, s * n:(s + 1) * n].copy_(e.reset())
    streams = [torch.cuda.Stream() for _ in range(S)]
    graphs = []
    torch.cuda.synchronize()
    for s, e in enumerate(envs):
        sl = slice(s * n, (s + 1) * n)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(streams[s]):
            with torch.cuda.graph(gr, stream=streams[s]):
                e.fill_reset_pool(pool_n[s], counter=0)
                for t in range(T):
                    ppo.policy_fwd_native(obs[t, sl], rms.mean, rms.var, 10.0, params, dims, pol.log_std, eps[t, sl],
                                          act[t, sl], logp[t, sl])
                    e.step(act[t, sl], out=(obs[t + 1, sl], rew[t, sl], term[t, sl], trunc[t, sl]), counter=t + 1)
        graphs.append(gr)
    torch.cuda.synchronize()
    times = []
    main = torch.cuda.current_stream()
    for r in range(3 + reps):
        for e in envs:
            e.ctr_base.fill_(e.counter)
            e.counter += T
        obs[0].copy_(obs[T])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        for s in range(S):
            streams[s].wait_stream(main)
            with torch.cuda.stream(streams[s]):
                graphs[s].replay()
        for s in range(S):
            main.wait_stream(streams[s])
        e1.record(main)
        torch.cuda.synchronize()
        if r >= 3:
            times.append(e0.elapsed_time(e1))
    done = float((torch.maximum(term, trunc) > 0.5).float().mean())
    return {"B": B, "shards": S, "envs_per_shard": n, "ms_per_rollout": statistics.median(times),
            "ms_all": [round(x, 3) for x in times], "us_per_step": statistics.median(times) * 1e3 / T,
            "done_frac_per_step": done}


def main():
    B = int(os.environ.get("PROBE_B", "1024"))
    for S in [int(x) for x in os.environ.get("PROBE_S", "1,2,4,8").split(",")]:
        print(json.dumps(run(B, S)), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

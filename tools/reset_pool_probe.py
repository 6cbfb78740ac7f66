"""Rollout timing with / without the reset pool (PPOTrainer reset_pool), graph replay and eager, at one
batch size; under rocprofv3 --kernel-trace the dispatch timestamps give the per-step kernels."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjx, ppo  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402


def run(n, pf, graph, reps):
    cfg = reference_ppo_config()
    cfg.num_envs = n
    m = mjx_amd.load_model("humanoid_mjx")
    ecfg = resolve_ids(m, cfg.env_config)
    env = HumanoidEnv(mjx.put_model(m), ecfg, n, seed=1)
    tr = ppo.PPOTrainer(cfg, env, None, device="cuda", use_graph=graph, reset_pool=16 if pf else 0)
    for _ in range(2):
        tr.collect_rollout()
    torch.cuda.synchronize()
    ts, dones = [], 0.0
    for _ in range(reps):
        t0 = time.time()
        r = tr.collect_rollout()
        torch.cuda.synchronize()
        ts.append(time.time() - t0)
        dones += float((torch.maximum(r[4], r[5]) > 0.5).sum())
    return {"envs": n, "reset_pool": pf, "graph": graph, "rollout_ms": 1e3 * min(ts),
            "rollout_ms_mean": 1e3 * sum(ts) / len(ts), "done_per_step": dones / reps / cfg.rollout_length}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    for pf in (False, True):
        for graph in (True, False):
            if a.only and a.only != f"{int(pf)}{int(graph)}":
                continue
            print(json.dumps(run(a.envs, pf, graph, a.reps)), flush=True)

"""PPO throughput on one MI355X (BASELINE config C3: src/config.json hyper-parameters).

python tools/bench_ppo.py [--envs 2048] [--rollout 256] [--iters 3] [--seed 42]
Prints one JSON line: synced env-steps/s per iteration (rollout + GAE + 4x(T*B/65536) minibatch
updates), the rollout / update split, and the training returns of the iterations run.
"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--rollout", type=int, default=256)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-fused-policy", action="store_true", help="rollout policy as normalise + torch MLP + head")
    ap.add_argument("--reset-pool", type=int, default=16, help="pooled auto-resets per env (0: in place only)")
    a = ap.parse_args()
    cfg = reference_ppo_config()
    cfg.num_envs, cfg.rollout_length, cfg.seed = a.envs, a.rollout, a.seed
    m = mjx_amd.load_model("humanoid_mjx")
    sys_ = mjx.put_model(m)
    ecfg = resolve_ids(m, cfg.env_config)
    env = HumanoidEnv(sys_, ecfg, cfg.num_envs, seed=cfg.seed)
    tr = ppo.PPOTrainer(cfg, env, None, device="cuda", fused_policy=not a.no_fused_policy,
                        reset_pool=a.reset_pool)
    tr.iteration(0)  # warm-up (GEMM heuristics, allocator)
    tr.iteration(0)  # second rollout captures the rollout hipGraph
    res, t_roll = [], []
    for it in range(1, a.iters + 1):
        torch.cuda.synchronize()
        t0 = time.time()
        roll = tr.collect_rollout()
        torch.cuda.synchronize()
        t_roll.append(time.time() - t0)
        del roll
        res.append(tr.iteration(it))
    sps = [r["env_steps_per_sec"] for r in res]
    per_iter = cfg.num_envs * cfg.rollout_length / (sum(sps) / len(sps))
    rollout_s = sum(t_roll) / len(t_roll)
    print(json.dumps({
        "metric": "PPO env-steps/s (rollout + GAE + updates, synced)", "value": sum(sps) / len(sps),
        "envs": cfg.num_envs, "rollout_length": cfg.rollout_length, "minibatch": cfg.minibatch_size,
        "epochs": cfg.epochs, "iteration_s": per_iter, "rollout_s": rollout_s,
        "rollout_env_steps_per_s": cfg.num_envs * cfg.rollout_length / rollout_s,
        "train_return_avg": [r["train_return_avg"] for r in res]}))


if __name__ == "__main__":
    main()

"""PPO on the MI355X-native humanoid env (reference train_ppo.py CLI: --test / --config).

Single GPU:   python mujoco-mjx-lab_amd/train_ppo.py [--config path/config.json] [--iterations N]
Multi-GPU:    python -m torch.distributed.run --nproc-per-node G --master-addr 127.0.0.1 \\
                  mujoco-mjx-lab_amd/train_ppo.py --num-envs 8192 ...   (envs split across ranks)
Results go to results/<timestamp>_ppo/{config.json,logs/metrics.jsonl,checkpoints/} as in the
reference (src/checkpoint_utils.py:13-100).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjx  # noqa: E402
from mjx_amd.config import PPOConfig, reference_ppo_config  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402
from mjx_amd.ppo import PPOTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=None, help="reference-style config.json (env / ppo sections)")
    ap.add_argument("--test", action="store_true", help="tiny run (reference config_test.json spirit)")
    ap.add_argument("--iterations", type=int, default=None)
    ap.add_argument("--num-envs", type=int, default=None, help="total envs over all ranks")
    ap.add_argument("--model", default=None, help="humanoid_mjx | humanoid | path to .xml")
    ap.add_argument("--results-dir", default=None)
    ap.add_argument("--seed", type=int, default=None, help="override the config's seed")
    ap.add_argument("--jax-keys", action="store_true",
                    help="draw env resets from train_ppo.py's jax.random key chain (same reset stream as the reference)")
    a = ap.parse_args()

    cfg = PPOConfig.from_json(a.config) if a.config else reference_ppo_config()
    if a.test:
        cfg.num_envs, cfg.rollout_length, cfg.minibatch_size, cfg.total_iterations = 64, 16, 256, 3
        cfg.eval_interval = cfg.checkpoint_every = 2
    if a.num_envs:
        cfg.num_envs = a.num_envs
    if a.iterations:
        cfg.total_iterations = a.iterations
    if a.results_dir:
        cfg.results_dir = a.results_dir
    if a.seed is not None:
        cfg.seed = a.seed

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    model = mjx_amd.load_model(a.model or os.path.splitext(os.path.basename(cfg.xml_path))[0])
    sys_ = mjx.put_model(model)
    env_cfg = resolve_ids(model, cfg.env_config)
    env = HumanoidEnv(sys_, env_cfg, cfg.num_envs // world, device=local, seed=cfg.seed * 7919 + rank)
    eval_env = HumanoidEnv(sys_, env_cfg, 32, device=local, seed=cfg.seed + 10000) if rank == 0 else None
    out = None
    if rank == 0:
        out = os.path.join(cfg.results_dir, time.strftime("%Y%m%d_%H%M%S") + "_ppo")
    tr = PPOTrainer(cfg, env, eval_env, device=f"cuda:{local}", dist=dist, out_dir=out, jax_keys=a.jax_keys)
    tr.train()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""APG (backward-through-physics) on the MI355X-native humanoid env (reference train_apg.py).

Single GPU:   python mujoco-mjx-lab_amd/train_apg.py [--batch-size 2048 --horizon 128] [--steps N]
Multi-GPU:    python -m torch.distributed.run --nproc-per-node G --master-addr 127.0.0.1 \\
                  mujoco-mjx-lab_amd/train_apg.py --batch-size 8192 ...   (envs split across ranks)

Model options follow train_apg.py:101-112 + src/training_utils.py:95-103: `lighten_solver` sets
iterations = ls_iterations = 1, then the script's solver_options override to CG with 4/4.
Results go to results/<timestamp>_apg/{config.json,logs/metrics.jsonl,checkpoints/}.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjcf, mjx  # noqa: E402
from mjx_amd.apg import APGTrainer, HumanoidAPGEnv  # noqa: E402
from mjx_amd.config import APGConfig  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402


def apg_model(cfg: APGConfig, name: str = None, solver: str = "cg"):
    """Model with the APG solver options (training_utils.py:95-103, train_apg.py:101-105).
    solver="model" keeps the MJCF's own solver (Newton 10/20 for humanoid_mjx): the reference forces
    CG 4/4 because JAX differentiates through the Newton iterations (train_apg.py:101); with the
    implicit VJP (the converged optimality conditions) Newton is usable, and it avoids the
    truncated-solve blow-ups (DESIGN.md "Truncated solves")."""
    m = mjx_amd.load_model(name or os.path.splitext(os.path.basename(cfg.xml_path))[0])
    if solver == "model":
        return m
    if cfg.lighten_solver:
        m.iterations, m.ls_iterations = 1, 1
    m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=None, help="total envs over all ranks")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--model", default=None, help="humanoid_mjx | humanoid | path to .xml")
    ap.add_argument("--solver", default="cg", choices=["cg", "model"],
                    help="cg = train_apg.py's CG 4/4 override; model = the MJCF's solver")
    ap.add_argument("--vjp", default=None, choices=["unrolled", "implicit"],
                    help="solver derivative: unrolled = jax.grad through the iterations (default with --solver cg), "
                         "implicit = at the converged active set (default with --solver model)")
    ap.add_argument("--results-dir", default=None)
    ap.add_argument("--rms-in-loss-only", action="store_true",
                    help="observation statistics only from the observations of envs still in the loss "
                         "(APGConfig.rms_in_loss_only; not the reference's rule, which takes every rollout "
                         "observation, train_apg.py:290-292 -- the default)")
    ap.add_argument("--rms-all-obs", action="store_true", help="the default (kept for old command lines)")
    ap.add_argument("--rms-freeze-after", type=int, default=None,
                    help="no observation-statistics updates after this update (APGConfig.rms_freeze_after; not "
                         "the reference's rule, which updates them every 10 updates, train_apg.py:290-292)")
    a = ap.parse_args()

    cfg = APGConfig()
    for k in ("batch_size", "horizon", "lr", "seed"):
        if getattr(a, k) is not None:
            setattr(cfg, k, getattr(a, k))
    if a.steps:
        cfg.total_steps = a.steps
    if a.results_dir:
        cfg.results_dir = a.results_dir
    cfg.rms_in_loss_only = bool(a.rms_in_loss_only) and not a.rms_all_obs
    cfg.rms_freeze_after = a.rms_freeze_after

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    model = apg_model(cfg, a.model, a.solver)
    from mjx_amd.config import EnvConfig
    env = HumanoidEnv(mjx.put_model(model), resolve_ids(model, EnvConfig()), cfg.batch_size // world,
                      device=local, seed=cfg.seed * 7919 + rank)
    out = os.path.join(cfg.results_dir, time.strftime("%Y%m%d_%H%M%S") + "_apg") if rank == 0 else None
    vjp = a.vjp or ("unrolled" if a.solver == "cg" else "implicit")
    tr = APGTrainer(cfg, HumanoidAPGEnv(env, vjp), device=f"cuda:{local}", dist=dist, out_dir=out)
    tr.train()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""APG throughput on one MI355X (BASELINE config C4: train_apg.py, 2048 envs x 128 horizon,
backward through the simulator, CG 4/4 solver override, hidden 32x2, lr 5e-5, clip 0.3).

python tools/bench_apg.py [--envs 2048] [--horizon 128] [--updates 5]
Prints one JSON line: synced env-steps/s per update (rollout forward + VJP sweep + Adam), the
forward / backward split, and the returns of the updates run.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

from mjx_amd import mjx  # noqa: E402
from mjx_amd.apg import APGTrainer, HumanoidAPGEnv  # noqa: E402
from mjx_amd.config import APGConfig, EnvConfig  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402
from train_apg import apg_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--horizon", type=int, default=128)
    ap.add_argument("--updates", type=int, default=5)
    ap.add_argument("--solver", default="cg", choices=["cg", "model"], help="cg = train_apg.py override")
    ap.add_argument("--vjp", default=None, choices=["unrolled", "implicit"],
                    help="default: unrolled with --solver cg (jax.grad semantics), implicit with --solver model")
    a = ap.parse_args()
    vjp = a.vjp or ("unrolled" if a.solver == "cg" else "implicit")
    cfg = APGConfig()
    cfg.batch_size, cfg.horizon = a.envs, a.horizon
    m = apg_model(cfg, solver=a.solver)
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), cfg.batch_size, seed=cfg.seed)
    tr = APGTrainer(cfg, HumanoidAPGEnv(env, vjp), device="cuda")
    tr.update(0)  # warm-up (eager: library handles, GEMM choices)
    tr.update(1)  # captures the rollout + reverse sweep hipGraph (one-time)
    res = [tr.update(i) for i in range(2, a.updates + 2)]
    sps = sum(r["env_steps_per_sec"] for r in res) / len(res)
    # forward-only rollout time for the split (no tape, no backward)
    torch.cuda.synchronize()
    t0 = time.time()
    env.reset()
    for _ in range(cfg.horizon):
        o = torch.cat([env.data.get("qpos"), env.data.get("qvel")], 1)
        with torch.no_grad():
            act = tr.policy(o)
        env.step(act, auto_reset=False)
    torch.cuda.synchronize()
    fwd = time.time() - t0
    upd = cfg.batch_size * cfg.horizon / sps
    print(json.dumps({
        "metric": "APG env-steps/s (rollout + backward through sim + Adam, synced)", "value": sps,
        "envs": cfg.batch_size, "horizon": cfg.horizon, "solver": a.solver, "vjp": vjp, "update_s": upd,
        "forward_rollout_s": fwd, "backward_s_est": upd - fwd,
        "returns": [r["return"] for r in res], "grad_norms": [r["grad_norm"] for r in res],
        "nonfinite_envs": [r["nonfinite_envs"] for r in res]}))


if __name__ == "__main__":
    main()

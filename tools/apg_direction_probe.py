"""Why APG's return falls at BASELINE C4: a training run at 2048 x 128, CG 4/4
(train_apg.py:101-105), and at chosen updates a directional check on that update's own resets:
loss(theta0 + eps * step) for eps = 0.1, 1, 10, where step = theta1 - theta0 is the Adam step the
trainer took (the clipped gradient through Adam, lr 5e-5) and theta0's loss the one the update
computed; the observation statistics held at their pre-update values for every evaluation.
Per probed update it also logs the envs in the loss per step (first / last step / mean), the
per-env action-cotangent energy sum_t |dL/da_t|^2 (quantiles: the per-env gradient's size
through the policy) and the gradient norm before the clip. One JSON line per probed update.

python tools/apg_direction_probe.py VJP UPDATES [--rms-in-loss-only] [--probe 0,25,...] [--env-seed S]
    [--freeze-rms-after N] [--all-updates]
--all-updates: at EVERY update, the loss after the step on that update's own resets (one extra
rollout per update) beside the loss before it: the same-batch improvement rate; --freeze-rms-after N:
no observation-statistics updates after update N (is the decline the statistics' drift?)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-mjx-lab_amd")]
import torch  # noqa: E402

from mjx_amd import mjx  # noqa: E402
from mjx_amd.apg import APGTrainer, HumanoidAPGEnv  # noqa: E402
from mjx_amd.config import APGConfig, EnvConfig  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402
from train_apg import apg_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("vjp", choices=["implicit", "unrolled"])
    ap.add_argument("updates", type=int)
    ap.add_argument("--rms-in-loss-only", action="store_true")
    ap.add_argument("--probe", default="0,10,50,99,100,110,150,200,250,299")
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--horizon", type=int, default=128)
    ap.add_argument("--env-seed", type=int, default=None, help="env reset seed (default cfg.seed; train_apg.py "
                    "uses cfg.seed * 7919)")
    ap.add_argument("--freeze-rms-after", type=int, default=None)
    ap.add_argument("--all-updates", action="store_true")
    a = ap.parse_args()
    probe = {int(x) for x in a.probe.split(",") if x}
    cfg = APGConfig()
    cfg.batch_size, cfg.horizon = a.envs, a.horizon
    cfg.rms_in_loss_only = bool(a.rms_in_loss_only)
    m = apg_model(cfg, solver="cg")
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), cfg.batch_size,
                      seed=cfg.seed if a.env_seed is None else a.env_seed)
    aenv = HumanoidAPGEnv(env, a.vjp)
    tr = APGTrainer(cfg, aenv, device="cuda", use_graph=False)
    params = list(tr.policy.parameters())
    for it in range(a.updates):
        if a.freeze_rms_after is not None and it > a.freeze_rms_after:
            cfg.rms_update_every = 10 ** 9
        if a.all_updates and it not in probe:  # the step's effect on its own batch
            c0 = env.counter
            rms0 = (tr.rms.mean.clone(), tr.rms.var.clone(), tr.rms.count.clone())
            met = tr.update(it)
            rms1 = (tr.rms.mean, tr.rms.var, tr.rms.count)
            use_norm = it >= cfg.obs_warmup_steps and cfg.normalize_observations
            tr.rms.mean, tr.rms.var, tr.rms.count = rms0
            env.counter = c0
            with torch.no_grad(), torch.enable_grad():
                after = float(tr.loss_and_grad(use_norm)[0])
            tr.rms.mean, tr.rms.var, tr.rms.count = rms1
            print(json.dumps({"update": it, "return": met["return"], "loss_before": met["loss"], "loss_after": after,
                              "improved": after < met["loss"]}), flush=True)
            continue
        if it not in probe:
            tr.update(it)
            continue
        tr.diag = {}
        c0 = env.counter
        rms0 = (tr.rms.mean.clone(), tr.rms.var.clone(), float(tr.rms.count) if not torch.is_tensor(tr.rms.count)
                else tr.rms.count.clone())
        th0 = [p.detach().clone() for p in params]
        met = tr.update(it)
        ga_sq = tr.diag["ga_sq"]
        tr.diag = None
        th1 = [p.detach().clone() for p in params]
        rms1 = (tr.rms.mean.clone(), tr.rms.var.clone(), tr.rms.count.clone() if torch.is_tensor(tr.rms.count)
                else float(tr.rms.count))
        use_norm = it >= cfg.obs_warmup_steps and cfg.normalize_observations
        tr.rms.mean, tr.rms.var, tr.rms.count = rms0
        losses = {}
        with torch.no_grad():
            for eps in (0.0, 0.1, 1.0, 10.0):
                for p, x0, x1 in zip(params, th0, th1):
                    p.copy_(x0 + eps * (x1 - x0))
                env.counter = c0
                with torch.enable_grad():
                    loss, _, traj, dropped = tr.loss_and_grad(use_norm)
                losses[str(eps)] = float(loss)
                if eps == 0.0:
                    alive = traj[1].float().sum(1)  # envs in the loss per step
            for p, x1 in zip(params, th1):
                p.copy_(x1)
        tr.rms.mean, tr.rms.var, tr.rms.count = rms1
        q = torch.quantile(ga_sq.float().sqrt().cpu(), torch.tensor([0.5, 0.9, 0.99, 1.0])).tolist()
        step_norm = float(torch.sqrt(sum(((x1 - x0) ** 2).sum() for x0, x1 in zip(th0, th1))))
        print(json.dumps({
            "update": it, "vjp": a.vjp, "use_norm": bool(use_norm), "rms_in_loss_only": cfg.rms_in_loss_only,
            "loss_update": met["loss"], "return": met["return"], "grad_norm_preclip": met["grad_norm"],
            "loss_at_eps": losses, "descent": {k: losses[k] < losses["0.0"] for k in ("0.1", "1.0", "10.0")},
            "step_norm": step_norm, "reverse_nonfinite_envs": met["reverse_nonfinite_envs"],
            "forward_dropped_envs": met["forward_dropped_envs"],
            "envs_in_loss": {"step0": float(alive[0]), "last": float(alive[-1]), "mean": float(alive.mean())},
            "ga_norm_quantiles_p50_p90_p99_max": q}), flush=True)


if __name__ == "__main__":
    main()

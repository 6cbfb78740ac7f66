"""Where one C3 PPO iteration goes (1024 envs x 256 x 4 epochs, minibatch 65,536): rollout (one
hipGraph replay), the between-phase work (observation statistics, value net over (T + 1) B
observations, GAE, minibatch permutations) and the update (16 minibatch graph replays), timed with
events on the trainer's stream after 2 warm-up iterations (graph capture). One JSON line.

PROBE_B=envs (default 1024); PROBE_MB=rows: the minibatch rows of one rank. With PROBE_DP=1 the
trainer runs its data-parallel path on a one-rank gloo group (graph A, the all-reduce of both nets'
gradients, graph B per minibatch), so PROBE_MB=8192 is one C5 rank's update at 8 GPUs (128
minibatch steps) without the other ranks' link time."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-mjx-lab_amd")]
import bench  # noqa: E402
from mjx_amd.ppo import compute_gae, make_index_batches  # noqa: E402


def main():
    args = bench.parse()
    dist = None
    backend = {"1": "gloo", "gloo": "gloo", "nccl": "nccl"}.get(os.environ.get("PROBE_DP", ""))
    if backend:  # PROBE_DP=nccl: RCCL on one rank (the all-reduce stays on the stream, as at 8 GPUs)
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(bench.free_port()))
        torch.cuda.set_device(0)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=0, world_size=1)
    tr = bench.ppo_trainer(args, int(os.environ.get("PROBE_B", "1024")), dist, 0, 0)
    if os.environ.get("PROBE_MB"):
        tr.cfg.minibatch_size = int(os.environ["PROBE_MB"])
    for it in range(2):
        tr.iteration(it)
    cfg, dev = tr.cfg, tr.device
    ms = {"rollout": [], "between": [], "update": [], "total": []}
    ar_ms, n_ar = [], []
    for _ in range(5):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        torch.cuda.synchronize()
        ev[0].record()
        obs_t, act_t, logp_t, r_t, te_t, tr_t = tr.collect_rollout()
        ev[1].record()
        T, B = r_t.shape
        tr.rms.update(obs_t, None)
        with torch.no_grad():
            obs_n = tr.rms.normalize(obs_t)
            last_n = tr.rms.normalize(tr.obs)
            v = tr.value(torch.cat([obs_n, last_n[None]], 0).reshape((T + 1) * B, -1)).reshape(T + 1, B)
            adv, ret = compute_gae(r_t, v, te_t, tr_t, cfg.gamma, cfg.lam)
        idx = make_index_batches(T * B, cfg.minibatch_size, cfg.epochs, tr.idx_gen, dev)
        ev[2].record()
        evs = [] if dist is not None else None
        tr.updater.run(obs_n.reshape(T * B, -1), act_t.reshape(T * B, -1), logp_t.reshape(-1), ret.reshape(-1),
                       adv.reshape(-1), idx, evs)
        ev[3].record()
        torch.cuda.synchronize()
        ms["rollout"].append(ev[0].elapsed_time(ev[1]))
        ms["between"].append(ev[1].elapsed_time(ev[2]))
        ms["update"].append(ev[2].elapsed_time(ev[3]))
        ms["total"].append(ev[0].elapsed_time(ev[3]))
        if evs is not None:
            from mjx_amd.ppo import event_ms
            ar_ms.append(sum(event_ms(e) for e in evs))
            n_ar.append(len(evs))
    line = {k: round(statistics.median(v), 3) for k, v in ms.items()}
    line.update(envs=tr.env.num_envs, minibatch_rows=int(idx.shape[1]), minibatches=int(idx.shape[0]),
                data_parallel=dist is not None)
    if ar_ms:
        line.update(allreduce_total_ms=round(statistics.median(ar_ms), 3), allreduces=n_ar[0],
                    allreduce_backend=f"{backend}, one rank (no link time)")
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    sys.argv = sys.argv[:1]
    main()

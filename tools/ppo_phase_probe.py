"""Where one C3 PPO iteration goes (1024 envs x 256 x 4 epochs, minibatch 65,536): rollout (one
hipGraph replay), the between-phase work (observation statistics, value net over (T + 1) B
observations, GAE, minibatch permutations) and the update (16 minibatch graph replays), timed with
events on the trainer's stream after 2 warm-up iterations (graph capture). One JSON line."""
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
    tr = bench.ppo_trainer(args, int(os.environ.get("PROBE_B", "1024")), None, 0, 0)
    for it in range(2):
        tr.iteration(it)
    cfg, dev = tr.cfg, tr.device
    ms = {"rollout": [], "between": [], "update": [], "total": []}
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
        tr.updater.run(obs_n.reshape(T * B, -1), act_t.reshape(T * B, -1), logp_t.reshape(-1), ret.reshape(-1),
                       adv.reshape(-1), idx, None)
        ev[3].record()
        torch.cuda.synchronize()
        ms["rollout"].append(ev[0].elapsed_time(ev[1]))
        ms["between"].append(ev[1].elapsed_time(ev[2]))
        ms["update"].append(ev[2].elapsed_time(ev[3]))
        ms["total"].append(ev[0].elapsed_time(ev[3]))
    print(json.dumps({k: round(statistics.median(v), 3) for k, v in ms.items()}), flush=True)


if __name__ == "__main__":
    sys.argv = sys.argv[:1]
    main()

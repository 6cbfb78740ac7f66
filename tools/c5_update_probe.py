"""One rank's C5 PPO update (bench.c5_rank_update: 1024 envs x 256 steps, 4 epochs x 32 minibatches of
8,192 rows through the data-parallel update graphs, identity collective), REPS medians, one JSON line.
Under rocprofv3 --kernel-trace it gives the per-kernel breakdown of the minibatch step.
    python tools/c5_update_probe.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-mjx-lab_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    torch.cuda.set_device(0)
    out = bench.c5_rank_update(0, reps=5)
    runs = [out["ppo_c5_rank_update_ms"]]
    for _ in range(reps - 1):
        runs.append(bench.c5_rank_update(0, reps=5)["ppo_c5_rank_update_ms"])
    out["runs_ms"] = runs
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

#!/bin/bash
# Round-4 seed spread of the PPO return curve: seeds 42..46 at 1024 envs (BASELINE
# C3) and 2048 envs (src/config.json), 400 iterations each, the reference's hyper-parameters;
# metrics.jsonl per run under gpurun_out/ppo_seeds_r4/ (summarised by tools/summarize_seeds.py).
set -o pipefail
O=gpurun_out/ppo_seeds_r4; mkdir -p $O
for B in 1024 2048; do
  for S in 42 43 44 45 46; do
    timeout -k 10 300 python -u mujoco-mjx-lab_amd/train_ppo.py --seed $S --num-envs $B --iterations 400 \
      --results-dir $O/s${S}_b$B > $O/s${S}_b$B.log 2>&1 || { tail -5 $O/s${S}_b$B.log; exit 1; }
    f=$(ls $O/s${S}_b$B/*/logs/metrics.jsonl) && cp $f $O/s${S}_b$B.metrics.jsonl && rm -rf $O/s${S}_b$B
    tail -1 $O/s${S}_b$B.metrics.jsonl | cut -c1-200
  done
done

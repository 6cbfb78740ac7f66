#!/bin/bash
# BASELINE config C3: PPO with src/config.json hyper-parameters, seeds 42/43/44 at B=2048 and seed 42
# at B=1024 (README), 500 iterations each, plus seed 42 with train_ppo.py's jax.random reset-key
# chain. Each run has its own time limit; chained with &&.
set -o pipefail
mkdir -p gpurun_out/curves
export TMPDIR=/tmp
run() {  # name, extra args (checkpoints are dropped: gpurun_out travels back only under 64 MiB)
  timeout -k 10 400 python mujoco-mjx-lab_amd/train_ppo.py --iterations 500 --results-dir gpurun_out/curves/$1 "${@:2}" \
      > gpurun_out/curves/$1.log 2>&1 && rm -rf gpurun_out/curves/$1/*/checkpoints
}
run s42_b2048 --num-envs 2048 &&
run s43_b2048 --num-envs 2048 --config tools/configs/seed43.json &&
run s44_b2048 --num-envs 2048 --config tools/configs/seed44.json &&
run s42_b1024 --num-envs 1024 &&
run s42_b2048_jaxkeys --num-envs 2048 --jax-keys

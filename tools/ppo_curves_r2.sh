#!/bin/bash
# Learning check of the current trainer (reset pool, fused policy, native losses): seed 42 at 2048
# and at C3's 1024 envs, 500 iterations each (src/config.json hyper-parameters).
set -o pipefail
mkdir -p gpurun_out/curves2
export TMPDIR=/tmp
run() {
  timeout -k 10 400 python mujoco-mjx-lab_amd/train_ppo.py --iterations 500 --results-dir gpurun_out/curves2/$1 "${@:2}" \
      > gpurun_out/curves2/$1.log 2>&1 && rm -rf gpurun_out/curves2/$1/*/checkpoints
}
run s42_b2048 --num-envs 2048 &&
run s42_b1024 --num-envs 1024

#!/bin/bash
# APG learning check at BASELINE config C4 size (train_apg.py: 2048 envs x 128 horizon, CG 4/4 solver
# override, hidden 32x2, lr 5e-5, clip 0.3): 300 updates with the implicit VJP, and 100 with the
# reference's unrolled (jax.grad) semantics; metrics.jsonl per run under gpurun_out/apgc4.
mkdir -p gpurun_out/apgc4
export TMPDIR=/tmp
timeout -k 10 400 python -u mujoco-mjx-lab_amd/train_apg.py --batch-size 2048 --horizon 128 --steps 300 --vjp implicit \
    --results-dir gpurun_out/apgc4/implicit > gpurun_out/apgc4/implicit.log 2>&1 || exit $?
timeout -k 10 300 python -u mujoco-mjx-lab_amd/train_apg.py --batch-size 2048 --horizon 128 --steps 100 --vjp unrolled \
    --results-dir gpurun_out/apgc4/unrolled > gpurun_out/apgc4/unrolled.log 2>&1 || exit $?
rm -rf gpurun_out/apgc4/*/*/checkpoints

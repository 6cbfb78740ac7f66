#!/bin/bash
# APG learning check (BASELINE config C4: 2048 envs x 128 horizon, train_apg.py's CG 4/4 solver
# override, implicit VJP): 300 updates, metrics.jsonl under gpurun_out/apgcurve.
set -o pipefail
mkdir -p gpurun_out/apgcurve
export TMPDIR=/tmp
timeout -k 10 600 python mujoco-mjx-lab_amd/train_apg.py --steps 300 --vjp implicit --results-dir gpurun_out/apgcurve/cg44_implicit \
    > gpurun_out/apgcurve/cg44_implicit.log 2>&1 && rm -rf gpurun_out/apgcurve/cg44_implicit/*/checkpoints

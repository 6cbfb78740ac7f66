#!/bin/bash
# APG learning check at BASELINE config C4 size (train_apg.py: 2048 envs x 128 horizon, CG 4/4 solver
# override, hidden 32x2, lr 5e-5, clip 0.3): 300 updates with the reference's unrolled (jax.grad)
# semantics and with the implicit VJP, observation statistics from in-loss observations (default);
# then 150 unrolled updates with every observation in the statistics (the reference's rule).
# metrics.jsonl per run under gpurun_out/apgc4.
mkdir -p gpurun_out/apgc4
export TMPDIR=/tmp
run() {  # name steps vjp [extra]
  timeout -k 10 400 python -u mujoco-mjx-lab_amd/train_apg.py --batch-size 2048 --horizon 128 --steps $2 --vjp $3 $4 \
      --results-dir gpurun_out/apgc4/$1 > gpurun_out/apgc4/$1.log 2>&1
}
run unrolled 300 unrolled && run implicit 300 implicit && run unrolled_allobs 150 unrolled --rms-all-obs
rc=$?
rm -rf gpurun_out/apgc4/*/*/checkpoints
exit $rc

#!/bin/bash
# Round-4 APG learning check at BASELINE C4 (train_apg.py: 2048 envs x 128 horizon, CG 4/4, hidden 32x2,
# lr 5e-5, clip 0.3, normalisation from update 100): 300 updates each, implicit and unrolled VJP, with
# the opt-in in-loss observation statistics (--rms-in-loss-only); the reference rule (the default)
# collapses at update 100 in both modes (profiles/r4/apg_direction_*_ref.jsonl). metrics.jsonl per run.
set -o pipefail
O=gpurun_out/apgc4_r4; mkdir -p $O
export TMPDIR=/tmp
run() {  # name steps vjp [extra]
  timeout -k 10 400 python -u mujoco-mjx-lab_amd/train_apg.py --batch-size 2048 --horizon 128 --steps $2 --vjp $3 $4 \
      --results-dir $O/$1 > $O/$1.log 2>&1 || return $?
  f=$(ls $O/$1/*/logs/metrics.jsonl) && cp $f $O/$1.metrics.jsonl && rm -rf $O/$1
}
run implicit_inloss 300 implicit --rms-in-loss-only && run unrolled_inloss 300 unrolled --rms-in-loss-only

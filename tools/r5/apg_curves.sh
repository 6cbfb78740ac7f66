#!/bin/bash
# Round-5 APG record at BASELINE C4 (train_apg.py: 2048 envs x 128 horizon, CG 4/4, hidden 32x2, lr 5e-5,
# clip 0.3, normalisation from update 100), 300 updates per run on the final sources: the reference's
# statistics rule (the default) with the implicit and the unrolled VJP, and the opt-in configuration
# (--rms-in-loss-only --rms-freeze-after 100, implicit). metrics.jsonl per run (reverse_nonfinite_envs:
# the unrolled VJP's cut envs per update).
set -o pipefail
O=gpurun_out/apgc4_r5; mkdir -p $O
export TMPDIR=/tmp
run() {  # name vjp [extra...]
  local name=$1 vjp=$2; shift 2
  timeout -k 10 400 python -u mujoco-mjx-lab_amd/train_apg.py --batch-size 2048 --horizon 128 --steps 300 --vjp $vjp "$@" \
      --results-dir $O/$name > $O/$name.log 2>&1 || return $?
  f=$(ls $O/$name/*/logs/metrics.jsonl) && cp $f $O/$name.metrics.jsonl && rm -rf $O/$name
  echo "$name done"
}
run implicit_ref implicit && run unrolled_ref unrolled && \
run implicit_inloss_frozen implicit --rms-in-loss-only --rms-freeze-after 100 && \
run unrolled_inloss_frozen unrolled --rms-in-loss-only --rms-freeze-after 100

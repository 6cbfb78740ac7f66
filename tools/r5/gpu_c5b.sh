#!/bin/bash
# round 5: one C5 rank's update phase through a one-rank RCCL group (tools/ppo_phase_probe.py, PROBE_DP=nccl,
# PROBE_MB=8192): eager collective between graphs (MJL_DP_CAPTURE=0) vs the collective captured in the
# minibatch step's graph (=1), one all-reduce vs two buckets; interleaved, 2 reps each. Then the DP graph
# test with capture on.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
for rep in 1 2; do
  for cfg in "0 0" "0 1" "1 0" "1 1"; do
    set -- $cfg
    MJL_DP_CAPTURE=$1 MJL_DP_BUCKETS=$2 PROBE_DP=nccl PROBE_MB=8192 timeout -k 10 240 python tools/ppo_phase_probe.py \
      > $O/probe_c$1_b$2_$rep.json 2> $O/probe_c$1_b$2_$rep.err || { echo "probe c=$1 b=$2 failed"; tail -5 $O/probe_c$1_b$2_$rep.err; exit 1; }
    echo "capture=$1 buckets=$2 rep=$rep $(tail -1 $O/probe_c$1_b$2_$rep.json)"
  done
done

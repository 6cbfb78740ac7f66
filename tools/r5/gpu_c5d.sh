#!/bin/bash
# round 5: thread-local graph capture (RCCL's watchdog event queries no longer invalidate a capture): the PPO,
# APG and DP GPU tests, then the one-rank RCCL C5 probe with buckets forced on (3 reps: the race that broke
# the rollout capture) and with the defaults.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ppo_graph.py tests/test_dp_gpu.py tests/test_ppo.py tests/test_apg.py -m gpu -x -q \
  --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2
if [ $rc -ne 0 ]; then grep -B5 -A40 "^____" $O/pytest.log | head -80; exit $rc; fi
for run in b1_1 b1_2 b1_3 bauto_1; do
  b=${run%_*}; b=${b#b}
  MJL_DP_BUCKETS=$b PROBE_DP=nccl PROBE_MB=8192 timeout -k 10 240 python tools/ppo_phase_probe.py > $O/probe_$run.json 2> $O/probe_$run.err \
    || { echo "probe $run failed"; grep -v "^frame" $O/probe_$run.err | tail -5; exit 1; }
  echo "$run $(tail -1 $O/probe_$run.json)"
done

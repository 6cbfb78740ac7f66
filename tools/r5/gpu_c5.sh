#!/bin/bash
# round 5: the data-parallel twin update with the bucketed all-reduce (MJL_DP_BUCKETS): DP graph == eager bit
# for bit, the 8-rank C5 rehearsal, the twin tests; then one C5 rank's update phase through a one-rank RCCL
# group (tools/ppo_phase_probe.py, PROBE_DP=nccl, PROBE_MB=8192), buckets on and off, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ppo_graph.py tests/test_dp_gpu.py tests/test_twin.py -m gpu -x -v \
  --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2
if [ $rc -ne 0 ]; then grep -B5 -A40 "^____" $O/pytest.log | head -80; exit $rc; fi
for rep in 1 2; do
  for b in 1 0; do
    MJL_DP_BUCKETS=$b PROBE_DP=nccl PROBE_MB=8192 timeout -k 10 300 python tools/ppo_phase_probe.py > $O/probe_b${b}_$rep.json 2> $O/probe_b${b}_$rep.err \
      || { echo "probe b=$b failed"; tail -5 $O/probe_b${b}_$rep.err; exit 1; }
    echo "buckets=$b rep=$rep $(tail -1 $O/probe_b${b}_$rep.json)"
  done
done

#!/bin/bash
# round 5: captured-collective DP step (default over RCCL) and the bucketed path: graph == eager bit for bit
# (gloo and one-rank RCCL), the 8-rank C5 rehearsal; then the phase probe with the defaults (one-rank RCCL:
# captured, one bucket) and with buckets forced on.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ppo_graph.py tests/test_dp_gpu.py -m gpu -x -v \
  --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2
if [ $rc -ne 0 ]; then grep -B5 -A40 "^____" $O/pytest.log | head -80; exit $rc; fi
for b in auto 1; do
  MJL_DP_BUCKETS=$b PROBE_DP=nccl PROBE_MB=8192 timeout -k 10 240 python tools/ppo_phase_probe.py > $O/probe_b$b.json 2> $O/probe_b$b.err \
    || { echo "probe failed"; tail -5 $O/probe_b$b.err; exit 1; }
  echo "buckets=$b $(tail -1 $O/probe_b$b.json)"
done

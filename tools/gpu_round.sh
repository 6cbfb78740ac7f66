#!/bin/bash
# One GPU-box pass: the -m gpu suite (per-test time limit), smoke, then the round's measurement
# record (tools/profile_round.sh: bench JSON, rocprofv3 stats, FETCH/WRITE PMC passes).
# Every GPU step has its own time limit; steps chained with && so a failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
bash tools/profile_round.sh
rc=$?
echo "gpu_round rc=$rc"
exit $rc

#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprof kernel-trace of the bench command.
# Every GPU step has its own time limit; steps are chained with && so a failure stops the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
    python bench.py --steps 20 --no-extras --no-cpu > gpurun_out/prof.log 2>&1
rc=$?
echo "final rc=$rc"
exit $rc

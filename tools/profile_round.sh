#!/bin/bash
# One GPU-box pass producing the round's measurement record (copied to profiles/ by
# tools/summarize_profiles.py): the bench JSON line, the rocprofv3 --kernel-trace --stats summary of
# the same bench command, and the two HBM-traffic PMC passes (FETCH_SIZE and WRITE_SIZE cannot share
# a pass on gfx950). Every GPU step has its own time limit; steps are chained with &&.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B="python bench.py --no-extras --no-cpu --steps 50"
timeout -k 10 400 python bench.py > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o trace -- \
    $B > gpurun_out/prof/trace.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o fetch -- \
    $B > gpurun_out/prof/fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o write -- \
    $B > gpurun_out/prof/write.log 2>&1
rc=$?
echo "profile rc=$rc"
exit $rc

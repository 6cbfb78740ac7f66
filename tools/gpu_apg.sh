#!/bin/bash
# APG on the GPU box: gradient parity test (GPU tape + VJP vs oracle finite differences), then the
# C4 throughput bench (2048 envs x 128 horizon, CG 4/4) and the same with the model's Newton solver.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_apg.py tests/test_adjoint.py -m gpu -q -x > gpurun_out/apg_test.log 2>&1 &&
timeout -k 10 400 python tools/bench_apg.py > gpurun_out/apg_bench.log 2>&1 &&
timeout -k 10 400 python tools/bench_apg.py --solver model > gpurun_out/apg_bench_newton.log 2>&1
rc=$?
echo "final rc=$rc"
exit $rc

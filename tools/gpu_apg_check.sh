# APG path check: the APG / tape / adjoint GPU tests, the record + replay kernel times and C4 (implicit)
export TMPDIR=/tmp
O=gpurun_out/${1:-apgcheck}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_apg.py tests/test_vjp_tape.py tests/test_adjoint.py > $O/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vjp -o t -- python tools/prof_target.py vjp 2048 256 > $O/vjp.log 2>&1 &&
timeout -k 10 300 python tools/bench_apg.py --vjp implicit > $O/apg.log 2>&1 &&
timeout -k 10 300 python tools/bench_apg.py --vjp unrolled > $O/apg_unrolled.log 2>&1
rc=$?; find $O -name '*_kernel_trace.csv' -delete; exit $rc

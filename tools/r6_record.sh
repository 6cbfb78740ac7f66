# Round 6: the LDS-row APG record -- its parity tests, then kernel times of the record / replay and C4
export TMPDIR=/tmp
O=gpurun_out/${1:-r6u}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_adjoint.py tests/test_apg.py > $O/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vjp -o t -- python tools/prof_target.py vjp 2048 256 > $O/vjp.log 2>&1 &&
timeout -k 10 300 python tools/bench_apg.py --vjp implicit > $O/apg.log 2>&1
rc=$?; find $O -name '*_kernel_trace.csv' -delete; exit $rc

# round 3: unbranched env-step / VJP-record state loads — full GPU suite, then the default bench line
mkdir -p gpurun_out/r3h
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3h/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r3h/bench.json 2> gpurun_out/r3h/bench.err || exit $?
cat gpurun_out/r3h/bench.json

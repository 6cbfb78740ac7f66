# round 3: replay-VJP prologue with batched slot loads — the adjoint / APG tests, then the APG legs of the bench
mkdir -p gpurun_out/r3g
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_apg.py tests/test_adjoint.py tests/test_gpu_configs.py -m gpu > gpurun_out/r3g/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --no-extras --no-ppo --no-cpu --steps 20 --warmup 5 > gpurun_out/r3g/bench_apg.json 2> gpurun_out/r3g/bench_apg.err || exit $?
exit $rc

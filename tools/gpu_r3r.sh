# lean replay VJP incl. unrolled CG: tests, stamps (both modes), kernel times lean vs full, APG legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_adjoint.py tests/test_apg.py tests/test_gpu_configs.py -m gpu > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --no-extras --no-ppo --no-cpu --steps 20 --warmup 5 > $O/bench_apg.json 2> $O/bench_apg.err || exit $?
grep -v amdgpu.ids $O/replay_times.txt | head -15

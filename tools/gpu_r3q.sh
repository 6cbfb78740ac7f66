# lean replay VJP incl. unrolled CG: tests, stamps (both modes), kernel times lean vs full, APG legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_adjoint.py tests/test_apg.py tests/test_gpu_configs.py -m gpu > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so REPLAY=1 timeout -k 10 200 python tools/vjp_times.py > $O/replay_times.txt 2>&1 || exit $?
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so REPLAY=1 VJP=unrolled timeout -k 10 200 python tools/vjp_times.py > $O/replay_times_unrolled.txt 2>&1 || exit $?
for L in 1 0; do
  MJL_VJP_LEAN=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vjp$L -o t -- python tools/prof_target.py vjp 2048 128 > $O/vjp$L.log 2>&1 || exit $?
  find $O/vjp$L -name '*_kernel_trace.csv' -delete
done
timeout -k 10 400 python -u bench.py --no-extras --no-ppo --no-cpu --steps 20 --warmup 5 > $O/bench_apg.json 2> $O/bench_apg.err || exit $?
grep -v amdgpu.ids $O/replay_times.txt | head -15

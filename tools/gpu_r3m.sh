# round 3: reverse passes with their model records prefetched — adjoint / tape / APG tests, replay-VJP
# phase stamps, replay kernel time at 2048 envs, APG bench legs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3m
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_adjoint.py tests/test_apg.py tests/test_gpu_configs.py -m gpu > gpurun_out/r3m/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so REPLAY=1 timeout -k 10 200 python tools/vjp_times.py > gpurun_out/r3m/replay_times.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m/vjp -o t -- python tools/prof_target.py vjp 2048 128 > gpurun_out/r3m/vjp.log 2>&1 || exit $?
find gpurun_out/r3m/vjp -name '*_kernel_trace.csv' -delete
timeout -k 10 400 python -u bench.py --no-extras --no-ppo --no-cpu --steps 20 --warmup 5 > gpurun_out/r3m/bench_apg.json 2> gpurun_out/r3m/bench_apg.err || exit $?
grep -v amdgpu.ids gpurun_out/r3m/replay_times.txt

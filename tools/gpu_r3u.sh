# APG replay: RNE reverse in registers (recompute by lane shuffle, tree reverse one barrier per level)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_adjoint.py tests/test_apg.py tests/test_gpu_configs.py -m gpu > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so REPLAY=1 timeout -k 10 200 python tools/vjp_times.py > $O/replay_times.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-extras --no-ppo --no-cpu --steps 20 --warmup 5 > $O/bench_apg.json 2> $O/bench_apg.err || exit $?
grep -v amdgpu.ids $O/replay_times.txt | head -22

# replay-VJP iteration: adjoint / tape tests, then phase stamps and the replay kernel time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3n}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_adjoint.py -m gpu > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so REPLAY=1 timeout -k 10 200 python tools/vjp_times.py > $O/replay_times.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vjp -o t -- python tools/prof_target.py vjp 2048 128 > $O/vjp.log 2>&1 || exit $?
find $O/vjp -name '*_kernel_trace.csv' -delete
grep -v amdgpu.ids $O/replay_times.txt
grep vjp_kernel $O/vjp/t_kernel_stats.csv | cut -d, -f1-8

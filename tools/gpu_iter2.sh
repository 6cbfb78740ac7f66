set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_ppo.py > gpurun_out/bench_ppo.log 2>&1 &&
timeout -k 10 300 python mujoco-mjx-lab_amd/train_ppo.py --test --results-dir gpurun_out/results > gpurun_out/train_test.log 2>&1

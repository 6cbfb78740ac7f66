set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rpool
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_reset_pool.py tests/test_ppo.py tests/test_gpu_parity.py -m gpu > gpurun_out/rpool/pytest.log 2>&1 && \
timeout -k 10 300 python tools/reset_pool_probe.py --envs 2048 > gpurun_out/rpool/probe_2048.jsonl 2>/dev/null && \
timeout -k 10 300 python tools/reset_pool_probe.py --envs 1024 > gpurun_out/rpool/probe_1024.jsonl 2>/dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rpool/trace -o rp -- python tools/reset_pool_probe.py --envs 2048 --reps 2 --only 11 > gpurun_out/rpool/trace.log 2>&1

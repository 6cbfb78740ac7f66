set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pol
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ppo.py -m gpu > gpurun_out/pol/pytest.log 2>&1 && \
timeout -k 10 300 python tools/reset_pool_probe.py --envs 2048 --only 11 > gpurun_out/pol/probe.jsonl 2>/dev/null && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pol/trace -o trace -- python tools/reset_pool_probe.py --envs 2048 --reps 2 --only 11 > gpurun_out/pol/trace.log 2>&1

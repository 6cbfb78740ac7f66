set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ploss
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ppo.py tests/test_gpu_configs.py tests/test_bench.py -m gpu > gpurun_out/ploss/pytest.log 2>&1 && \
timeout -k 10 300 python tools/ppo_update_probe.py enqueue > gpurun_out/ploss/enqueue.txt 2>&1 && \
for r in 1 2; do timeout -k 10 200 python tools/bench_ppo.py --envs 2048 --iters 6 > gpurun_out/ploss/ppo2048_$r.json 2>/dev/null && \
timeout -k 10 200 python tools/bench_ppo.py --envs 1024 --iters 6 > gpurun_out/ploss/ppo1024_$r.json 2>/dev/null || exit 1; done

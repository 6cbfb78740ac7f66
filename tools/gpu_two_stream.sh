set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/two
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ppo.py tests/test_gpu_configs.py -m gpu > gpurun_out/two/pytest.log 2>&1 && \
timeout -k 10 300 python tools/ppo_update_probe.py two > gpurun_out/two/probe.txt 2>&1 && \
for r in 1 2 3; do for s in 1 0; do MJL_TWO_STREAM=$s timeout -k 10 200 python tools/bench_ppo.py --envs 1024 --iters 12 > gpurun_out/two/ppo1024_s${s}_$r.json 2>/dev/null && \
MJL_TWO_STREAM=$s timeout -k 10 200 python tools/bench_ppo.py --envs 2048 --iters 12 > gpurun_out/two/ppo2048_s${s}_$r.json 2>/dev/null || exit 1; done; done

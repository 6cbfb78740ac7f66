set -o pipefail
mkdir -p gpurun_out/prof_ppo
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_ppo.py tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/prof_ppo/test.log 2>&1 &&
timeout -k 10 300 python tools/bench_ppo.py --envs 2048 --iters 3 > gpurun_out/prof_ppo/bench.json 2>&1 &&
timeout -k 10 300 python tools/bench_ppo.py --envs 1024 --iters 3 > gpurun_out/prof_ppo/bench1024.json 2>&1

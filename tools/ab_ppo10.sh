set -o pipefail
mkdir -p gpurun_out/ab10
for r in 1 2; do
  timeout -k 10 200 python _ab_head/tools/bench_ppo.py --envs 2048 --iters 10 > gpurun_out/ab10/head_$r.json 2>/dev/null && \
  timeout -k 10 200 python tools/bench_ppo.py --envs 2048 --iters 10 > gpurun_out/ab10/pool_$r.json 2>/dev/null || exit 1
done

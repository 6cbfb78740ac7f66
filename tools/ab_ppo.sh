# interleaved PPO A/B: the HEAD worktree (_ab_head) vs this tree without / with pooled resets
set -o pipefail
N=${ENVS:-2048}
mkdir -p gpurun_out/abppo_$N

for r in 1 2; do
  timeout -k 10 200 python _ab_head/tools/bench_ppo.py --envs $N --iters 4 > gpurun_out/abppo_$N/head_$r.json 2>/dev/null && \
  timeout -k 10 200 python tools/bench_ppo.py --envs $N --iters 4 --reset-pool 0 > gpurun_out/abppo_$N/nopf_$r.json 2>/dev/null && \
  timeout -k 10 200 python tools/bench_ppo.py --envs $N --iters 4 > gpurun_out/abppo_$N/pf_$r.json 2>/dev/null || exit 1
done

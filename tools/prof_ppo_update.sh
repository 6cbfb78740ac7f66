# rocprofv3 kernel stats of PPO iterations at 2048 envs (rollout + update), for the update breakdown
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/profppo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profppo -o ppo -- python tools/bench_ppo.py --envs 2048 --iters 3 > gpurun_out/profppo/run.log 2>&1

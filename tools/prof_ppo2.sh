set -o pipefail
mkdir -p gpurun_out/prof_ppo
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ppo/trace -o trace -- \
    python tools/bench_ppo.py --envs 2048 --iters 2 > gpurun_out/prof_ppo/trace.log 2>&1

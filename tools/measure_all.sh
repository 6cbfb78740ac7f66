#!/bin/bash
# One GPU-box pass for the round's full measurement record: the kernel profile (tools/profile_round.sh:
# bench JSON, rocprofv3 --kernel-trace --stats, FETCH_SIZE / WRITE_SIZE passes), then the PPO (C3)
# and APG (C4) throughput benches. Every GPU step has its own limit; steps chained with &&.
set -o pipefail
mkdir -p gpurun_out/prof_ppo gpurun_out/prof_apg
export TMPDIR=/tmp
bash tools/profile_round.sh &&
timeout -k 10 300 python tools/bench_ppo.py --envs 2048 --iters 3 > gpurun_out/prof_ppo/bench.json 2>&1 &&
timeout -k 10 300 python tools/bench_ppo.py --envs 1024 --iters 3 > gpurun_out/prof_ppo/bench1024.json 2>&1 &&
timeout -k 10 400 python tools/bench_apg.py > gpurun_out/prof_apg/apg_bench.log 2>&1 &&
timeout -k 10 400 python tools/bench_apg.py --solver model > gpurun_out/prof_apg/apg_bench_newton.log 2>&1
rc=$?
echo "measure rc=$rc"
exit $rc

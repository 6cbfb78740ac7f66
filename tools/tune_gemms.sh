#!/bin/bash
# Regenerate mjx_amd/tuning/gfx950_tunableop.csv: PyTorch TunableOp tunes every GEMM shape the
# workloads run (default bench legs: C3 PPO, return curve, C4 APG; the update at 2048 envs; the C5
# per-rank 8,192-row shard), each process reading and extending the same results file. Run on the
# GPU box; then copy gpurun_out/tune/tunableop_results0.csv into mujoco-mjx-lab_amd/mjx_amd/tuning/.
mkdir -p gpurun_out/tune
rm -f gpurun_out/tune/tunableop_results0.csv
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_results%d.csv
timeout -k 10 500 python -u bench.py --no-cpu > gpurun_out/tune/bench.json 2> gpurun_out/tune/bench.err || exit $?
timeout -k 10 300 python -u tools/ppo_update_probe.py graph 2048 > gpurun_out/tune/upd.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ppo_update_probe.py shard > gpurun_out/tune/shard.txt 2>&1 || exit $?
wc -l gpurun_out/tune/tunableop_results0.csv

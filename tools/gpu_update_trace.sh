set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/utrace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/utrace -o ut -- python tools/ppo_update_probe.py enqueue > gpurun_out/utrace/run.log 2>&1

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 240 python tools/cg_blowup.py > gpurun_out/cg_blowup.log 2>&1

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_variants.sh > gpurun_out/ab.log 2>&1 && 
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so timeout -k 10 120 python tools/phase_times.py > gpurun_out/phase.log 2>&1

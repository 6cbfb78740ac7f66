set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
# optional: parity of one extra variant (PARITY_VARIANT=name)
if [ -n "$PARITY_VARIANT" ]; then
  MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_$PARITY_VARIANT.so timeout -k 10 500 \
    python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu_variant.log 2>&1; rc=$?
  echo "variant pytest rc=$rc" >> gpurun_out/pytest_gpu_variant.log
  case $rc in 124|137|134|139) exit $rc;; esac
fi
bash tools/ab_variants.sh > gpurun_out/ab.log 2>&1 &&
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so timeout -k 10 120 python tools/phase_times.py > gpurun_out/phase.log 2>&1

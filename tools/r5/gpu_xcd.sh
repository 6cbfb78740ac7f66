#!/bin/bash
# round 5: XCD-aware env order (block_env) against env = blockIdx.x (the MJL_BLOCK_ORDER build): GPU parity
# of the physics, env step, reset pool and replay VJP on the new order, then per kernel family and order a
# rocprofv3 kernel trace and the FETCH_SIZE / WRITE_SIZE passes (2048 envs), the two orders interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_reset_pool.py tests/test_vjp_tape.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "^____" $O/pytest.log | head -60; exit $rc; }
LIBB=mujoco-mjx-lab_amd/mjx_amd/libmjx355_blockorder.so
prof() {  # tag, lib ('' = product), prof_target args...
  local tag=$1 lib=$2; shift 2
  local env=""; [ -n "$lib" ] && export MJX355_LIB=$PWD/$lib || unset MJX355_LIB
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag/trace -o trace -- \
    python tools/prof_target.py "$@" > $O/$tag.trace.log 2>&1 || { echo "$tag trace failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$tag/fetch -o fetch -- \
    python tools/prof_target.py "$@" > $O/$tag.fetch.log 2>&1 || { echo "$tag fetch failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/$tag/write -o write -- \
    python tools/prof_target.py "$@" > $O/$tag.write.log 2>&1 || { echo "$tag write failed"; exit 1; }
  find $O/$tag -name '*_kernel_trace.csv' -delete
  echo "$tag ok"
}
for MODE in envstep envstep_pool speedtest vjp; do
  N=200; [ $MODE = vjp ] && N=256
  prof ${MODE}_xcd "" $MODE 2048 $N
  prof ${MODE}_block $LIBB $MODE 2048 $N
done
unset MJX355_LIB
python tools/r5/traffic_summary.py $O

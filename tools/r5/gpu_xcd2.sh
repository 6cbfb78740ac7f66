#!/bin/bash
# round 5: env order A/B, three builds -- chunked XCD order (the product: runs of 16 envs per XCD),
# env = blockIdx.x (MJL_BLOCK_ORDER), one contiguous eighth per XCD (MJL_XCD_CONTIG) -- GPU parity on the
# product build, then per kernel family two interleaved rounds of kernel traces, and the FETCH_SIZE /
# WRITE_SIZE passes on the product build (2048 envs).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_reset_pool.py tests/test_vjp_tape.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "^____" $O/pytest.log | head -60; exit $rc; }
L=mujoco-mjx-lab_amd/mjx_amd
run() {  # tag, lib ('' = product), pass (trace / fetch / write), prof_target args...
  local tag=$1 lib=$2 pass=$3; shift 3
  if [ -n "$lib" ]; then export MJX355_LIB=$PWD/$L/$lib; else unset MJX355_LIB; fi
  local opt="--stats"; [ $pass = fetch ] && opt="--pmc FETCH_SIZE"; [ $pass = write ] && opt="--pmc WRITE_SIZE"
  timeout -k 10 300 rocprofv3 --kernel-trace $opt --output-format csv -d $O/$tag/$pass -o $pass -- \
    python tools/prof_target.py "$@" > $O/$tag.$pass.log 2>&1 || { echo "$tag $pass failed"; exit 1; }
  find $O/$tag -name '*_kernel_trace.csv' -delete
}
for MODE in speedtest envstep_pool envstep vjp; do
  N=200; [ $MODE = vjp ] && N=256
  for R in 1 2; do
    run ${MODE}_chunk_$R "" trace $MODE 2048 $N
    run ${MODE}_block_$R libmjx355_blockorder.so trace $MODE 2048 $N
    run ${MODE}_contig_$R libmjx355_xcdcontig.so trace $MODE 2048 $N
  done
  run ${MODE}_chunk_1 "" fetch $MODE 2048 $N
  run ${MODE}_chunk_1 "" write $MODE 2048 $N
  echo "$MODE ok"
done
unset MJX355_LIB
python tools/r5/traffic_summary.py $O > /dev/null && echo summary ok

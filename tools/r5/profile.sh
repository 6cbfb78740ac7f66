#!/bin/bash
# Round-5 measurement record (as tools/profile_r3.sh): rocprofv3 --kernel-trace --stats of the default bench command, then per
# kernel family (speed test, env step with / without the reset pool, APG replay VJP) a kernel trace and
# the HBM (FETCH_SIZE, WRITE_SIZE) and SQ counter passes, each pass its own run. Exit on any fault /
# timeout (status other than 0).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${PROF_OUT:-prof5}
mkdir -p $O
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}
step bench_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_trace -o trace -- \
     python bench.py --gpus 1 --steps 20 --warmup 5
find $O/bench_trace -name '*_kernel_trace.csv' -delete  # keep the stats (the trace is ~10^5 rows)
for MODE in speedtest envstep envstep_pool envstep_nr vjp; do
  N=200; [ $MODE = vjp ] && N=256
  step ${MODE}_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$MODE/trace -o trace -- \
       python tools/prof_target.py $MODE 2048 $N
  step ${MODE}_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$MODE/fetch -o fetch -- \
       python tools/prof_target.py $MODE 2048 $N
  step ${MODE}_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/$MODE/write -o write -- \
       python tools/prof_target.py $MODE 2048 $N
  step ${MODE}_sq1 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
       --output-format csv -d $O/$MODE/sq1 -o sq1 -- python tools/prof_target.py $MODE 2048 $N
  step ${MODE}_sq2 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH \
       --output-format csv -d $O/$MODE/sq2 -o sq2 -- python tools/prof_target.py $MODE 2048 $N
done
echo ALL_OK >> $O/status.txt

#!/bin/bash
# The round's GPU calls in one parameterised script (replaces the per-call tools/r5/gpu_*.sh):
#   tools/gpu_round.sh <out-name> <step> [<step> ...]
# Steps (each under its own time limit; the first failure ends the call, nothing after it runs):
#   suite        the GPU test suite (pytest -m gpu)                  -> <out>/pytest.log
#   smoke        __graft_entry__.smoke()                              -> <out>/smoke.log
#   bench        the driver's default bench command                  -> <out>/bench.json
#   trace        rocprofv3 --kernel-trace --stats of the bench       -> <out>/bench_trace/
#   c5           one rank's C5 update (tools/c5_update_probe.py)      -> <out>/c5.log
#   c5trace      rocprofv3 kernel trace of the C5 update probe        -> <out>/c5_trace/
#   prof:<mode>  kernel trace + FETCH/WRITE + 2 SQ passes of tools/prof_target.py <mode> (2048 envs)
#   py:<script>  python tools/<script> (extra args after '='; ',' for spaces) -> <out>/<script>.log
#   exe:<binary> tools/<binary> built here (args after '='; ',' for spaces)  -> <out>/<binary>.log
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "[$(date +%T)] $name" >> $O/status.txt
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt
  if [ $rc -ne 0 ]; then
    echo "$name failed rc=$rc"
    tail -30 $O/$name.log
    exit $rc
  fi
}
for S in "$@"; do
  case $S in
    suite) step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 && tail -1 $O/bench.log > $O/bench.json ;;
    trace) step bench_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_trace -o trace -- \
             python bench.py --gpus 1 --steps 20 --warmup 5
           find $O/bench_trace -name '*_kernel_trace.csv' -delete ;;
    c5) step c5 400 python tools/c5_update_probe.py 3 ;;
    c5trace) step c5_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_trace -o trace -- \
               python tools/c5_update_probe.py 1 ;;
    prof:*)
      M=${S#prof:}
      N=200; [ $M = vjp ] && N=256
      step ${M}_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$M/trace -o trace -- \
           python tools/prof_target.py $M 2048 $N
      step ${M}_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$M/fetch -o fetch -- \
           python tools/prof_target.py $M 2048 $N
      step ${M}_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/$M/write -o write -- \
           python tools/prof_target.py $M 2048 $N
      step ${M}_sq1 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU \
           SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/$M/sq1 -o sq1 -- \
           python tools/prof_target.py $M 2048 $N
      step ${M}_sq2 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
           SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --output-format csv -d $O/$M/sq2 -o sq2 -- \
           python tools/prof_target.py $M 2048 $N
      find $O/$M -name '*_kernel_trace.csv' -size +8M -delete ;;
    py:*)
      A=${S#py:}
      SCRIPT=${A%%=*}
      ARGS=""; [ "$A" != "$SCRIPT" ] && ARGS=${A#*=}
      step $(basename $SCRIPT .py) 600 python tools/$SCRIPT ${ARGS//,/ } ;;
    exe:*)
      A=${S#exe:}
      B=${A%%=*}
      ARGS=""; [ "$A" != "$B" ] && ARGS=${A#*=}
      step $B 300 ./tools/$B ${ARGS//,/ } ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo ALL_OK >> $O/status.txt

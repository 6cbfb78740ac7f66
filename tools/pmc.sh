#!/bin/bash
# Counter passes for the step kernel (one rocprofv3 run per pass, --pmc only with --kernel-trace).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
MODE=${1:-speedtest}
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS " \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  P=${P//\?/}
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/pmc/p$i -o p$i -- \
      python tools/prof_target.py $MODE 2048 10 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> gpurun_out/pmc/status.txt
  case $rc in 124|137|134|139) exit $rc;; esac
done

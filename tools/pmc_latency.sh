#!/bin/bash
# Latency counter passes for the speed-test kernel at B = 1 (one lone wave) and B = 2048:
# SQ_INST_LEVEL_* / SQ_INSTS_* = mean in-flight cycles per LDS / vector-memory / scalar-memory
# instruction. One rocprofv3 run per pass, --pmc only with --kernel-trace.
set -o pipefail
mkdir -p gpurun_out/pmcl
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmcl/counters_list.txt 2>&1 || true
i=0
for B in 1 2048; do
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/pmcl/p$i -o p$i -- \
      python tools/prof_target.py speedtest $B 10 > gpurun_out/pmcl/p$i.log 2>&1
  rc=$?
  echo "B $B pass $i rc=$rc" >> gpurun_out/pmcl/status.txt
  case $rc in 124|137|134|139) exit $rc;; esac
done
done

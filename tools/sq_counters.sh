#!/bin/bash
# Two SQ PMC passes over the speed-test kernel (instruction mix, wave / busy / wait cycles): is the
# kernel issue-bound (VALU instructions x 4 cycles ~ wave cycles) or latency-bound?
set -o pipefail
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
B="python bench.py --no-extras --cpu-seconds 1 --steps 20 --warmup 3"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/sq/p1 -o p1 -- $B > gpurun_out/sq/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD \
    --output-format csv -d gpurun_out/sq/p2 -o p2 -- $B > gpurun_out/sq/p2.log 2>&1
rc=$?
echo "sq rc=$rc"
exit $rc

# counter passes on the dense-layer micro-benchmark's forward 128x128x32 variant (variant 0)
mkdir -p gpurun_out/mlppmc
export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/mlppmc/p$i -o p$i -- ./tools/mlp_micro 0 > gpurun_out/mlppmc/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
find gpurun_out/mlppmc -name '*_kernel_trace.csv' -delete

# Round 6: two envs per wave at the step kernel's LDS residency, and its SQ counters
export TMPDIR=/tmp
O=gpurun_out/r6x; mkdir -p $O
timeout -k 10 200 ./tools/twoenv_micro 50 > $O/twoenv.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o sq -- ./tools/twoenv_micro 50 > $O/sq.log 2>&1

# replay-VJP counters at 640 vs 2048 envs: instruction-cache misses and the SQ wait split
export TMPDIR=/tmp
O=gpurun_out/vjppmc
mkdir -p $O
for B in 640 2048; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $O/ic$B -o ic -- python tools/prof_target.py vjp $B 128 > $O/ic$B.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $O/sq$B -o sq -- python tools/prof_target.py vjp $B 128 > $O/sq$B.log 2>&1 || exit $?
done
ls $O/*/

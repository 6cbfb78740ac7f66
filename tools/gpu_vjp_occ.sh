# replay-VJP launch time against batch size (5 blocks/CU by LDS: 1280 envs = one full round)
export TMPDIR=/tmp
mkdir -p gpurun_out/vjpocc
for B in 640 1280 2048 2560; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vjpocc/b$B -o t -- python tools/prof_target.py vjp $B 128 > gpurun_out/vjpocc/b$B.log 2>&1 || exit $?
  find gpurun_out/vjpocc/b$B -name '*_kernel_trace.csv' -delete
done

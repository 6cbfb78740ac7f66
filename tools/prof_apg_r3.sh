# kernel breakdown of APG C4 updates (2048 x 128, CG 4/4), implicit and unrolled
export TMPDIR=/tmp
O=gpurun_out/prof_apg_r3
mkdir -p $O
for V in implicit unrolled; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$V -o t -- \
      python tools/bench_apg.py --updates 4 --solver cg --vjp $V > $O/$V.log 2>&1 || exit $?
  find $O/$V -name '*_kernel_trace.csv' -delete
done

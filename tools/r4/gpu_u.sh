# round 4: the head's bias + tanh folded into the twin loss launch or not (same process, interleaved),
# plus a kernel trace of each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 400 python -u tools/ppo_update_probe.py fold > $O/ab.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/ab.txt
for f in 1 0; do
  MJL_TWIN_FOLD_HEAD=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof$f -o run -- python -u tools/ppo_update_probe.py c5twin > $O/prof$f.txt 2>&1 || exit $?
  t=$(find $O/prof$f -name '*kernel_trace.csv' | head -1)
  python tools/trace_by_grid.py "$t" 8 > $O/by_grid$f.txt && rm -rf $O/prof$f
  echo "fold=$f"; cat $O/by_grid$f.txt
done

# round 4: twin update timing repeatability (two runs of the probe on one box)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
for k in 1 2; do
  timeout -k 10 300 python -u tools/ppo_update_probe.py twinonly > $O/ab$k.txt 2>&1 || exit $?
  grep -v amdgpu.ids $O/ab$k.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python -u tools/ppo_update_probe.py c5twin > $O/prof.txt 2>&1 || exit $?
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/trace_by_grid.py "$f" 20 > $O/by_grid.txt && cat $O/by_grid.txt && rm -rf $O/prof

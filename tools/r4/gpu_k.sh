# round 4: twin column-sum partial chunk A/B, unrolled surrogate staging; twin tests; kernel trace of the C5-shape twin update
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
true
rc=0
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest.log | grep -B5 -A40 "^____" | head -80; exit $rc; fi
true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u tools/ppo_update_probe.py c5twin > $O/prof.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/prof.txt | tail -5
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/trace_by_grid.py "$f" 60 > $O/by_grid.txt && cat $O/by_grid.txt && rm -rf $O/prof

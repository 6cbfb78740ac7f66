# round 4: the loss-head kernel with two threads per row (element-parallel staging + tanh): tests,
# twin timing, kernel trace, then the measurement record on these sources (profile.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_twin.py tests/test_ppo_graph.py tests/test_dp_gpu.py tests/test_ppo.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest.log | grep -B5 -A40 "^____" | head -100; exit $rc; fi
timeout -k 10 300 python -u tools/ppo_update_probe.py twinonly > $O/ab.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python -u tools/ppo_update_probe.py c5twin > $O/prof.txt 2>&1 || exit $?
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/trace_by_grid.py "$f" 8 > $O/by_grid.txt && cat $O/by_grid.txt && rm -rf $O/prof
bash tools/r4/profile.sh || exit $?
echo PROFILE_OK

# round 4: twin graphs with the next minibatch prefetched on a side stream (two buffer sets, one graph
# per parity): graph / twin / DP tests, interleaved A/B, kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4w
mkdir -p $O
MJL_TWIN_PREFETCH=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ppo_graph.py tests/test_twin.py tests/test_dp_gpu.py tests/test_ppo.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest.log | grep -B5 -A40 "^____" | head -100; exit $rc; fi
timeout -k 10 400 python -u tools/ppo_update_probe.py prefetch > $O/ab.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/ab.txt

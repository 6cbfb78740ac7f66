# round 4: surrogate rows per block (MJL_SURR_ROWS 256 / 128 / 64) with the counters advanced by the loss
# launch and 32-row head-backward chunks: twin tests, update time per setting, kernel trace per setting
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_twin.py tests/test_ppo_graph.py tests/test_ppo.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest.log | grep -B5 -A40 "^____" | head -100; exit $rc; fi
for rb in 256 128 64; do
  MJL_SURR_ROWS=$rb timeout -k 10 300 python -u tools/ppo_update_probe.py twinonly > $O/t$rb.txt 2>&1 || exit $?
  echo "rows=$rb"; grep -v amdgpu.ids $O/t$rb.txt
done
for rb in 256 64; do
  MJL_SURR_ROWS=$rb timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof$rb -o run -- python -u tools/ppo_update_probe.py c5twin > $O/prof$rb.txt 2>&1 || exit $?
  f=$(find $O/prof$rb -name '*kernel_trace.csv' | head -1)
  python tools/trace_by_grid.py "$f" 24 > $O/by_grid$rb.txt && rm -rf $O/prof$rb
  echo "rows=$rb"; cat $O/by_grid$rb.txt
done

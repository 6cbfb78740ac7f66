# round 4, second GPU call: twin update (both nets as one batched pass per layer) + the C5 8-rank test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_twin.py tests/test_ppo_graph.py tests/test_dp_gpu.py tests/test_ppo.py > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest.log | grep -B5 -A40 "^____" | head -80; exit $rc; fi
for T in 1 0; do
  MJL_TWIN_UPDATE=$T timeout -k 10 300 python -u tools/ppo_phase_probe.py > $O/phase_c3_twin$T.json 2> $O/phase_c3_twin$T.err || exit $?
  MJL_TWIN_UPDATE=$T PROBE_DP=1 PROBE_MB=8192 timeout -k 10 300 python -u tools/ppo_phase_probe.py > $O/phase_c5_twin$T.json 2> $O/phase_c5_twin$T.err || exit $?
  cat $O/phase_c3_twin$T.json $O/phase_c5_twin$T.json
done
PROBE_DP=1 PROBE_MB=8192 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o t -- python tools/ppo_phase_probe.py > $O/prof_c5.log 2>&1 || exit $?
echo ALL_OK

# round 4: twin update with one Adam launch for both nets, the value gradient in the head kernel and
# device-row index / statistics tables (no per-minibatch host copies): tests, A/B, C5 phase split;
# then the APG / solver-timing / Hessian-variant probes (tools/r4/gpu_e.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_twin.py tests/test_ppo_graph.py tests/test_ppo.py tests/test_dp_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest.log | grep -B5 -A40 "^____" | head -80; exit $rc; fi
timeout -k 10 200 python -u tools/ppo_update_probe.py twin > $O/ab.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/ab.txt
for T in 1 0; do
  MJL_TWIN_UPDATE=$T PROBE_DP=nccl PROBE_MB=8192 timeout -k 10 300 python -u tools/ppo_phase_probe.py > $O/phase_c5_nccl_twin$T.json 2> $O/phase_c5_nccl_twin$T.err || exit $?
  grep '^{' $O/phase_c5_nccl_twin$T.json
done
PROBE_DP=nccl PROBE_MB=8192 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o t -- python tools/ppo_phase_probe.py > $O/prof_c5.log 2>&1 || exit $?
echo ALL_OK_F
bash tools/r4/gpu_e.sh

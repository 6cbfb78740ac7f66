# round 4: twin update after the Adam / column-sum fixes (tests, A/B, phase split) and the APG C4 curves
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_twin.py tests/test_ppo_graph.py tests/test_ppo.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest.log | grep -B5 -A40 "^____" | head -80; exit $rc; fi
timeout -k 10 200 python -u tools/ppo_update_probe.py twin > $O/ab.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/ab.txt
for T in 1 0; do
  MJL_TWIN_UPDATE=$T PROBE_DP=nccl PROBE_MB=8192 timeout -k 10 300 python -u tools/ppo_phase_probe.py > $O/phase_c5_nccl_twin$T.json 2> $O/phase_c5_nccl_twin$T.err || exit $?
  MJL_TWIN_UPDATE=$T timeout -k 10 300 python -u tools/ppo_phase_probe.py > $O/phase_c3_twin$T.json 2> $O/phase_c3_twin$T.err || exit $?
  grep -h '^{' $O/phase_c5_nccl_twin$T.json $O/phase_c3_twin$T.json
done
PROBE_DP=nccl PROBE_MB=8192 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o t -- python tools/ppo_phase_probe.py > $O/prof_c5.log 2>&1 || exit $?
echo ALL_OK_H
bash tools/r4/apg_curves.sh || exit $?
for f in gpurun_out/apgc4_r4/*.metrics.jsonl; do echo $f; python3 -c "
import json
for l in open('$f'):
    r=json.loads(l)
    if r['step'] % 50 == 0 or r['step'] in (99,100,110,120,299): print(r['step'], round(r['return'],1), r.get('reverse_nonfinite_envs'), r.get('forward_dropped_envs'))
"; done
echo ALL_OK_APG

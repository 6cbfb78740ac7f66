# round 4: twin backward with one deferred reduction launch: tests + A/B, then the round-end suite / smoke / bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_twin.py tests/test_ppo_graph.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest.log | grep -B5 -A40 "^____" | head -80; exit $rc; fi
timeout -k 10 200 python -u tools/ppo_update_probe.py twin > $O/ab.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/ab.txt
bash tools/r4/gpu_final_a.sh

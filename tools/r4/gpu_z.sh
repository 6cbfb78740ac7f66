# round 4 end: the full GPU suite and smoke() on the final tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest_gpu.log | grep -B5 -A40 "^____" | head -80; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json; d=json.load(open('$O/bench.json')); print({k: d.get(k) for k in ['value', 'ppo_c3_ms_per_iter', 'ppo_update_tflops', 'ppo_c5_rank_update_ms', 'apg_c4_env_steps_per_s', 'apg_c4_implicit_env_steps_per_s']})"

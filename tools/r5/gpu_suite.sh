#!/bin/bash
# round 5: the full GPU suite (incl. the R1 / R3 / R5 / R6 pins and the twin ADVICE tests), smoke(), and
# the default bench line. Every GPU step under its own limit; stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r5d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -s > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest_gpu.log | tail -2; grep "^R6:" $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest_gpu.log | grep -B5 -A40 "^____" | head -80; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json; d=json.load(open('$O/bench.json')); print({k: d.get(k) for k in ['value', 'env_step_kernel_ms', 'env_step_pool_kernel_ms', 'env_step_noreset_kernel_ms', 'speedtest_humanoid_xml_b4096_steps_per_s', 'speedtest_sphere_b4096_steps_per_s', 'ppo_c3_ms_per_iter', 'ppo_c5_rank_update_ms', 'apg_c4_env_steps_per_s', 'apg_c4_implicit_env_steps_per_s']})"

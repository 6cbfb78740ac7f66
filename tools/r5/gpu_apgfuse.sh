#!/bin/bash
# round 5: the APG sweep's fused per-step launches (observation + policy forward, policy input backward +
# observation backward) and the apg_post load chain: GPU tests of the APG path, then the bench's APG leg
# with the fused launches on / off / on (MJL_APG_FUSED_OBS), and a kernel trace of one APG leg.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5f3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_apg.py tests/test_vjp_tape.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A40 "^____" $O/pytest.log | head -80; exit $rc; }
for F in 1 0 1; do
  MJL_APG_FUSED_OBS=$F timeout -k 10 400 python bench.py --no-cpu --no-extras --no-ppo --apg-updates 5 \
    > $O/bench_fused$F.json 2> $O/bench_fused$F.err || { echo "bench F=$F failed"; tail -20 $O/bench_fused$F.err; exit 1; }
  python - $O/bench_fused$F.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("extras", d)
keys = ["apg_c4_env_steps_per_s", "apg_c4_ms_per_update", "apg_c4_implicit_env_steps_per_s", "apg_c4_implicit_ms_per_update"]
print(sys.argv[1], {k: ex.get(k) for k in keys}, {k: ex.get("apg_vjp_roofline", {}).get(k) for k in ("kernel_ms_every_env_active", "kernel_ms_trainer_workload")})
PY
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- \
  python bench.py --no-cpu --no-extras --no-ppo --apg-updates 5 > $O/bench_trace.log 2>&1 || { echo "trace failed"; exit 1; }
find $O/trace -name '*_kernel_trace.csv' -delete
echo ALL_OK

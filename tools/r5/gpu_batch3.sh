#!/bin/bash
# round 5: the APG sweep's fused launches on the per-layer small-MLP kernels (forward slots sized by the
# layer widths): GPU tests, the bench APG leg fused on / off / on, a kernel trace of one APG leg.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_apg.py tests/test_vjp_tape.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest_apg.log 2>&1 || fail pytest_apg $O/pytest_apg.log
tail -1 $O/pytest_apg.log
show() { python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ["apg_c4_env_steps_per_s", "apg_c4_implicit_env_steps_per_s", "apg_c4_ms_per_update", "apg_c4_implicit_ms_per_update"]
print(sys.argv[1], {k: d.get(k) for k in keys}, {k: d.get("apg_vjp_roofline", {}).get(k) for k in ("kernel_ms_every_env_active", "kernel_ms_trainer_workload")})
PY
}
for F in 1 0 1; do
  MJL_APG_FUSED_OBS=$F timeout -k 10 400 python bench.py --no-cpu --no-extras --no-ppo --apg-updates 5 \
    > $O/bench_apg_fused$F.json 2> $O/bench_apg_fused$F.err || fail bench_apg $O/bench_apg_fused$F.err
  show $O/bench_apg_fused$F.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/apg_trace -o trace -- \
  python bench.py --no-cpu --no-extras --no-ppo --apg-updates 5 > $O/apg_trace.log 2>&1 || fail apg_trace $O/apg_trace.log
find $O/apg_trace -name '*_kernel_trace.csv' -delete
python - $O/apg_trace <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:8]:
        print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us", r["Name"][:80])
PY
echo ALL_OK

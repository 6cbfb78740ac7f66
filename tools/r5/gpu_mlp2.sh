#!/bin/bash
# round 5: the small-MLP kernels with each layer's loads issued together: APG GPU tests, the kernels alone
# (kernel trace), the bench APG leg
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_apg.py tests/test_vjp_tape.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest_apg.log 2>&1 || fail pytest_apg $O/pytest_apg.log
tail -1 $O/pytest_apg.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python tools/prof_target.py apgmlp 2048 200 > $O/trace.log 2>&1 || fail trace $O/trace.log
find $O -name '*_kernel_trace.csv' -delete
python - $O <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "small_mlp" in r["Name"]:
            print("avg", round(float(r["AverageNs"]) / 1e3, 2), "us", r["Name"][:60])
PY
for i in 1 2; do
timeout -k 10 400 python bench.py --no-cpu --no-extras --no-ppo --apg-updates 5 > $O/bench_apg$i.json 2> $O/bench_apg$i.err || fail bench $O/bench_apg$i.err
python - $O/bench_apg$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d.get(k) for k in ["apg_c4_env_steps_per_s", "apg_c4_implicit_env_steps_per_s"]})
PY
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/apg_trace -o trace -- \
  python bench.py --no-cpu --no-extras --no-ppo --apg-updates 5 > $O/apg_trace.log 2>&1 || fail apg_trace $O/apg_trace.log
find $O/apg_trace -name '*_kernel_trace.csv' -delete
python - $O/apg_trace <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:7]:
        print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us", r["Name"][:80])
PY
echo ALL_OK

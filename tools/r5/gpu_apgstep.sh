#!/bin/bash
# round 5: the APG rollout physics through the env-step kernel (rows in LDS) against the record kernel
# (rows and tape in global memory), 2048 envs, CG 4/4 (tools/prof_target.py apgstep / vjp)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
for M in apgstep vjp; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$M -o t -- python tools/prof_target.py $M 2048 256 > $O/$M.log 2>&1 || { tail $O/$M.log; exit 1; }
  find $O/$M -name '*_kernel_trace.csv' -delete
  python - $O/$M $M <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:4]:
        print(sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us", r["Name"][:80])
PY
done

#!/bin/bash
# round 5 diagnostic: the APG record kernel with and without the implicit VJP's Hc factor (a temporary build with the
# record path's `solver_hessian` + `chol_factor_solve` block compiled out, not kept in the sources; its gradients are wrong, only the record's time is read), 2048 envs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5h2
mkdir -p $O
for R in 1 2; do for V in prod nohc; do
  if [ $V = prod ]; then unset MJX355_LIB; else export MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/libmjx355_nohc.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${V}_$R -o t -- python tools/prof_target.py vjp 2048 128 > $O/${V}_$R.log 2>&1 || { tail $O/${V}_$R.log; exit 1; }
  find $O/${V}_$R -name '*_kernel_trace.csv' -delete
  python - $O/${V}_$R $V <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "vjp_kernel" in r["Name"]:
            print(sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us", r["Name"][:80])
PY
done; done

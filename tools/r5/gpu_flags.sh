#!/bin/bash
# round 5: compiler scheduling variants of the product library (default -O2; -mllvm
# -amdgpu-sched-strategy=max-ilp / iterative-ilp; -O3), kernel times of the speed test and the pooled
# env step at 2048 envs, two interleaved rounds (rocprofv3 --stats).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5v
mkdir -p $O
L=mujoco-mjx-lab_amd/mjx_amd
for R in 1 2; do
  for V in default vmaxilp vitilp vo3; do
    if [ $V = default ]; then unset MJX355_LIB; else export MJX355_LIB=$PWD/$L/libmjx355_$V.so; fi
    for MODE in speedtest envstep_pool; do
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${MODE}_${V}_$R -o t -- \
        python tools/prof_target.py $MODE 2048 200 > $O/${MODE}_${V}_$R.log 2>&1 || { echo "$MODE $V failed"; tail -5 $O/${MODE}_${V}_$R.log; exit 1; }
      find $O/${MODE}_${V}_$R -name '*_kernel_trace.csv' -delete
      python - $O/${MODE}_${V}_$R $MODE $V $R <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Name"] and (", 2, 2>" in r["Name"] or ", 3, 2>" in r["Name"]):
            print(sys.argv[2], sys.argv[3], sys.argv[4], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
    done
  done
done
echo ALL_OK

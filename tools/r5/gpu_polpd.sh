#!/bin/bash
# round 5: the rollout policy kernel's weight prefetch depth (MJL_POL_PD chunks of 16 k in flight: 2 =
# the previous kernel, 4 = product, 6): parity test, kernel times at 1024 / 2048 envs, the C3 leg
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
L=$PWD/mujoco-mjx-lab_amd/mjx_amd
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_ppo.py tests/test_ppo_graph.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1 || fail pytest $O/pytest.log
tail -1 $O/pytest.log
for R in 1 2; do for B in 1024 2048; do for V in pd2 pd4 pd6; do
  if [ $V = pd4 ]; then unset MJX355_LIB; else export MJX355_LIB=$L/libmjx355_$V.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pol_${B}_${V}_$R -o t -- \
    python tools/prof_target.py policy $B 400 > $O/pol_${B}_${V}_$R.log 2>&1 || fail pol $O/pol_${B}_${V}_$R.log
  find $O/pol_${B}_${V}_$R -name '*_kernel_trace.csv' -delete
  python - $O/pol_${B}_${V}_$R $B $V <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "policy_rollout" in r["Name"]:
            print("policy B", sys.argv[2], sys.argv[3], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done; done; done
unset MJX355_LIB
for V in pd4 pd2 pd4; do
  if [ $V = pd4 ]; then unset MJX355_LIB; else export MJX355_LIB=$L/libmjx355_$V.so; fi
  timeout -k 10 400 python bench.py --workload ppo > $O/bench_ppo_$V.json 2> $O/bench_ppo_$V.err || fail bench $O/bench_ppo_$V.err
  python -c "import json,sys; d=json.loads(open('$O/bench_ppo_$V.json').read().strip().splitlines()[-1]); print('$V', d['value'], d['ms_per_step'], d.get('ppo_c3_phase_ms'))"
done
echo ALL_OK

#!/bin/bash
# round 5: the rollout policy kernel with each layer's first weight chunks and bias loaded during the
# previous layer: bit-for-bit against the previous build (libmjx355_polprev.so), parity test, kernel times
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5pp
mkdir -p $O
L=$PWD/mujoco-mjx-lab_amd/mjx_amd
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
timeout -k 10 120 python tools/r5/pol_bits.py $O/new.pt > $O/bits_new.log 2>&1 || fail bits_new $O/bits_new.log
MJX355_LIB=$L/libmjx355_polprev.so timeout -k 10 120 python tools/r5/pol_bits.py $O/prev.pt > $O/bits_prev.log 2>&1 || fail bits_prev $O/bits_prev.log
python -c "
import torch
a, b = torch.load('$O/new.pt', weights_only=True), torch.load('$O/prev.pt', weights_only=True)
for B in a: print('B', B, 'act equal', torch.equal(a[B][0], b[B][0]), 'logp equal', torch.equal(a[B][1], b[B][1]))"
timeout -k 10 300 python -u -m pytest tests/test_ppo.py tests/test_ppo_graph.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1 || fail pytest $O/pytest.log
tail -1 $O/pytest.log
for R in 1 2; do for B in 1024 2048; do for V in new prev; do
  if [ $V = new ]; then unset MJX355_LIB; else export MJX355_LIB=$L/libmjx355_polprev.so; fi
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
echo ALL_OK

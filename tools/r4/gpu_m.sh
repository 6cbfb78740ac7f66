# round 4: dense-kernel tile shapes (MJL_DENSE_CFG 0-4) against bmm + elementwise pass, per launch
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
for c in 0 1 2 3 4; do
  MJL_DENSE_CFG=$c timeout -k 10 120 python -u tools/dense_probe.py > $O/cfg$c.jsonl 2>$O/cfg$c.err || { tail -20 $O/cfg$c.err; exit 1; }
  cat $O/cfg$c.jsonl
done

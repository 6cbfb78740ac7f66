#!/bin/bash
# A/B the compiled variants in mujoco-mjx-lab_amd/mjx_amd/variants/ (one process each), ROUNDS
# interleaved passes (default 2) so that clock drift hits every variant alike.
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for f in mujoco-mjx-lab_amd/mjx_amd/variants/*.so; do
    n=$(basename $f .so)
    MJX355_LIB=$PWD/$f timeout -k 10 120 python bench.py --no-extras --no-cpu --steps 40 > gpurun_out/ab_$n.log 2>&1
    rc=$?
    case $rc in 124|137|134|139) echo "$f rc=$rc"; exit $rc;; esac
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['value']), round(d['roofline']['kernel_ms'],4))"
  done
done

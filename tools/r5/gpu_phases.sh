#!/bin/bash
# round 5: where the tree-ordered factor's cycles go: per-phase s_memtime stamps (MJL_TIMING build) with
# the tree kernels and with the dense ones; the pooled env step at 1024 envs (one wave per SIMD) both ways.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
for t in 1 0; do  # (MJL_TREE read at model creation)
  MJL_TREE=$t MJX355_LIB=mujoco-mjx-lab_amd/mjx_amd/libmjx355_timing.so timeout -k 10 300 python tools/phase_times.py \
    > $O/phases_tree$t.txt 2>&1 || { echo "phases $t failed"; tail -5 $O/phases_tree$t.txt; exit 1; }
done
prof() {  # tag, tree flag, prof_target args...
  local tag=$1 tree=$2; shift 2
  MJL_TREE=$tree timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag/trace -o trace -- \
    python tools/prof_target.py "$@" > $O/$tag.trace.log 2>&1 || { echo "$tag trace failed"; exit 1; }
  echo "$tag ok"
}
prof envstep_pool_1024 1 envstep_pool 1024 200
prof envstep_pool_1024_dense 0 envstep_pool 1024 200
prof speedtest_1024 1 speedtest 1024 200
prof speedtest_1024_dense 0 speedtest 1024 200
python tools/r5/sq_summary.py $O > /dev/null && python tools/r5/show.py $O/summary.json
grep -v "^ *$" $O/phases_tree1.txt | head -40
grep -v "^ *$" $O/phases_tree0.txt | head -40

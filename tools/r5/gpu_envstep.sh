#!/bin/bash
# round 5: env-step kernel with kernarg-late reset / tail arguments (SGPR spills 178 -> 94) and the
# tree-ordered factor kernels (DHumT): GPU parity (physics + env step + reset pool + KATs), then per kernel
# family a rocprofv3 kernel trace and one SQ pass (VALU / waves / cycles), 2048 envs; the pooled env step
# also at C3's 1024 (one-wave kernel); speed test and env step also with MJL_TREE=0 (the dense factors).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_reset_pool.py tests/test_kat_gpu.py tests/test_touch_kat.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "^____" $O/pytest.log | head -60; exit $rc; }
prof() {  # tag, tree flag, prof_target args...
  local tag=$1 tree=$2; shift 2
  MJL_TREE=$tree timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag/trace -o trace -- \
    python tools/prof_target.py "$@" > $O/$tag.trace.log 2>&1 || { echo "$tag trace failed"; exit 1; }
  MJL_TREE=$tree timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY \
    --output-format csv -d $O/$tag/sq -o sq -- python tools/prof_target.py "$@" > $O/$tag.sq.log 2>&1 || { echo "$tag sq failed"; exit 1; }
  find $O/$tag -name '*_kernel_trace.csv' -delete
  echo "$tag ok"
}
prof speedtest_2048 1 speedtest 2048 200
prof speedtest_2048_dense 0 speedtest 2048 200
prof envstep_2048 1 envstep 2048 200
prof envstep_pool_2048 1 envstep_pool 2048 200
prof envstep_pool_2048_dense 0 envstep_pool 2048 200
prof envstep_nr_2048 1 envstep_nr 2048 200
prof envstep_pool_1024 1 envstep_pool 1024 200
python tools/r5/sq_summary.py $O

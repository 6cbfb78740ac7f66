# round 4, first GPU call: env-step prologue without the private-segment EnvArgs + one-wave kernels
# parity of the touched paths, one-wave A/B (interleaved), rocprofv3 stats + WRITE_SIZE of the env step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_reset_pool.py > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for W in 1 0 1 0; do
  MJL_ONE_WAVE=$W timeout -k 10 200 python tools/onewave_ab.py >> $O/onewave_ab.jsonl 2>> $O/onewave_ab.err || exit $?
done
cat $O/onewave_ab.jsonl
for M in envstep envstep_pool; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_$M -o t -- python tools/prof_target.py $M 2048 40 > $O/st_$M.log 2>&1 || exit $?
  find $O/st_$M -name '*_kernel_trace.csv' -delete
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/pmc_${M}_$P -o p -- python tools/prof_target.py $M 2048 10 > $O/pmc_${M}_$P.log 2>&1 || exit $?
  done
done
echo ALL_OK

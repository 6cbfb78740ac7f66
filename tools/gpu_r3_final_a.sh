# round-3 final record, part A: full GPU suite, smoke, the default bench line (part B:
# tools/profile_r3.sh, the rocprofv3 stats and counter passes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo FINAL_A_OK

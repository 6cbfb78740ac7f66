# round 4 end (after the twin-update launch reductions): the full GPU suite, smoke(), the default bench
# line, then the measurement record (rocprofv3 stats of the bench command, per-kernel PMC passes) and
# the N = 2 bench line rehearsed on the one GPU (2 ranks on cuda:0 over gloo)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -v amdgpu.ids $O/pytest_gpu.log | grep -B5 -A40 "^____" | head -80; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-1200 $O/bench.json
bash tools/r4/profile.sh || exit $?
echo PROFILE_OK
MJL_BENCH_REHEARSAL=1 timeout -k 10 500 python bench.py --gpus 2 --no-cpu --steps 20 > gpurun_out/prof4/rehearsal_n2.json 2> gpurun_out/prof4/rehearsal_n2.err || exit $?
tail -c 600 gpurun_out/prof4/rehearsal_n2.json
timeout -k 10 300 python -u tools/ppo_update_probe.py twinonly > $O/twin_update.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/twin_update.txt

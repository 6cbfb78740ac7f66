# round 4 end: the measurement record (rocprofv3 stats of the bench command, per-kernel PMC passes),
# then the N = 2 bench line rehearsed on the one GPU (2 ranks on cuda:0 over gloo)
set -o pipefail
export TMPDIR=/tmp
bash tools/r4/profile.sh || exit $?
echo PROFILE_OK
MJL_BENCH_REHEARSAL=1 timeout -k 10 500 python bench.py --gpus 2 --no-cpu --steps 20 > gpurun_out/prof4/rehearsal_n2.json 2> gpurun_out/prof4/rehearsal_n2.err || exit $?
tail -c 1500 gpurun_out/prof4/rehearsal_n2.json

# round 4: APG C4 direction probes + solver sub-phase stamps (timing build) + Hessian two-accumulator A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
V=mujoco-mjx-lab_amd/mjx_amd/variants
for r in 1 2; do
  for n in a_prev hess2; do
    MJX355_LIB=$PWD/$V/libmjx355_$n.so timeout -k 10 200 python tools/onewave_ab.py > $O/ab_$n.$r.json 2>> $O/ab.err || exit $?
    echo "$n $(cat $O/ab_$n.$r.json)"
  done
done
MJX355_LIB=$PWD/$V/libmjx355_timing.so timeout -k 10 200 python tools/envstep_phases.py > $O/envstep_phases.json 2> $O/envstep_phases.err || exit $?
MJX355_LIB=$PWD/$V/libmjx355_timing.so timeout -k 10 200 python tools/phase_times.py > $O/phase_times.txt 2> $O/phase_times.err || exit $?
grep '^{' $O/envstep_phases.json | cut -c1-3000
bash tools/r4/gpu_c.sh || exit $?
echo ALL_OK_E

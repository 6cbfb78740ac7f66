#!/bin/bash
# A/B of the gradient-noise Newton exit (MJL_GNOISE_EXIT builds in tools/_ab): env-step stage stamps
# (iterations of each launch's slowest env), then the speed test + env-step launch times per build,
# interleaved twice. The A/B builds are made beforehand on the CPU (the exit itself was dropped
# after this measurement; it was a `gsq <= (k eps)^2 * sum(|Ma|+|f|+|J'f|)^2` break after
# the MJX tolerance test in solver_t, under -DMJL_GNOISE_EXIT=k), e.g.
#   hipcc $HIPFLAGS -DMJL_TIMING [-DMJL_GNOISE_EXIT=16] -o tools/_ab/libtiming[_gn16].so capi.hip
set -o pipefail
O=gpurun_out/gnoise; mkdir -p $O
for v in timing timing_gn16; do
  MJX355_LIB=$PWD/tools/_ab/lib$v.so timeout -k 10 200 python -u tools/envstep_phases.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/phases.log || exit 1
done
cat $O/phases.log
for r in 1 2; do
  for v in product gn16; do
    if [ $v = product ]; then L=$PWD/mujoco-mjx-lab_amd/mjx_amd/libmjx355.so; else L=$PWD/tools/_ab/lib$v.so; fi
    MJX355_LIB=$L timeout -k 10 200 python -u bench.py --no-ppo --no-apg --no-cpu > $O/bench_${v}_${r}.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('$O/bench_${v}_${r}.json')); print('$v', $r, round(d['value']/1e6,2), round(d['env_step_kernel_ms']*1e3,1), round(d['env_step_pool_kernel_ms']*1e3,1), d['roofline']['workload_mean_ncon_nefc_iter'], d['env_step_roofline']['workload_mean_ncon_nefc_iter'])" | tee -a $O/bench.log
  done
done

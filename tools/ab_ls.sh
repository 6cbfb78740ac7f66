set -o pipefail
mkdir -p gpurun_out
V=mujoco-mjx-lab_amd/mjx_amd/variants
for f in old new; do
  MJX355_LIB=$PWD/$V/libmjx355_$f.so timeout -k 10 120 python bench.py --no-extras --no-cpu --steps 40 > gpurun_out/ab_$f.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$f.log').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['roofline']['kernel_ms'],4))"
done
for f in timing; do
  echo "== $f"
  MJX355_LIB=$PWD/$V/libmjx355_$f.so timeout -k 10 120 python tools/phase_times.py 2>&1 | grep -v amdgpu.ids || exit 1
done

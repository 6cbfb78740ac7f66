# round 4: twin update timing repeatability (two runs of the probe on one box)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
for k in 1 2; do
  timeout -k 10 300 python -u tools/ppo_update_probe.py twinonly > $O/ab$k.txt 2>&1 || exit $?
  grep -v amdgpu.ids $O/ab$k.txt
done

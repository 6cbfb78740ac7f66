# A/B the policy-kernel variants in mujoco-mjx-lab_amd/mjx_amd/variants/ on the PPO rollout (graph replay)
set -o pipefail
mkdir -p gpurun_out/abpol
for r in 1 2; do
  for f in mujoco-mjx-lab_amd/mjx_amd/variants/*.so; do
    n=$(basename $f .so)
    MJX355_LIB=$PWD/$f timeout -k 10 200 python tools/reset_pool_probe.py --envs 2048 --only 11 > gpurun_out/abpol/${n}_$r.jsonl 2>/dev/null || exit 1
    echo "$n $(cat gpurun_out/abpol/${n}_$r.jsonl)"
  done
done

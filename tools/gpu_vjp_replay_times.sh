# per-phase stamps of the APG replay VJP (MJL_TIMING variant), implicit and unrolled
set -o pipefail
mkdir -p gpurun_out/vjpt
export MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so
REPLAY=1 timeout -k 10 200 python tools/vjp_times.py > gpurun_out/vjpt/replay_implicit.txt 2>&1 || exit $?
REPLAY=1 VJP=unrolled timeout -k 10 200 python tools/vjp_times.py > gpurun_out/vjpt/replay_unrolled.txt 2>&1 || exit $?
cat gpurun_out/vjpt/replay_implicit.txt gpurun_out/vjpt/replay_unrolled.txt | grep -v amdgpu.ids

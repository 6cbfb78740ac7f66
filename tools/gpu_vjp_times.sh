set -o pipefail
mkdir -p gpurun_out/vjpt
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so timeout -k 10 200 python tools/vjp_times.py > gpurun_out/vjpt/vjp_times.txt 2>&1

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/unr
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_apg.py tests/test_adjoint.py tests/test_gpu_configs.py -m gpu > gpurun_out/unr/pytest.log 2>&1 && \
timeout -k 10 300 python tools/bench_apg.py --solver cg --vjp unrolled > gpurun_out/unr/cg_unrolled.json 2> gpurun_out/unr/cg_unrolled.err && \
timeout -k 10 300 python tools/bench_apg.py --solver cg --vjp implicit > gpurun_out/unr/cg_implicit.json 2> gpurun_out/unr/cg_implicit.err && \
SOLVER=cg44 VJP=unrolled MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/variants/libmjx355_timing.so timeout -k 10 200 python tools/vjp_times.py > gpurun_out/unr/unrolled_times.txt 2>&1

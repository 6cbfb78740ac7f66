set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tape
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_vjp_tape.py tests/test_apg.py tests/test_adjoint.py tests/test_gpu_configs.py -m gpu > gpurun_out/tape/pytest.log 2>&1 && \
timeout -k 10 300 python tools/bench_apg.py --solver cg --vjp implicit > gpurun_out/tape/cg_implicit.json 2> gpurun_out/tape/cg_implicit.err && \
timeout -k 10 300 python tools/bench_apg.py --solver cg --vjp unrolled > gpurun_out/tape/cg_unrolled.json 2> gpurun_out/tape/cg_unrolled.err && \
timeout -k 10 300 python tools/bench_apg.py --solver model > gpurun_out/tape/model.json 2> gpurun_out/tape/model.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tape/trace -o trace -- python tools/bench_apg.py --solver cg --vjp implicit --updates 3 > gpurun_out/tape/trace.log 2>&1

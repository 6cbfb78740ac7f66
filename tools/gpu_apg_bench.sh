set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/apgb
timeout -k 10 300 python tools/bench_apg.py --solver cg --vjp implicit > gpurun_out/apgb/cg_implicit.json 2> gpurun_out/apgb/cg_implicit.err && \
timeout -k 10 300 python tools/bench_apg.py --solver cg --vjp unrolled > gpurun_out/apgb/cg_unrolled.json 2> gpurun_out/apgb/cg_unrolled.err && \
timeout -k 10 300 python tools/bench_apg.py --solver model > gpurun_out/apgb/model.json 2> gpurun_out/apgb/model.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/apgb/trace -o trace -- python tools/bench_apg.py --solver cg --vjp implicit --updates 3 > gpurun_out/apgb/trace.log 2>&1

set -o pipefail
mkdir -p gpurun_out/prof_apg
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_apg/trace -o trace -- \
    python tools/bench_apg.py --updates 2 --solver ${SOLVER:-model} ${VJP:+--vjp $VJP} > gpurun_out/prof_apg/trace.log 2>&1

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/apgu
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/apgu/trace -o trace -- python tools/bench_apg.py --solver cg --vjp unrolled --updates 3 > gpurun_out/apgu/trace.log 2>&1

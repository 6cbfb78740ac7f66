set -o pipefail
mkdir -p gpurun_out/suite
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/suite/pytest.log 2>&1

# round 3, first GPU call: the whole GPU suite, then the default bench line, then the update probe
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3a/pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err && \
timeout -k 10 300 python -u tools/ppo_update_probe.py shard > gpurun_out/r3a/shard.txt 2>&1

# round 3: tuned GEMM table (mjx_amd/tunable.py) — update / APG / DP tests with it active, the update
# probes (2048-env update; C5 shard), then the default bench line
mkdir -p gpurun_out/r3j
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ppo_graph.py tests/test_ppo.py tests/test_mlp_kernels.py tests/test_apg.py tests/test_dp_gpu.py tests/test_gpu_configs.py -m gpu > gpurun_out/r3j/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/ppo_update_probe.py graph 2048 > gpurun_out/r3j/upd.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ppo_update_probe.py shard > gpurun_out/r3j/shard.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r3j/bench.json 2> gpurun_out/r3j/bench.err || exit $?
cat gpurun_out/r3j/upd.txt gpurun_out/r3j/shard.txt

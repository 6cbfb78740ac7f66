# round 3: two-stream data-parallel update — tests, then the C5 per-rank shard and the C3 update, fused MLP on / off
mkdir -p gpurun_out/r3f
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_ppo_graph.py tests/test_dp_gpu.py tests/test_mlp_kernels.py -m gpu > gpurun_out/r3f/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 1 0; do
  MJL_FUSED_MLP=$v timeout -k 10 300 python -u tools/ppo_update_probe.py shard >> gpurun_out/r3f/shard.txt 2>&1 || exit $?
  echo "--- fused=$v" >> gpurun_out/r3f/shard.txt
done
exit $rc

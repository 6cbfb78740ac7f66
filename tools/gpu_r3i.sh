# round 3: fused tanh backward + bias-gradient column sum in the PPO update — kernel / layer tests,
# update graph tests, then the update probe (graph) and the C3 leg
mkdir -p gpurun_out/r3i
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mlp_kernels.py tests/test_ppo_graph.py tests/test_ppo.py -m gpu > gpurun_out/r3i/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for t in 1 0; do
  MJL_TANH_FUSED=$t timeout -k 10 200 python -u tools/ppo_update_probe.py graph 2048 >> gpurun_out/r3i/upd.txt 2>&1 || exit $?
  echo "--- tanh_fused=$t" >> gpurun_out/r3i/upd.txt
done
timeout -k 10 300 python -u bench.py --workload ppo --no-cpu > gpurun_out/r3i/bench_ppo.json 2> gpurun_out/r3i/bench_ppo.err || exit $?
cat gpurun_out/r3i/upd.txt

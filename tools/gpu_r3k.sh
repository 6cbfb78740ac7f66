# round 3: loss kernels with wave reductions and parallel final stages, 32-bit gather — PPO tests,
# the update probe, and its kernel breakdown
mkdir -p gpurun_out/r3k
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ppo.py tests/test_ppo_graph.py tests/test_dp_gpu.py tests/test_mlp_kernels.py -m gpu > gpurun_out/r3k/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/ppo_update_probe.py graph 2048 > gpurun_out/r3k/upd.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3k/prof -o upd -- python tools/ppo_update_probe.py graph 2048 > gpurun_out/r3k/prof.log 2>&1 || exit $?
cat gpurun_out/r3k/upd.txt

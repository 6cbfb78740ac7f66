# round 3: the dense-layer kernels (tests), the update with and without them (A/B, interleaved)
mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_mlp_kernels.py tests/test_ppo_graph.py tests/test_ppo.py tests/test_dp_gpu.py -m gpu > gpurun_out/r3d/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 1 0 1 0; do
  MJL_FUSED_MLP=$v timeout -k 10 300 python -u tools/ppo_update_probe.py graph 2048 >> gpurun_out/r3d/ab.txt 2>&1 || exit $?
  echo "--- fused=$v" >> gpurun_out/r3d/ab.txt
done
MJL_FUSED_MLP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d/tr1 -o tr -- python tools/ppo_update_probe.py graph 2048 > gpurun_out/r3d/tr1.log 2>&1 || exit $?
MJL_FUSED_MLP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d/tr0 -o tr -- python tools/ppo_update_probe.py graph 2048 > gpurun_out/r3d/tr0.log 2>&1 || exit $?
find gpurun_out/r3d -name '*_kernel_trace.csv' -delete
exit $rc

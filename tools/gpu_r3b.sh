# round 3: GPU suite (failures reported, not fatal), then the default bench line and the update probe;
# any fault / abort / timeout (exit status other than 0 or 1) stops the script
mkdir -p gpurun_out/r3b
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3b/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err
rc2=$?
echo "bench rc=$rc2"
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 300 python -u tools/ppo_update_probe.py shard > gpurun_out/r3b/shard.txt 2>&1
echo "probe rc=$?"
exit $rc

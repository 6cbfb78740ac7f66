# kernel breakdown of the PPO update at 2048 envs (graph replays; tools/ppo_update_probe.py graph)
export TMPDIR=/tmp
mkdir -p gpurun_out/profupd
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profupd -o upd -- python tools/ppo_update_probe.py graph 2048 > gpurun_out/profupd/run.log 2>&1

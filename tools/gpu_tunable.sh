# PyTorch TunableOp on the PPO update's GEMMs: tune during the eager first update, then time graph replays
mkdir -p gpurun_out/tunable
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable/tunableop_results%d.csv
timeout -k 10 500 python -u tools/ppo_update_probe.py graph 2048 > gpurun_out/tunable/upd_tune.txt 2>&1 || exit $?
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 200 python -u tools/ppo_update_probe.py graph 2048 > gpurun_out/tunable/upd_tuned.txt 2>&1 || exit $?
grep -v "^reading\|^  " gpurun_out/tunable/upd_tuned.txt | tail -8

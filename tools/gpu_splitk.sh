# split-K row count of the update's weight gradients, each with in-process TunableOp tuning (fair GEMM choice)
mkdir -p gpurun_out/splitk
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1
for r in 2048 4096 8192 1024; do
  export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/splitk/tun_$r_%d.csv
  MJL_SPLIT_ROWS=$r timeout -k 10 300 python -u tools/ppo_update_probe.py graph 2048 > gpurun_out/splitk/upd_$r.txt 2>&1 || exit $?
  echo "split_rows=$r: $(grep '^update' gpurun_out/splitk/upd_$r.txt | tail -2 | tr '\n' ' ')"
done

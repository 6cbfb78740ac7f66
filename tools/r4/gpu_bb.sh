# round 4: split-K slices of the twin update thin layers (output, input) weight gradients at C5 per-rank shape
# (the caller's 4 against 2 and 8; 2 / 8 are not in the tuned GEMM table)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4bb
mkdir -p $O
timeout -k 10 400 python -u tools/ppo_update_probe.py thin > $O/ab.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/ab.txt

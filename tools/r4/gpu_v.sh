# round 4: the default bench line with the per-rank C5 update key
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print({k: d.get(k) for k in ['value', 'ppo_c3_ms_per_iter', 'ppo_update_tflops', 'ppo_c5_rank_update_ms', 'ppo_c5_rank_update_steps', 'ppo_c5_rank_update_twin']})"

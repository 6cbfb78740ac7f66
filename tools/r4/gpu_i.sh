# round 4: APG C4 same-batch improvement at every update (two env seeds) and with frozen observation
# statistics after update 100; then the PPO seed spread (5 seeds x 1024 / 2048 envs x 400 iterations)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
P="python -u tools/apg_direction_probe.py implicit 300 --rms-in-loss-only --probe ''"
timeout -k 10 300 python -u tools/apg_direction_probe.py implicit 300 --rms-in-loss-only --probe "" --all-updates --env-seed 332598 > $O/apg_allupd_s332598.jsonl 2> $O/apg1.err || exit $?
timeout -k 10 300 python -u tools/apg_direction_probe.py implicit 300 --rms-in-loss-only --probe "" --all-updates --env-seed 42 > $O/apg_allupd_s42.jsonl 2> $O/apg2.err || exit $?
timeout -k 10 300 python -u tools/apg_direction_probe.py implicit 300 --rms-in-loss-only --probe "" --all-updates --env-seed 332598 --freeze-rms-after 100 > $O/apg_allupd_s332598_frozen.jsonl 2> $O/apg3.err || exit $?
for f in $O/apg_allupd_*.jsonl; do python3 -c "
import json
r=[json.loads(l) for l in open('$f') if l.startswith('{')]
def seg(a,b):
    s=[x for x in r if a<=x['update']<b]
    return round(sum(x['return'] for x in s)/len(s),1), round(sum(x['improved'] for x in s)/len(s),2)
print('$f', [(a,b,seg(a,b)) for a,b in ((0,50),(50,100),(100,150),(150,200),(200,250),(250,300))])
"; done
echo ALL_OK_APG
bash tools/r4/ppo_seeds.sh || exit $?
python tools/summarize_seeds.py gpurun_out/ppo_seeds_r4 > $O/seeds_summary.json && echo ALL_OK_SEEDS

# round 4: APG at C4 (2048 x 128, CG 4/4): training runs with directional checks of the Adam step on
# the update's own resets (tools/apg_direction_probe.py), implicit and unrolled VJP, the reference's
# observation statistics (every observation) and the in-loss-only variant
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 400 python -u tools/apg_direction_probe.py implicit 300 > $O/implicit_ref.jsonl 2> $O/implicit_ref.err || exit $?
timeout -k 10 400 python -u tools/apg_direction_probe.py implicit 300 --rms-in-loss-only > $O/implicit_inloss.jsonl 2> $O/implicit_inloss.err || exit $?
timeout -k 10 400 python -u tools/apg_direction_probe.py unrolled 300 > $O/unrolled_ref.jsonl 2> $O/unrolled_ref.err || exit $?
for f in $O/*.jsonl; do echo $f; python3 -c "
import json,sys
for l in open('$f'):
    r=json.loads(l); print(r['update'], round(r['return'],1), r['descent'], {k:round(v,3) for k,v in r['loss_at_eps'].items()}, r['envs_in_loss'], [round(x,2) for x in r['ga_norm_quantiles_p50_p90_p99_max']], r['reverse_nonfinite_envs'])
"; done
echo ALL_OK

#!/bin/bash
# round 5: (a) the APG sweep's fused launches: GPU tests, bench APG leg fused on / off / on, a kernel
# trace of one APG leg; (b) the PPO rollout policy on the vector ALUs (MJL_POL_VALU=1) against the
# matrix-core kernel: its parity test, rocprofv3 kernel times at 1024 / 2048 envs, the C3 leg both ways.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_apg.py tests/test_vjp_tape.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest_apg.log 2>&1 || fail pytest_apg $O/pytest_apg.log
tail -1 $O/pytest_apg.log
MJL_POL_VALU=1 timeout -k 10 300 python -u -m pytest tests/test_ppo.py -m gpu -x -q -k "rollout_policy or fused_rollout" \
  --timeout 200 --timeout-method thread > $O/pytest_polvalu.log 2>&1 || fail pytest_polvalu $O/pytest_polvalu.log
tail -1 $O/pytest_polvalu.log
show() { python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ["metric", "value", "ms_per_step", "apg_c4_env_steps_per_s", "apg_c4_implicit_env_steps_per_s", "ppo_c3_env_steps_per_s", "ppo_c3_ms_per_iter",
        "ppo_c3_phase_ms", "ppo_policy_roofline"]
print(sys.argv[1], {k: d.get(k) for k in keys if k in d}, {k: d.get("apg_vjp_roofline", {}).get(k) for k in ("kernel_ms_every_env_active", "kernel_ms_trainer_workload")})
PY
}
for F in 1 0 1; do
  MJL_APG_FUSED_OBS=$F timeout -k 10 400 python bench.py --no-cpu --no-extras --no-ppo --apg-updates 5 \
    > $O/bench_apg_fused$F.json 2> $O/bench_apg_fused$F.err || fail bench_apg $O/bench_apg_fused$F.err
  show $O/bench_apg_fused$F.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/apg_trace -o trace -- \
  python bench.py --no-cpu --no-extras --no-ppo --apg-updates 5 > $O/apg_trace.log 2>&1 || fail apg_trace $O/apg_trace.log
find $O/apg_trace -name '*_kernel_trace.csv' -delete
for B in 1024 2048; do
  for V in 0 1 0 1; do
    MJL_POL_VALU=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pol_${B}_v$V -o t -- \
      python tools/prof_target.py policy $B 400 > $O/pol_${B}_v$V.log 2>&1 || fail pol $O/pol_${B}_v$V.log
    find $O/pol_${B}_v$V -name '*_kernel_trace.csv' -delete
    python - $O/pol_${B}_v$V $B $V <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "policy_rollout" in r["Name"]:
            print("policy B", sys.argv[2], "valu", sys.argv[3], r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
  done
done
for V in 0 1; do
  MJL_POL_VALU=$V timeout -k 10 400 python bench.py --workload ppo > $O/bench_ppo_v$V.json 2> $O/bench_ppo_v$V.err \
    || fail bench_ppo $O/bench_ppo_v$V.err
  show $O/bench_ppo_v$V.json
done
echo ALL_OK

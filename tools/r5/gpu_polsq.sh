#!/bin/bash
# round 5: SQ counters of the rollout policy kernel alone (tools/prof_target.py policy, 1024 envs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ps
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
  --output-format csv -d $O/sq1 -o sq1 -- python tools/prof_target.py policy 1024 200 > $O/sq1.log 2>&1 || { tail $O/sq1.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU \
  --output-format csv -d $O/sq2 -o sq2 -- python tools/prof_target.py policy 1024 200 > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
find $O -name '*_kernel_trace.csv' -delete
python - $O <<'PY'
import csv, glob, sys
acc = {}
for f in glob.glob(sys.argv[1] + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "policy_rollout" not in r["Kernel_Name"]:
            continue
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
w = sum(acc["SQ_WAVES"]) / len(acc["SQ_WAVES"])
print("waves", w)
for k, v in sorted(acc.items()):
    m = sum(v) / len(v)
    print(k, round(m, 1), "per wave", round(m / w, 1))
PY

#!/bin/bash
# round 5: the APG policy's small-MLP kernels alone (tools/prof_target.py apgmlp, 2048 rows): kernel trace
# and two SQ counter passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python tools/prof_target.py apgmlp 2048 200 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
  --output-format csv -d $O/sq1 -o sq1 -- python tools/prof_target.py apgmlp 2048 200 > $O/sq1.log 2>&1 || { tail $O/sq1.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH \
  --output-format csv -d $O/sq2 -o sq2 -- python tools/prof_target.py apgmlp 2048 200 > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
find $O -name '*_kernel_trace.csv' -delete
python - $O <<'PY'
import csv, glob, sys
d = sys.argv[1]
for f in glob.glob(d + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "small_mlp" in r["Name"]:
            print("avg", round(float(r["AverageNs"]) / 1e3, 2), "us", r["Name"][:60])
acc = {}
for f in glob.glob(d + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "small_mlp" not in r["Kernel_Name"]:
            continue
        k = acc.setdefault(r["Kernel_Name"][:40], {})
        k.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for n, c in acc.items():
    w = sum(c["SQ_WAVES"]) / len(c["SQ_WAVES"])
    print(n, "waves", w, {k: round(sum(v) / len(v) / (1 if k in ("SQ_WAVES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES") else w), 1) for k, v in c.items()})
PY

"""Summarise a tools/r5/gpu_*.sh profile directory: per kernel family the step kernel's rocprofv3 average
duration (stats pass) and its SQ counters per wave (counter pass).  python tools/r5/sq_summary.py DIR"""
import csv
import glob
import json
import os
import sys


def main(d):
    out = {}
    for tag in sorted(os.listdir(d)):
        p = os.path.join(d, tag)
        if not os.path.isdir(p):
            continue
        recs = {}
        for f in glob.glob(os.path.join(p, "trace", "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "step_kernel" in r["Name"]:
                    recs[r["Name"]] = {"avg_us": float(r["AverageNs"]) / 1e3, "calls": int(r["Calls"])}
        sums = {}
        for f in glob.glob(os.path.join(p, "sq", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if "step_kernel" not in name:
                    continue
                c = sums.setdefault(name, {})
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for name, c in sums.items():
            rec = recs.setdefault(name, {})
            if c.get("SQ_WAVES"):
                w = c["SQ_WAVES"]
                for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_ANY"):
                    if k in c:  # (SQ_WAIT_ANY and SQ_WAVE_CYCLES count in units of 4 cycles)
                        rec[k.lower() + "_per_wave"] = c[k] / w * (4 if k == "SQ_WAIT_ANY" else 1)
                rec["wave_cycles"] = c["SQ_WAVE_CYCLES"] / w * 4
        out[tag] = recs
    print(json.dumps(out, indent=1))
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

"""Summarise tools/r5/gpu_xcd.sh: per tag the dominant kernel's rocprofv3 average duration and its HBM
bytes per launch, 2*FETCH_SIZE + WRITE_SIZE (kB counters; gfx950 FETCH_SIZE counts 128-B requests at 64 B,
MI355X_MICROARCH.md).  python tools/r5/traffic_summary.py DIR"""
import csv
import glob
import json
import os
import sys

KERNELS = ("step_kernel", "vjp_kernel<mjl::Dims<27, 17, 22, 20, 4, 4>, true, 2")


def hot(name):
    return any(k in name for k in KERNELS)


def per_kernel(files, counter):
    acc = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if not hot(r["Kernel_Name"]) or r["Counter_Name"] != counter:
                continue
            k = acc.setdefault(r["Kernel_Name"], {})
            d = r["Dispatch_Id"]
            k[d] = k.get(d, 0.0) + float(r["Counter_Value"])
    return {n: sum(v.values()) / len(v) for n, v in acc.items()}


def main(d):
    out = {}
    for tag in sorted(os.listdir(d)):
        p = os.path.join(d, tag)
        if not os.path.isdir(p):
            continue
        rec = {}
        for f in glob.glob(os.path.join(p, "trace", "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if hot(r["Name"]):
                    rec.setdefault(r["Name"], {}).update(avg_us=float(r["AverageNs"]) / 1e3, calls=int(r["Calls"]))
        for c in ("FETCH_SIZE", "WRITE_SIZE"):  # (pass directories fetch/ and write/)
            sub = c.split("_")[0].lower()
            for n, v in per_kernel(glob.glob(os.path.join(p, sub, "**", "*counter_collection.csv"), recursive=True), c).items():
                rec.setdefault(n, {})[c.lower() + "_kb"] = v
        for n, r in rec.items():
            if "fetch_size_kb" in r and "write_size_kb" in r:
                r["hbm_mb_per_launch"] = (2 * r["fetch_size_kb"] + r["write_size_kb"]) * 1024 / 1e6
        out[tag] = rec
    print(json.dumps(out, indent=1))
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

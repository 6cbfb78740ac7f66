"""Round measurement record from gpurun_out/prof<N>/ (tools/profile_r3.sh, tools/r4/profile.sh) into
profiles/. Usage: python tools/summarize_r3.py [round] [dir] (default r3 gpurun_out/prof3; round 4:
r4 gpurun_out/prof4, files under profiles/r4/).

Per kernel family (speed test, env step with in-place resets / with the reset pool / without resets,
APG replay VJP): the rocprofv3 --stats average duration, HBM bytes per launch (2 x FETCH_SIZE +
WRITE_SIZE: gfx950 FETCH_SIZE tallies 128-B requests at 64 B, WRITE_SIZE is exact;
MI355X_MICROARCH.md "HBM"), and the SQ counters per wave (= per env-step; SQ cycle counters in units
of 4 cycles). Writes profiles/r3_kernels.json, the bench-command stats as profiles/r3_bench_kernel_stats.csv,
and profiles/pmc_traffic.json (read by bench.py for `traffic` while the kernel sources are unchanged).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
from mjx_amd import _lib  # noqa: E402

ROUND = sys.argv[1] if len(sys.argv) > 1 else "r3"
P = os.path.join(ROOT, sys.argv[2]) if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof3")
# round 4 added the waves-per-SIMD template argument (2 at the 2048-env launches profiled here)
_MW = ", 2>" if ROUND != "r3" else ">"
KERNELS = {
    "speedtest": "step_kernel<mjl::Dims<27, 17, 22, 20, 48, 16>, 2" + _MW,
    "envstep": "step_kernel<mjl::Dims<27, 17, 22, 20, 48, 16>, 3" + _MW,
    "envstep_pool": "step_kernel<mjl::Dims<27, 17, 22, 20, 48, 16>, 3" + _MW,
    "envstep_nr": "step_kernel<mjl::Dims<27, 17, 22, 20, 48, 16>, 3" + _MW,
    "vjp": "vjp_kernel<mjl::Dims<27, 17, 22, 20, 4, 4>, true, 2, true>",
}
TRAFFIC_KEY = {"speedtest": "bytes_per_launch", "envstep": "env_step_bytes_per_launch",
               "vjp": "vjp_bytes_per_launch"}


def one(pattern):
    hits = sorted(glob.glob(os.path.join(P, pattern), recursive=True))
    return hits[0] if hits else None


def stats_avg_ns(path, kernel):
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Name"]:
                return float(row["AverageNs"]), int(row["Calls"])
    return None, 0


def counters(path, kernel):
    """{counter: [per-dispatch values]} for dispatches of `kernel`."""
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                out.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return out


def steady(v):
    return v[len(v) // 10:] if len(v) > 10 else v


def mean(v):
    v = steady(v)
    return sum(v) / len(v) if v else None


def main():
    out = os.path.join(ROOT, "profiles")
    pre = os.path.join(out, ROUND, "") if ROUND in ("r4", "r5", "r6") else os.path.join(out, ROUND + "_")
    os.makedirs(os.path.dirname(pre), exist_ok=True)
    rec = {"round": ROUND, "src_hash": _lib.source_hash(), "envs": 2048,
           "units": {"kernel_us": "rocprofv3 --stats AverageNs / 1e3",
                     "hbm_bytes_per_launch": "2 * FETCH_SIZE + WRITE_SIZE (KB counters x 1024)",
                     "sq_per_wave": "counter / SQ_WAVES per dispatch (SQ_*CYCLES and WAIT/ACTIVE in units of 4 cycles)"},
           "kernels": {}}
    for mode, kern in KERNELS.items():
        r = {"kernel": kern}
        st = one(f"{mode}/trace/**/trace_kernel_stats.csv")
        if st:
            ns, calls = stats_avg_ns(st, kern)
            r["kernel_us"], r["calls"] = (ns / 1e3 if ns else None), calls
            shutil.copy(st, f"{pre}{mode}_kernel_stats.csv")
        f = one(f"{mode}/fetch/**/fetch_counter_collection.csv")
        w = one(f"{mode}/write/**/write_counter_collection.csv")
        if f and w:
            fk, wk = mean(counters(f, kern).get("FETCH_SIZE", [])), mean(counters(w, kern).get("WRITE_SIZE", []))
            r["fetch_size_kb"], r["write_size_kb"] = fk, wk
            r["hbm_bytes_per_launch"] = (2.0 * fk + wk) * 1024.0 if fk is not None and wk is not None else None
        sq = {}
        for p in ("sq1", "sq2"):
            c = one(f"{mode}/{p}/**/{p}_counter_collection.csv")
            if c:
                sq.update(counters(c, kern))
        if "SQ_WAVES" in sq:
            waves = mean(sq["SQ_WAVES"])
            r["sq_waves_per_dispatch"] = waves
            r["sq_per_wave"] = {k: mean(v) / waves for k, v in sorted(sq.items())
                                if k not in ("SQ_WAVES", "GRBM_GUI_ACTIVE") and mean(v) is not None}
            if "GRBM_GUI_ACTIVE" in sq:
                r["grbm_gui_active"] = mean(sq["GRBM_GUI_ACTIVE"])
        rec["kernels"][mode] = r
    b = one("bench_trace/**/trace_kernel_stats.csv")
    if b:
        shutil.copy(b, f"{pre}bench_kernel_stats.csv")
        rec["bench_command_stats"] = {m: (stats_avg_ns(b, k)[0] or 0) / 1e3 for m, k in KERNELS.items()
                                      if m in ("speedtest", "envstep", "vjp")}
    json.dump(rec, open(f"{pre}kernels.json", "w"), indent=1)
    traffic = {"round": ROUND, "src_hash": rec["src_hash"], "envs": 2048,
               "formula": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts 128-B requests at 64 B)"}
    for mode, key in TRAFFIC_KEY.items():
        k = rec["kernels"].get(mode, {})
        traffic[key] = k.get("hbm_bytes_per_launch")
        traffic[key.replace("bytes_per_launch", "kernel")] = KERNELS[mode]
    json.dump(traffic, open(os.path.join(out, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()

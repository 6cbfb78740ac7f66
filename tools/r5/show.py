"""Print a tools/r5/sq_summary.py summary.json as one line per (profile tag, kernel)."""
import json
import sys

d = json.load(open(sys.argv[1]))
for t, ks in d.items():
    for k, v in ks.items():
        mode = k.split(">, ")[-1].split(">")[0] if ">, " in k else "?"
        tree = "T" if ", 1>, " in k else "D"
        print(f"{t:26s} mode,mw {mode:5s}{tree} {v.get('avg_us', 0):8.2f}us n={v.get('calls')} "
              f"valu {v.get('sq_insts_valu_per_wave', 0):7.0f} salu {v.get('sq_insts_salu_per_wave', 0):6.0f} "
              f"lds {v.get('sq_insts_lds_per_wave', 0):5.0f} cyc {v.get('wave_cycles', 0):7.0f} "
              f"wait {v.get('sq_wait_any_per_wave', 0):7.0f}")

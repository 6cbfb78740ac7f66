"""Seed spread of the PPO return curves: mean +- std (population, over seeds) of train_return_avg at
iterations 100 / 200 / 300 / 399 and of eval_return at 100 / 200 / 300, per env count, from
DIR/s{seed}_b{envs}.metrics.jsonl (tools/r4/ppo_seeds.sh). Prints one JSON document."""
import glob
import json
import os
import re
import statistics
import sys


def load(path):
    rows = {}
    with open(path) as f:
        for line in f:
            r = json.loads(line)
            rows[int(r["step"])] = r
    return rows


def main(d):
    runs = {}
    for p in sorted(glob.glob(os.path.join(d, "s*_b*.metrics.jsonl"))):
        m = re.match(r"s(\d+)_b(\d+)\.metrics\.jsonl", os.path.basename(p))
        runs.setdefault(int(m.group(2)), {})[int(m.group(1))] = load(p)
    out = {}
    for envs, by_seed in sorted(runs.items()):
        res = {"seeds": sorted(by_seed)}
        for key, its in (("train_return_avg", (100, 200, 300, 399)), ("eval_return", (100, 200, 300))):
            for it in its:
                v = [r[it][key] for r in by_seed.values() if it in r and key in r[it]]
                if v:
                    res[f"{key}@{it}"] = {"mean": statistics.fmean(v), "std": statistics.pstdev(v),
                                          "min": min(v), "max": max(v), "n": len(v),
                                          "values": {s: r[it][key] for s, r in sorted(by_seed.items())
                                                     if it in r and key in r[it]}}
        sps = [statistics.median(x["env_steps_per_sec"] for k, x in r.items() if k >= 10) for r in by_seed.values()]
        res["env_steps_per_s_median"] = statistics.fmean(sps)
        out[str(envs)] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ppo_seeds_r4")

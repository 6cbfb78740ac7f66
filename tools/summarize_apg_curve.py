"""Summarise the APG C4 learning-check runs (tools/apg_curve_c4.sh) into profiles/r3_apg_c4_curve.json:
per run, 10-update means of return / forward-dropped / reverse-nonfinite envs and the env-steps/s median."""
import glob
import json
import sys

import numpy as np

out = {"config": "2048 envs x 128 horizon, CG 4/4, hidden 32x2, lr 5e-5, clip 0.3, obs normalisation from update 100, "
                 "statistics every 10 updates; MI355X, 1 GPU", "runs": {}}
for name in ("unrolled", "implicit", "unrolled_allobs"):
    paths = glob.glob(f"gpurun_out/apgc4/{name}/*/logs/metrics.jsonl")
    if not paths:
        continue
    rows = [json.loads(line) for line in open(paths[0])]
    ret = np.array([r["return"] for r in rows])
    blocks = range(0, len(rows), 10)
    out["runs"][name] = {
        "updates": len(rows),
        "rms_in_loss_only": name != "unrolled_allobs",
        "vjp": "implicit" if name == "implicit" else "unrolled",
        "return_mean_per_10": [round(float(ret[i:i + 10].mean()), 3) for i in blocks],
        "forward_dropped_mean_per_10": [round(float(np.mean([r["forward_dropped_envs"] for r in rows[i:i + 10]])), 1) for i in blocks],
        "reverse_nonfinite_mean_per_10": [round(float(np.mean([r["reverse_nonfinite_envs"] for r in rows[i:i + 10]])), 1) for i in blocks],
        "grad_norm_finite_frac": float(np.isfinite([r["grad_norm"] for r in rows]).mean()),
        "env_steps_per_s_median": float(np.median([r["env_steps_per_sec"] for r in rows[2:]])),
    }
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "profiles/r3_apg_c4_curve.json", "w"), indent=1)

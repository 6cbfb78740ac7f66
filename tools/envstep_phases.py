"""Diagnostic: where the PPO env step's time goes, per env and for each launch's slowest env.
Needs the MJL_TIMING build (s_memtime stamps, lane 0): MJX355_LIB=<timing lib>. 1024 envs (C3) with
the trainer's reset pool, uniform random actions; after 2 x 128 warm-up steps, 20 measured steps.
Prints mean cycles per stage over all envs, the same for the slowest env of each launch, and how
the slowest env's Newton iterations compare with the mean."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import mjx_amd  # noqa: E402
from mjx_amd import _lib, mjx  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402

STAGES = [("state loads", 36, 0), ("kinematics", 0, 1), ("com_pos+crb+M", 1, 2), ("velocity", 2, 3),
          ("factor M", 3, 4), ("collision+rows", 4, 5), ("solver", 5, 6), ("sensors", 6, 7),
          ("integrate", 7, 8), ("env post", 8, 37), ("reset merge", 37, 38), ("write-back", 38, 39)]
# the solver's accumulated sub-phase stamps (TACC slots) and counters (TCOUNT)
SOLVER_SUBS = {9: "warm start", 10: "line search (+step)", 11: "update + convergence", 12: "hessian J'DJ",
               13: "cholesky factor+solve", 28: "ls: M s, J s", 29: "ls: |s|, c1, c2, p0", 30: "ls: segment test + q",
               31: "ls: 3-point loop", 14: "count: 3-point iterations", 15: "count: line searches"}


def main():
    B = int(os.environ.get("PROBE_B", "1024"))
    L = _lib.lib()
    L.mjl_debug_set_stamps.argtypes = [C.c_void_p]
    cfg = reference_ppo_config()
    m = mjx_amd.load_model("humanoid_mjx")
    sys_ = mjx.put_model(m)
    env = HumanoidEnv(sys_, resolve_ids(m, cfg.env_config), B, device=0, seed=42, store_derived=True)
    env.enable_reset_pool(16)
    pool_n = torch.full((1,), 4, dtype=torch.int32, device="cuda")
    buf = torch.zeros((B, 48), dtype=torch.int64, device="cuda")
    L.mjl_debug_set_stamps(C.c_void_p(buf.data_ptr()))
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(2):
        env.fill_reset_pool(pool_n)
        for _ in range(128):
            env.step(torch.rand((B, env.act_dim), generator=g, device="cuda") * 2 - 1)
    env.fill_reset_pool(pool_n)
    rows, slow, it_all, it_slow, ev_us = [], [], [], [], []
    subs_all, subs_slow = [], []
    for _ in range(20):
        act = torch.rand((B, env.act_dim), generator=g, device="cuda") * 2 - 1
        torch.cuda.synchronize()
        buf.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.step(act)
        e1.record()
        torch.cuda.synchronize()
        ev_us.append(e0.elapsed_time(e1) * 1e3)
        s = buf.cpu().numpy().astype(np.float64)
        st = env.data.get("stats").cpu().numpy()
        d = np.stack([s[:, b] - s[:, a] for _, a, b in STAGES], 1)
        tot = s[:, 39] - s[:, 36]
        k = int(np.argmax(tot))
        rows.append(d)
        slow.append(d[k])
        sv = np.stack([s[:, i] for i in SOLVER_SUBS], 1)
        subs_all.append(sv)
        subs_slow.append(sv[k])
        it_all.append(st[:, 2].mean())
        it_slow.append(st[k, 2])
    d = np.concatenate(rows)
    sl = np.stack(slow)
    out = {"B": B, "launch_us_median": float(np.median(ev_us)), "mean_total_cycles": float(d.sum(1).mean()),
           "slowest_total_cycles": float(sl.sum(1).mean()),
           "mean_newton_iters": float(np.mean(it_all)), "slowest_env_newton_iters": float(np.mean(it_slow)),
           "stages_mean": {n: round(float(d[:, i].mean())) for i, (n, _, _) in enumerate(STAGES)},
           "stages_slowest": {n: round(float(sl[:, i].mean())) for i, (n, _, _) in enumerate(STAGES)}}
    sa, ss = np.concatenate(subs_all), np.stack(subs_slow)
    out["solver_subs_mean"] = {n: round(float(sa[:, j].mean()), 2) for j, n in enumerate(SOLVER_SUBS.values())}
    out["solver_subs_slowest"] = {n: round(float(ss[:, j].mean()), 2) for j, n in enumerate(SOLVER_SUBS.values())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

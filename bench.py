"""Benchmark: humanoid env-steps/s on MI355X (BASELINE.json metric), one process per GPU.

Workload (BASELINE.json configs[1], the reference's speed-test row, mjx_humanoid_speed_test.py:
48-108): models/humanoid_mjx.xml, 2048 envs per GPU; every step starts from a fresh make_data state
at qpos0 with qvel[0] = linspace(0, 1, B) and runs one full mjx.step (collision, constraints, Newton
solve, implicitfast integration), output qpos[0]. One "step" = one launch over the batch. The state
is re-initialised inside the kernel each launch, so every launch does the full work (nothing is
hoisted the way XLA may hoist the reference's loop-invariant fori_loop body).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--envs B]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

REF_DEVICE_STEPS_PER_S = 72618.0  # HUMANOID_MJX device steps/s (README.md:77), batch 4096
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)
F32_PEAK_TFLOPS = 157.3           # MI355X_MICROARCH.md: peak FP32 matrix (dense) = FP32 vector
SPEEDTEST_KERNEL = "step_kernel<mjl::Dims<27, 17, 22, 20, 48, 16>, 2>"  # rocprofv3 kernel name


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--envs", type=int, default=2048)
    p.add_argument("--model", default="humanoid_mjx")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    p.add_argument("--no-extras", action="store_true", help="skip the secondary measurements")
    return p.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist, rank, world, local
    torch.cuda.set_device(0)
    return None, 0, 1, 0


def barrier(dist):
    if dist is not None:
        dist.barrier()


def timed_launches(fn, steps, warmup, dist):
    """W untimed + K timed launches. Returns (wall seconds, mean kernel ms from HIP events on the
    launch stream)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return wall, e0.elapsed_time(e1) / steps


def max_over_ranks(x, dist, local):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=torch.device("cuda", local))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_traffic(B: int):
    """HBM bytes per speed-test launch from the committed rocprofv3 PMC passes (tools/profile_round.sh),
    used only when they were taken on the current kernel sources and this batch size."""
    from mjx_amd import _lib
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("src_hash") != _lib.source_hash() or int(t.get("envs", -1)) != B:
        return None
    return t.get("bytes_per_launch")


def cpu_baseline(model, budget_s: float):
    """Oracle (CPU restatement, fp64) on the same speed-test workload, one env per host thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from concurrent.futures import ThreadPoolExecutor

    from oracle import Oracle
    orc = Oracle(model)
    probe = np.linspace(0.0, 1.0, 8)
    t = time.perf_counter()
    orc.speedtest(probe)
    per = (time.perf_counter() - t) / probe.size
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, min(16, avail))
    n_per_thread = max(8, int(budget_s / max(per, 1e-6) / 2))
    vel = np.linspace(0.0, 1.0, n_per_thread)
    workers = [Oracle(model) for _ in range(threads)]
    t = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda w: w.speedtest(vel), workers))
    dt = time.perf_counter() - t
    total = threads * n_per_thread
    return {"value": total / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{total} humanoid_mjx speed-test steps (fresh qpos0 state, qvel[0]=linspace(0,1)), "
                      f"fp64 oracle, {threads} host threads, {dt:.1f} s; single-thread {1.0 / per:.0f} steps/s"}


def main():
    args = parse()
    dist, rank, world, local = dist_setup(args)
    import mjx_amd
    from mjx_amd import mjx

    model = mjx_amd.load_model(args.model)
    sys_ = mjx.put_model(model)
    B = args.envs
    d = mjx.make_data(sys_, B, device=local)
    vel = torch.linspace(0.0, 1.0, B, device=f"cuda:{local}")
    out = torch.empty_like(vel)

    wall, kern_ms = timed_launches(lambda: mjx.speedtest_step(sys_, d, vel, out), args.steps, args.warmup, dist)
    wall = max_over_ranks(wall, dist, local)
    value = B * args.steps * world / wall
    ms_per_step = wall / args.steps * 1e3

    # solver statistics of exactly these states (a forward pass from the same fresh state), for the
    # algorithmic FLOP count of one env-step (mjx_amd/flops.py, DESIGN.md "Roofline")
    from mjx_amd import flops as flops_mod
    ds = mjx.make_data(sys_, B, device=local)
    qv = torch.zeros((B, sys_.nv), device=f"cuda:{local}")
    qv[:, 0] = vel
    ds.set("qvel", qv)
    mjx.forward(sys_, ds)
    wst = ds.get("stats").double().mean(0).cpu().numpy()
    fl = flops_mod.step_flops(model, float(wst[0]), float(wst[1]), float(wst[2]), nact=float(wst[3]))
    achieved_tflops = fl["total"] * B / (kern_ms * 1e-3) / 1e12
    bytes_per_env = 8  # speed test: 4 B vel in + 4 B qpos[0] out; the state never leaves LDS
    achieved_gbs = bytes_per_env * B / (kern_ms * 1e-3) / 1e9
    traffic = pmc_traffic(B)

    extras = {}
    if not args.no_extras and rank == 0:
        # trajectory mode: carried state + random ctrl, full mjx.step with warm start (1048 B/env-step
        # state traffic for the fused env step; mjl_step reads qpos/qvel/qacc_ws/ctrl/time, writes the same)
        dd = mjx.make_data(sys_, B, device=local)
        dd.set_option(0, 0)
        g = torch.Generator(device=f"cuda:{local}").manual_seed(0)
        ctrl = torch.rand((B, sys_.nu), generator=g, device=f"cuda:{local}") * 2 - 1
        tw, tk = timed_launches(lambda: mjx.step(sys_, dd, ctrl), args.steps, args.warmup, None)
        extras["trajectory_mode_steps_per_s"] = B * args.steps / tw
        # fused PPO env step (physics + reward + obs + auto-reset) with random actions
        from mjx_amd.config import reference_ppo_config
        from mjx_amd.envs import HumanoidEnv, resolve_ids
        cfg = reference_ppo_config().env_config
        resolve_ids(model, cfg)
        env = HumanoidEnv(sys_, cfg, B, device=local, seed=1)
        env.reset()
        act = torch.rand((B, sys_.nu), generator=g, device=f"cuda:{local}") * 2 - 1
        ew, ek = timed_launches(lambda: env.step(act), args.steps, args.warmup, None)
        extras["env_step_steps_per_s"] = B * args.steps / ew
        extras["env_step_kernel_ms"] = ek
        extras["env_step_hbm_gbs"] = 1048 * B / (ek * 1e-3) / 1e9
        dd.set_option(0, 1)
        mjx.step(sys_, dd, ctrl)
        st = dd.get("stats").cpu().numpy()
        extras["trajectory_mean_ncon_nefc_iter"] = [float(x) for x in st[:, :3].mean(0)]
        # the reference's own batch size for the README row
        d4 = mjx.make_data(sys_, 4096, device=local)
        v4 = torch.linspace(0.0, 1.0, 4096, device=f"cuda:{local}")
        o4 = torch.empty_like(v4)
        w4, _ = timed_launches(lambda: mjx.speedtest_step(sys_, d4, v4, o4), args.steps, args.warmup, None)
        extras["speedtest_b4096_steps_per_s"] = 4096 * args.steps / w4
        extras["speedtest_b4096_vs_readme"] = extras["speedtest_b4096_steps_per_s"] / REF_DEVICE_STEPS_PER_S

    if rank == 0:
        cpu = cpu_baseline(model, args.cpu_seconds) if world == 1 else None
        line = {
            "metric": "humanoid env-steps/sec (whole node)",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": value / REF_DEVICE_STEPS_PER_S,
            "dtype": "f32",
            "data": "synthetic (speed-test states: qpos0, qvel[0]=linspace(0,1,B))",
            "config": {"workload": f"{args.model}.xml speed-test step (fresh state per step), {B} envs per GPU",
                       "envs_per_gpu": B, "parallelism": f"env-sharded x{world}, no collective",
                       "baseline_note": "vs_baseline divides by the README HUMANOID_MJX row (72,618 steps/s, batch 4096)"},
            "roofline": {"bound": "mfma", "achieved": achieved_tflops, "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved_tflops / F32_PEAK_TFLOPS, "traffic": traffic,
                         "kernel": SPEEDTEST_KERNEL, "kernel_ms": kern_ms,
                         "flops_per_env_step": fl["total"],
                         "workload_mean_ncon_nefc_iter": [float(x) for x in wst[:3]],
                         "workload_mean_active_rows_per_hessian": float(wst[3]),
                         "hbm_algorithmic_bytes_per_launch": bytes_per_env * B,
                         "hbm_achieved_gbs": achieved_gbs, "hbm_frac": achieved_gbs / HBM_PEAK_GBS,
                         "note": "FP32 roof (dense MFMA = vector peak); achieved = algorithmic FP32 FLOPs "
                                 "(mjx_amd/flops.py) / kernel time; traffic = HBM bytes per launch from the "
                                 "committed FETCH_SIZE/WRITE_SIZE passes (profiles/, DESIGN.md)"},
            "cpu_baseline": cpu,
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

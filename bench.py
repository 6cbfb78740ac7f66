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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--workload", default="speedtest", choices=["speedtest", "ppo"])
    p.add_argument("--steps", type=int, default=None, help="timed steps (speedtest launches: 50; ppo iterations: 3)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (speedtest: 5; ppo: 2, graph capture)")
    p.add_argument("--envs", type=int, default=None, help="envs per GPU (speedtest: 2048; ppo: 1024)")
    p.add_argument("--model", default="humanoid_mjx")
    p.add_argument("--cpu-steps", type=int, default=10000, help="CPU baseline: steps per env (C1: 10,000)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    p.add_argument("--no-extras", action="store_true", help="skip the secondary measurements")
    a = p.parse_args(argv)
    ppo = a.workload == "ppo"
    if a.steps is None:
        a.steps = 3 if ppo else 50
    if a.warmup is None:
        a.warmup = 2 if ppo else 5
    if a.envs is None:
        a.envs = 1024 if ppo else 2048
    return a


def launch_cmd(argv, n: int, port: int):
    """The child command that runs this script on n ranks of one node (rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
                         f"torch.distributed.run --nproc-per-node {args.gpus}, or without WORLD_SIZE")
    if world > 1:
        import torch.distributed as dist
        if os.environ.get("MJL_BENCH_REHEARSAL") == "1":
            # rehearsal of the N-rank path on a one-GPU box: every rank on cuda:0 over gloo (RCCL
            # refuses two ranks on one device); its numbers are not scaling measurements
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
            return dist, rank, world, 0
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


def cpu_model_name() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(steps: int):
    """BASELINE config C1 (mjx_humanoid_speed_test.py:140 HUMANOID row): humanoid.xml,
    1 env x `steps` carried steps from qpos0, ctrl = 0 and ctrl ~ U[-1,1] (seed 0); single thread,
    best of 3, then one env per core on every core this process may use, best of 3; warm-up run
    excluded. MuJoCo is not importable on the box (plan B), so the timed CPU path is this
    build's serial C++ restatement (oracle/, kind "port") in its fp32 instantiation, the GPU's
    arithmetic type. `cores` = the threads used: the CPUs in this process's affinity mask, capped by
    OMP_NUM_THREADS when set (the pool's CPU share per GPU, 16; os.cpu_count() shows the host)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from concurrent.futures import ThreadPoolExecutor

    import mjx_amd
    from oracle import Oracle
    m = mjx_amd.load_model("humanoid")
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(avail, share) if share > 0 else avail)
    rng = np.random.default_rng(0)
    ctrls = {"ctrl0": np.zeros((steps, m.nu)), "ctrlU": rng.uniform(-1.0, 1.0, (steps, m.nu))}

    def run(ctrl):
        o = Oracle(m, use_float=True)
        s = o.new_state()
        t = time.perf_counter()
        o.rollout(s, ctrl)
        return time.perf_counter() - t

    res = {}
    t_all = time.perf_counter()
    for name, ctrl in ctrls.items():
        run(ctrl[:200])  # warm-up (page-in, allocator), not timed
        single = min(run(ctrl) for _ in range(3))
        best = None
        with ThreadPoolExecutor(threads) as ex:
            for _ in range(3):
                t = time.perf_counter()
                list(ex.map(lambda _i: run(ctrl), range(threads)))
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
        res[name] = (steps / single, threads * steps / best)
    total_s = time.perf_counter() - t_all
    return {"value": res["ctrlU"][1], "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model_name(), "host_cpus": os.cpu_count(), "affinity_cpus": avail,
            "single_thread": {k: v[0] for k, v in res.items()}, "all_cores": {k: v[1] for k, v in res.items()},
            "sample": f"C1: humanoid.xml (Newton 100/50, Euler + eulerdamp), 1 env x {steps} carried steps "
                      f"from qpos0 per thread, ctrl U[-1,1] seed 0 (value) and ctrl 0; oracle/ C++ "
                      f"restatement, fp32; single thread best of 3, then {threads} threads x 1 env, best of 3; "
                      f"{total_s:.1f} s in all"}


def run_ppo(args, dist, rank, world, local):
    """BASELINE config C5 (C3 at N = 1): PPO with src/config.json values, args.envs envs per rank,
    T = 256, 4 epochs, global minibatch 65,536 (each rank takes its share of every minibatch), one
    RCCL all-reduce of the flattened policy + value gradients per minibatch (train_ppo.py:233-252)."""
    from mjx_amd import mjx, ppo
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    import mjx_amd
    cfg = reference_ppo_config()
    cfg.num_envs, cfg.rollout_length = args.envs * world, 256
    m = mjx_amd.load_model(args.model)
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, cfg.env_config), args.envs, device=local,
                      seed=cfg.seed * 7919 + rank)
    tr = ppo.PPOTrainer(cfg, env, None, device=f"cuda:{local}", dist=dist)
    for it in range(max(2, args.warmup)):  # >= 2: the second rollout captures the rollout graph
        tr.iteration(it)
    tr.allreduce_events = []
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = [tr.iteration(it) for it in range(args.steps)]
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    wall = max_over_ranks(time.perf_counter() - t0, dist, local)
    ar = [a.elapsed_time(b) for a, b in tr.allreduce_events]
    ar_ms = max_over_ranks(sum(ar) / len(ar) if ar else 0.0, dist, local)
    nmb = len(ar) // max(1, args.steps)
    total = float(args.envs * world * cfg.rollout_length * args.steps)
    grad_numel = sum(p.numel() for p in list(tr.policy.parameters()) + list(tr.value.parameters()))
    return {
        "metric": "humanoid PPO env-steps/sec (whole node)", "value": total / wall, "unit": "env-steps/s",
        "n_gpus": world, "steps": args.steps, "warmup": max(2, args.warmup), "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (env resets drawn on the device; random-init policy / value nets)",
        "config": {"workload": f"PPO src/config.json: {args.envs} envs per GPU x {cfg.rollout_length} rollout x "
                               f"{cfg.epochs} epochs, global minibatch {cfg.minibatch_size}",
                   "envs_per_gpu": args.envs, "global_envs": args.envs * world,
                   "parallelism": (f"env-sharded x{world}, {'RCCL' if dist.get_backend() == 'nccl' else 'gloo'} all-reduce "
                                   f"per minibatch") if world > 1 else "1 GPU"},
        "step": "one PPO iteration (rollout + GAE + updates), synced",
        "rccl_ranks": world if dist is not None and dist.get_backend() == "nccl" else 0,
        "rehearsal": os.environ.get("MJL_BENCH_REHEARSAL") == "1",
        "allreduce_ms_per_minibatch": ar_ms if dist is not None else None,
        "minibatches_per_iteration": nmb if dist is not None else cfg.epochs * (args.envs * cfg.rollout_length // cfg.minibatch_size),
        "allreduce_bytes": 4 * grad_numel,
        "train_return_avg": [r["train_return_avg"] for r in res],
        "roofline": None, "cpu_baseline": None,
    }


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launch the N ranks as a child process (nothing here has touched the GPU yet) and pass
        # its status through; rank 0 of the child prints the JSON line
        import subprocess
        sys.exit(subprocess.run(launch_cmd(sys.argv[1:], args.gpus, free_port())).returncode)
    dist, rank, world, local = dist_setup(args)
    if args.workload == "ppo":
        line = run_ppo(args, dist, rank, world, local)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
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
        cpu = cpu_baseline(args.cpu_steps) if world == 1 and not args.no_cpu else None
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
        if os.environ.get("MJL_BENCH_REHEARSAL") == "1":
            line["rehearsal"] = True
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

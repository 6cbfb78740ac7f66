"""Benchmark: humanoid env-steps/s on MI355X (BASELINE.json metric), one process per GPU.

Headline (`value`, BASELINE.json configs[1], the reference's speed-test row,
mjx_humanoid_speed_test.py:48-108): models/humanoid_mjx.xml, 2048 envs per GPU; every step starts
from a fresh make_data state at qpos0 with qvel[0] = linspace(0, 1, B) and runs one full mjx.step
(collision, constraints, Newton solve, implicitfast integration), output qpos[0]. One "step" = one
launch over the batch. The state is re-initialised inside the kernel each launch, so every launch does
the full work (nothing is hoisted the way XLA may hoist the reference's loop-invariant fori_loop body).

The same line carries the metric's other half and the other BASELINE configs, each timed in this run:
  * N = 1: the fused PPO env step with its roofline; C3 PPO (src/config.json, 1024 envs x 256 x 4
    epochs x 65,536) throughput and its return@iteration (train_return_avg at iterations 0/25/50/100
    and eval_return at 100, train_ppo.py:321-424); C4 APG (2048 x 128, CG 4/4, backward through the
    simulator, train_apg.py:258-315) under both solve derivatives, with the replay VJP kernel's
    roofline; the CPU legs (C1 humanoid.xml carried steps, and the speed-test states themselves).
  * N > 1: C5, PPO with 1024 envs per rank and the per-minibatch RCCL all-reduce of both nets'
    gradients timed (train_ppo.py:233-252), next to the sharded speed test.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--envs B]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

REF_DEVICE_STEPS_PER_S = 72618.0  # HUMANOID_MJX device steps/s (README.md:77), batch 4096
REF_HUMANOID_XML_STEPS_PER_S = 6176.0  # README.md:76 HUMANOID row (humanoid.xml)
REF_SPHERE_STEPS_PER_S = 5957372.0     # README.md:78 SPHERE row
SPHERE_XML = ("<mujoco><worldbody><body><freejoint/><geom size='.15' mass='1' type='sphere'/></body></worldbody>"
              "</mujoco>")               # mjx_humanoid_speed_test.py:29-40
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)
F32_PEAK_TFLOPS = 157.3           # MI355X_MICROARCH.md: peak FP32 matrix (dense) = FP32 vector
SPEEDTEST_KERNEL = "step_kernel<mjl::Dims<27, 17, 22, 20, 48, 16>, 2, 2>"  # rocprofv3 kernel name
ENV_STEP_BYTES = 1048             # 113 floats in + 149 out per fused env step
PPO_CURVE_ITERS = (0, 25, 50, 100)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--workload", default="all", choices=["all", "speedtest", "ppo"],
                   help="all: the headline speed test plus every leg; speedtest: the headline only; "
                        "ppo: the PPO leg alone as the headline (C3 / C5)")
    p.add_argument("--steps", type=int, default=None, help="timed steps (speedtest launches: 50; ppo iterations: 3)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (speedtest: 5; ppo: 2, graph capture)")
    p.add_argument("--speedtest-launch", choices=["graph", "eager"], default="graph",
                   help="the headline's K timed steps as one hipGraph replay (default) or K eager launches")
    p.add_argument("--envs", type=int, default=None, help="envs per GPU (speedtest: 2048; ppo: 1024)")
    p.add_argument("--model", default="humanoid_mjx")
    p.add_argument("--ppo-envs", type=int, default=1024, help="PPO leg: envs per GPU (C3 / C5: 1024)")
    p.add_argument("--ppo-iters", type=int, default=3, help="PPO leg: timed iterations")
    p.add_argument("--ppo-curve", type=int, default=PPO_CURVE_ITERS[-1],
                   help="PPO leg (N = 1): train to this iteration for return@iter (0: no curve)")
    p.add_argument("--apg-envs", type=int, default=2048)
    p.add_argument("--apg-horizon", type=int, default=128)
    p.add_argument("--apg-updates", type=int, default=3, help="APG leg: timed updates per solve derivative")
    p.add_argument("--cpu-steps", type=int, default=10000, help="CPU baseline: steps per env (C1: 10,000)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    p.add_argument("--no-extras", action="store_true", help="skip the secondary speed-test measurements")
    p.add_argument("--no-ppo", action="store_true", help="skip the PPO leg")
    p.add_argument("--no-apg", action="store_true", help="skip the APG leg")
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


def sync(device):
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


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


def timed_graph(fn, steps, warmup, dist):
    """As timed_launches, with the K launches captured as one hipGraph and replayed once (the launch-bound
    loop on the GPU's own queue: no per-launch host dispatch between the steps). W eager warmup launches
    and one untimed replay first. Returns (wall seconds, mean ms per step from HIP events around the
    replay), or None if the capture is refused."""
    from mjx_amd.ppo import graph_capture
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with graph_capture(g):
            for _ in range(steps):
                fn()
    except RuntimeError:
        torch.cuda.synchronize()
        return None
    g.replay()
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    g.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return wall, e0.elapsed_time(e1) / steps


def timed_steps(fn, args, dist):
    """The speed-test legs' timing: one graph replay of K steps (args.speedtest_launch == "graph"), else or
    if the capture is refused K eager launches."""
    if getattr(args, "speedtest_launch", "graph") == "graph":
        r = timed_graph(fn, args.steps, args.warmup, dist)
        if r is not None:
            return r
    return timed_launches(fn, args.steps, args.warmup, dist)


def max_over_ranks(x, dist, device="cuda"):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=torch.device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_traffic(B: int, key: str = "bytes_per_launch"):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (tools/profile_round.sh), used only
    when they were taken on the current kernel sources and this batch size."""
    from mjx_amd import _lib
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("src_hash") != _lib.source_hash() or int(t.get("envs", -1)) != B:
        return None
    return t.get(key)


def gather_over_ranks(x, dist, device="cuda") -> list:
    """[x of rank 0, x of rank 1, ...] (one value per rank), or [x] single-process."""
    if dist is None:
        return [x]
    t = torch.tensor([x], dtype=torch.float64, device=torch.device(device))
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def build_info() -> dict:
    """The native library this run loaded and the source hash it was built from (equal to the tree's:
    _lib.lib() refuses a stale library unless MJX355_LIB overrides it)."""
    from mjx_amd import _lib
    return _lib.build_info()


def free_gpu():
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


# ------------------------------------------------------------------------------------ CPU legs
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


def physical_cores(cpus=None) -> int:
    """Distinct (package, core) pairs among `cpus` (default: every online CPU), from sysfs topology;
    the logical count when the topology is unreadable."""
    cpus = sorted(cpus) if cpus is not None else list(range(os.cpu_count() or 1))
    seen = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            with open(base + "physical_package_id") as f:
                pkg = f.read().strip()
            with open(base + "core_id") as f:
                core = f.read().strip()
        except OSError:
            return len(cpus)
        seen.add((pkg, core))
    return len(seen)


def cpu_threads():
    """(threads, affinity CPUs): the CPUs in this process's affinity mask, capped by OMP_NUM_THREADS when
    set (the pool's CPU share per GPU, 16; os.cpu_count() shows the host)."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(len(aff), share) if share > 0 else len(aff)), aff


def cpu_baseline(steps: int, speedtest_envs: int = 2048):
    """BASELINE config C1 (mjx_humanoid_speed_test.py:140 HUMANOID row): humanoid.xml,
    1 env x `steps` carried steps from qpos0, ctrl = 0 and ctrl ~ U[-1,1] (seed 0); single thread,
    best of 3, then one env per thread on the threads this process may use, best of 3; warm-up run
    excluded. Beside it, the headline's own workload on the CPU (`speedtest`): the humanoid_mjx
    speed-test step from the same fresh states (qvel[0] = linspace(0, 1, speedtest_envs)), split over
    the threads, best of 3. MuJoCo is not importable on the box (plan B), so the timed CPU
    path is this build's serial C++ restatement (oracle/, kind "port") in its fp32 instantiation, the
    GPU's arithmetic type; ctypes releases the GIL, so the threads run in parallel."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from concurrent.futures import ThreadPoolExecutor

    import mjx_amd
    from oracle import Oracle
    m = mjx_amd.load_model("humanoid")
    threads, aff = cpu_threads()
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
    c1_s = time.perf_counter() - t_all

    # the headline workload on the CPU: 2048 fresh speed-test states, split over the threads
    mj = mjx_amd.load_model("humanoid_mjx")
    vel = np.linspace(0.0, 1.0, speedtest_envs)
    chunks = np.array_split(vel, threads)
    orcs = [Oracle(mj, use_float=True) for _ in range(threads)]
    orcs[0].speedtest(vel[:8])  # warm-up
    t1 = time.perf_counter()
    s1 = min((lambda t: (orcs[0].speedtest(vel[:256]), time.perf_counter() - t)[1])(time.perf_counter())
             for _ in range(3))
    best = None
    with ThreadPoolExecutor(threads) as ex:
        for _ in range(3):
            t = time.perf_counter()
            list(ex.map(lambda k: orcs[k].speedtest(chunks[k]), range(threads)))
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
    st_s = time.perf_counter() - t1
    return {"value": res["ctrlU"][1], "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model_name(), "host_cpus": os.cpu_count(), "host_physical_cores": physical_cores(),
            "affinity_cpus": len(aff), "affinity_physical_cores": physical_cores(aff),
            "single_thread": {k: v[0] for k, v in res.items()}, "all_cores": {k: v[1] for k, v in res.items()},
            "speedtest": {"steps_per_s": speedtest_envs / best, "single_thread_steps_per_s": 256 / s1,
                          "envs": speedtest_envs, "threads": threads},
            "sample": f"C1: humanoid.xml (Newton 100/50, Euler + eulerdamp), 1 env x {steps} carried steps "
                      f"from qpos0 per thread, ctrl U[-1,1] seed 0 (value) and ctrl 0; oracle/ C++ "
                      f"restatement, fp32; single thread best of 3, then {threads} threads x 1 env, best of 3 "
                      f"({c1_s:.1f} s). speedtest: humanoid_mjx speed-test step from the headline's "
                      f"{speedtest_envs} fresh states over {threads} threads, best of 3 ({st_s:.1f} s)"}


# ---------------------------------------------------------------------------------- GPU legs
def speedtest(args, dist, world, local):
    """The headline: K speed-test launches over B envs per GPU, with the kernel's roofline."""
    import mjx_amd
    from mjx_amd import flops as flops_mod
    from mjx_amd import mjx
    model = mjx_amd.load_model(args.model)
    sys_ = mjx.put_model(model)
    B = args.envs
    d = mjx.make_data(sys_, B, device=local)
    vel = torch.linspace(0.0, 1.0, B, device=f"cuda:{local}")
    out = torch.empty_like(vel)
    step = lambda: mjx.speedtest_step(sys_, d, vel, out)  # noqa: E731
    # the timed K steps as one graph replay (eager launches timed beside it, reported as such)
    ew, ek = timed_launches(step, args.steps, args.warmup, dist)
    gr = timed_graph(step, args.steps, args.warmup, dist) if getattr(args, "speedtest_launch", "graph") == "graph" else None
    launch = "graph" if gr is not None else "eager"
    wall, kern_ms = gr if gr is not None else (ew, ek)
    wall = max_over_ranks(wall, dist)
    ew = max_over_ranks(ew, dist)
    value = B * args.steps * world / wall
    # solver statistics of exactly these states (a forward pass from the same fresh state), for the
    # algorithmic FLOP count of one env-step (mjx_amd/flops.py, DESIGN.md "Roofline")
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
    line = {
        "metric": "humanoid env-steps/sec (whole node)",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": value / REF_DEVICE_STEPS_PER_S,
        "dtype": "f32",
        "data": "synthetic (speed-test states: qpos0, qvel[0]=linspace(0,1,B); PPO / APG legs: env resets drawn "
                "on the device, random-init networks)",
        "config": {"workload": f"{args.model}.xml speed-test step (fresh state per step), {B} envs per GPU",
                   "envs_per_gpu": B, "parallelism": f"env-sharded x{world}, no collective in the speed test",
                   "baseline_note": "vs_baseline divides by the README HUMANOID_MJX row (72,618 steps/s, batch 4096)"},
        "build": build_info(),
        "speedtest_launch": launch,
        "speedtest_eager_ms_per_step": ew / args.steps * 1e3,
        "speedtest_eager_kernel_ms": ek,
        "roofline": {"bound": "valu", "achieved": achieved_tflops, "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved_tflops / F32_PEAK_TFLOPS, "traffic": pmc_traffic(B),
                     "kernel": SPEEDTEST_KERNEL, "kernel_ms": kern_ms,
                     "flops_per_env_step": fl["total"],
                     "workload_mean_ncon_nefc_iter": [float(x) for x in wst[:3]],
                     "workload_mean_active_rows_per_hessian": float(wst[3]),
                     "hbm_algorithmic_bytes_per_launch": bytes_per_env * B,
                     "hbm_achieved_gbs": achieved_gbs, "hbm_frac": achieved_gbs / HBM_PEAK_GBS,
                     "note": "bound: VALU issue / dependency latency of one env per wave (SQ counters, "
                             "DESIGN.md 3), priced against the FP32 roof (vector peak = dense MFMA peak); "
                             "achieved = algorithmic FP32 FLOPs (mjx_amd/flops.py) / kernel time; traffic = "
                             "HBM bytes per launch from the committed FETCH_SIZE/WRITE_SIZE passes (profiles/)"},
    }
    return line, (model, sys_)


def speedtest_extras(args, model, sys_, local):
    """Trajectory mode, the fused PPO env step (with its roofline) and the README's batch of 4096."""
    from mjx_amd import flops as flops_mod
    from mjx_amd import mjx
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    B = args.envs
    ex = {}
    dev = f"cuda:{local}"
    # trajectory mode: carried state + random ctrl, full mjx.step with warm start
    dd = mjx.make_data(sys_, B, device=local)
    dd.set_option(0, 0)
    g = torch.Generator(device=dev).manual_seed(0)
    ctrl = torch.rand((B, sys_.nu), generator=g, device=dev) * 2 - 1
    tw, tk = timed_launches(lambda: mjx.step(sys_, dd, ctrl), args.steps, args.warmup, None)
    ex["trajectory_mode_steps_per_s"] = B * args.steps / tw
    dd.set_option(0, 1)
    mjx.step(sys_, dd, ctrl)
    st = dd.get("stats").cpu().numpy()
    ex["trajectory_mean_ncon_nefc_iter"] = [float(x) for x in st[:, :3].mean(0)]
    # fused PPO env step (physics + reward + obs + auto-reset in place) with random actions
    cfg = reference_ppo_config().env_config
    resolve_ids(model, cfg)
    env = HumanoidEnv(sys_, cfg, B, device=local, seed=1)
    env.reset()
    act = torch.rand((B, sys_.nu), generator=g, device=dev) * 2 - 1
    for _ in range(50):  # off the all-standing reset states: a rollout's mix of contacts and resets
        env.step(act)
    ew, ek = timed_launches(lambda: env.step(act), args.steps, args.warmup, None)
    ex["env_step_steps_per_s"] = B * args.steps / ew
    ex["env_step_kernel_ms"] = ek
    ex["env_step_hbm_gbs"] = ENV_STEP_BYTES * B / (ek * 1e-3) / 1e9
    # the env step's solver statistics (a forward pass from the states it steps) and the share of envs
    # that finish per step (their wave also runs the reset's forward pass)
    done = 0.0
    for _ in range(20):
        _, _, te, tr = env.step(act)
        done += float(torch.maximum(te, tr).sum())
    reset_frac = done / (20 * B)
    env.data.set_option(0, 1)
    mjx.forward(sys_, env.data)
    est = env.data.get("stats").double().mean(0).cpu().numpy()
    env.data.set_option(0, 0)
    fl = flops_mod.env_step_flops(model, float(est[0]), float(est[1]), float(est[2]), nact=float(est[3]),
                                  reset_frac=reset_frac)
    # where the launch's extra time goes: the same steps without the reset merge, and with the PPO
    # trainer's reset pool (resets computed in bulk before the rollout, merged by the step)
    env.enable_reset_pool(16)
    npool = torch.tensor([16], dtype=torch.int32, device=dev)
    env.fill_reset_pool(npool)
    _, ex["env_step_pool_kernel_ms"] = timed_launches(lambda: env.step(act), args.steps, args.warmup, None)
    env.enable_reset_pool(0)
    _, ex["env_step_noreset_kernel_ms"] = timed_launches(lambda: env.step(act, auto_reset=False), args.steps,
                                                         args.warmup, None)
    tf = fl["total"] * B / (ek * 1e-3) / 1e12
    ex["env_step_roofline"] = {
        "bound": "valu", "achieved": tf, "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / F32_PEAK_TFLOPS,
        "kernel": "step_kernel<mjl::Dims<27, 17, 22, 20, 48, 16>, 3, 2>", "kernel_ms": ek,
        "flops_per_env_step": fl["total"], "flops_by_stage": {k: v for k, v in fl.items() if k != "total"},
        "workload_mean_ncon_nefc_iter": [float(x) for x in est[:3]],
        "workload_mean_active_rows_per_hessian": float(est[3]), "reset_frac_per_step": reset_frac,
        "traffic": pmc_traffic(B, "env_step_bytes_per_launch"),
        "hbm_algorithmic_bytes_per_launch": ENV_STEP_BYTES * B,
        "hbm_frac": ENV_STEP_BYTES * B / (ek * 1e-3) / 1e9 / HBM_PEAK_GBS}
    del env, dd
    # the README's HUMANOID row (humanoid.xml, 159 candidate pairs, Newton 100/50, Euler + eulerdamp;
    # mjx_humanoid_speed_test.py:140, README.md:76: 6,176 steps/s) on the same speed test at B envs
    import mjx_amd
    mh = mjx_amd.load_model("humanoid")
    sh = mjx.put_model(mh)
    dh = mjx.make_data(sh, B, device=local)
    dh.set_option(0, 0)
    vh = torch.linspace(0.0, 1.0, B, device=dev)
    oh = torch.empty_like(vh)
    hw, hk = timed_steps(lambda: mjx.speedtest_step(sh, dh, vh, oh), args, None)
    ex["speedtest_humanoid_xml_steps_per_s"] = B * args.steps / hw
    ex["speedtest_humanoid_xml_kernel_ms"] = hk
    ex["speedtest_humanoid_xml_vs_readme"] = ex["speedtest_humanoid_xml_steps_per_s"] / REF_HUMANOID_XML_STEPS_PER_S
    del dh
    # ... and at the README's own batch of 4096 (mjx_humanoid_speed_test.py:140)
    dh = mjx.make_data(sh, 4096, device=local)
    dh.set_option(0, 0)
    vh = torch.linspace(0.0, 1.0, 4096, device=dev)
    oh = torch.empty_like(vh)
    hw, hk = timed_steps(lambda: mjx.speedtest_step(sh, dh, vh, oh), args, None)
    ex["speedtest_humanoid_xml_b4096_steps_per_s"] = 4096 * args.steps / hw
    ex["speedtest_humanoid_xml_b4096_kernel_ms"] = hk
    ex["speedtest_humanoid_xml_b4096_vs_readme"] = 4096 * args.steps / hw / REF_HUMANOID_XML_STEPS_PER_S
    del dh
    # the README's SPHERE row (mjx_humanoid_speed_test.py:29-40,142, README.md:78: 5,957,372 steps/s):
    # one free sphere, no floor, default options (Euler, dt 0.002), batch 4096, fresh state per step
    from mjx_amd import mjcf
    ms = mjcf.compile_xml_string(SPHERE_XML)
    ss = mjx.put_model(ms)
    dsp = mjx.make_data(ss, 4096, device=local)
    dsp.set_option(0, 0)
    vs = torch.linspace(0.0, 1.0, 4096, device=dev)
    osp = torch.empty_like(vs)
    sw, sk = timed_steps(lambda: mjx.speedtest_step(ss, dsp, vs, osp), args, None)
    ex["speedtest_sphere_b4096_steps_per_s"] = 4096 * args.steps / sw
    ex["speedtest_sphere_b4096_kernel_ms"] = sk
    ex["speedtest_sphere_b4096_vs_readme"] = 4096 * args.steps / sw / REF_SPHERE_STEPS_PER_S
    del dsp
    # the reference's own batch size for the README row
    d4 = mjx.make_data(sys_, 4096, device=local)
    v4 = torch.linspace(0.0, 1.0, 4096, device=dev)
    o4 = torch.empty_like(v4)
    w4, _ = timed_steps(lambda: mjx.speedtest_step(sys_, d4, v4, o4), args, None)
    ex["speedtest_b4096_steps_per_s"] = 4096 * args.steps / w4
    ex["speedtest_b4096_vs_readme"] = ex["speedtest_b4096_steps_per_s"] / REF_DEVICE_STEPS_PER_S
    return ex


def ppo_leg(tr, iters: int, warmup: int, dist, device, curve=()) -> dict:
    """`warmup` untimed PPO iterations (>= 2 on the GPU: the second captures the rollout and update
    hipGraphs), `iters` timed ones (barrier + sync on both sides, max over ranks), then untimed ones up
    to max(curve) for train_return_avg at the iterations in `curve` (return@iter, train_ppo.py:379-380)."""
    from mjx_amd.ppo import event_ms
    returns, it = {}, [0]

    def one():
        r = tr.iteration(it[0])
        if it[0] in curve:
            returns[it[0]] = r["train_return_avg"]
        it[0] += 1
        return r

    for _ in range(warmup):
        one()
    tr.allreduce_events = []
    tr.phase_events = []
    sync(device)
    barrier(dist)
    sync(device)
    t0 = time.perf_counter()
    res = [one() for _ in range(iters)]
    sync(device)
    barrier(dist)
    sync(device)
    wall = max_over_ranks(time.perf_counter() - t0, dist, device)
    ar = [event_ms(e) for e in tr.allreduce_events]
    tr.allreduce_events = None
    ar_ms = max_over_ranks(sum(ar) / len(ar) if ar else 0.0, dist, device)
    # phase split of the timed iterations (events on the trainer's stream), median, max over ranks
    phases, update_per_rank = {}, []
    if tr.phase_events:
        import statistics
        for name, (a, b) in (("rollout", (0, 1)), ("between", (1, 2)), ("update", (2, 3))):
            med = statistics.median(e[a].elapsed_time(e[b]) for e in tr.phase_events)
            phases[name] = max_over_ranks(med, dist, device)
            if name == "update":
                update_per_rank = gather_over_ranks(med, dist, device)
    tr.phase_events = None
    while curve and it[0] <= max(curve):
        one()
    world = 1 if dist is None else dist.get_world_size()
    env_steps = float(tr.env.num_envs * world * tr.cfg.rollout_length * iters)
    # RCCL collectives captured in the update's step graph (ppo.DP_CAPTURE) have no events of their own:
    # their count comes from the updater, their time is inside the update phase
    up = tr.updater
    captured = dist is not None and bool(getattr(up, "captured_last_run", False))
    n_ar = up.collectives_last_run if captured else len(ar) // max(1, iters)
    return {"env_steps_per_s": env_steps / wall, "ms_per_iter": wall / iters * 1e3, "iters": iters,
            "warmup": warmup, "envs_per_rank": tr.env.num_envs, "ranks": world,
            "allreduce_ms": None if captured else ar_ms, "allreduces_per_iter": n_ar, "allreduce_captured": captured,
            "train_return_avg": [r["train_return_avg"] for r in res], "return_at_iter": returns,
            "next_iteration": it[0], "phase_ms": phases, "update_rows": getattr(tr, "last_update_rows", 0),
            "update_ms_per_rank": update_per_rank, "dp_buckets": getattr(up, "dp_buckets", 0),
            "capture_fallback_reason": getattr(up, "capture_fallback_reason", None)}


def c5_fields(res: dict, world: int, backend: str, grad_numel: int) -> dict:
    """The C5 keys of the bench line (data-parallel PPO, BASELINE configs[4])."""
    return {"ppo_c5_env_steps_per_s": res["env_steps_per_s"], "ppo_c5_ms_per_iter": res["ms_per_iter"],
            "ppo_c5_envs_per_rank": res["envs_per_rank"], "ppo_c5_global_envs": res["envs_per_rank"] * world,
            "allreduce_ms_per_minibatch": res["allreduce_ms"], "allreduces_per_iteration": res["allreduces_per_iter"],
            "allreduce_captured_in_graph": res.get("allreduce_captured", False),
            "allreduce_bytes": 4 * grad_numel, "collective_backend": backend, "collective_ranks": world,
            "rccl_ranks": world if backend == "nccl" else 0,
            "ppo_c5_train_return_avg": res["train_return_avg"], "ppo_c5_phase_ms_per_rank": res["phase_ms"],
            # which data-parallel path ran (a SCALE record then says it): gradient buckets per minibatch
            # step, why the in-graph collective capture was given up (null: it ran captured, or was not
            # attempted on this backend), and every rank's update-phase median
            "dp_buckets": res.get("dp_buckets", 0), "dp_capture_fallback_reason": res.get("capture_fallback_reason"),
            "ppo_c5_update_ms_per_rank": res.get("update_ms_per_rank", [])}


def ppo_trainer(args, envs, dist, rank, local, eval_envs=0):
    import mjx_amd
    from mjx_amd import mjx, ppo
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    world = 1 if dist is None else dist.get_world_size()
    cfg = reference_ppo_config()
    cfg.num_envs, cfg.rollout_length = envs * world, 256
    m = mjx_amd.load_model(args.model)
    sys_ = mjx.put_model(m)
    ecfg = resolve_ids(m, cfg.env_config)
    env = HumanoidEnv(sys_, ecfg, envs, device=local, seed=cfg.seed * 7919 + rank)
    ev = HumanoidEnv(sys_, ecfg, eval_envs, device=local, seed=cfg.seed + 10000) if eval_envs else None
    return ppo.PPOTrainer(cfg, env, ev, device=f"cuda:{local}", dist=dist)


def grad_numel(tr) -> int:
    """Floats in one per-minibatch all-reduce (the updater's gradient buffer)."""
    return tr.updater.allreduce_numel()


def update_roofline(tr, res) -> dict:
    """The PPO update phase against the FP32 matrix roof: algorithmic FLOPs of both nets' forward +
    backward over every minibatch row of one update (mjx_amd/flops.py ppo_update_flops) / the update
    phase's event time on the trainer's stream."""
    from mjx_amd import flops as flops_mod
    cfg = tr.cfg
    fl = flops_mod.ppo_update_flops(tr.env.obs_dim, tr.env.act_dim, cfg.policy_hidden_layer_specs,
                                    cfg.value_hidden_layer_specs)
    ms = res["phase_ms"].get("update")
    if not ms:
        return {}
    rows = res["update_rows"]
    tf = fl["total"] * rows / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": tf, "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / F32_PEAK_TFLOPS,
            "update_ms": ms, "rows_per_update": rows, "flops_per_row": fl["total"],
            "flops_per_row_by_net": {k: v for k, v in fl.items() if k != "total"},
            "twin_update": tr.updater.twin is not None,
            "note": "both nets' fwd + bwd GEMMs (fp32 on the matrix cores through hipBLASLt) + elementwise; "
                    "achieved = algorithmic FLOPs / update-phase time (HIP events on the trainer's stream)"}


def policy_roofline(tr, local) -> dict:
    """The rollout's fused policy launch (mjl_policy_fwd: normalisation + MLP + Gaussian head, one
    launch per rollout step) over the trainer's envs: 100 launches captured in one hipGraph, HIP events
    around its replay."""
    from mjx_amd import flops as flops_mod
    from mjx_amd import ppo
    bf, B = tr._buf, tr.env.num_envs
    if bf is None or tr._pol_dims is None:
        return {}

    def launch():
        ppo.policy_fwd_native(bf["obs"][0], tr.rms.mean, tr.rms.var, 10.0, tr._pol_params, tr._pol_dims,
                              tr.policy.log_std, bf["eps"][0], bf["act"][0], bf["logp"][0])

    dev = f"cuda:{local}"
    launch()
    sync(dev)
    n = 100
    g = torch.cuda.CUDAGraph()
    from mjx_amd.ppo import graph_capture
    with graph_capture(g):
        for _ in range(n):
            launch()
    g.replay()
    sync(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    sync(dev)
    kms = e0.elapsed_time(e1) / n
    del g
    cfg = tr.cfg
    fl = flops_mod.policy_rollout_flops(tr.env.obs_dim, tr.env.act_dim, cfg.policy_hidden_layer_specs)
    tf = fl["total"] * B / (kms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": tf, "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / F32_PEAK_TFLOPS,
            "kernel": "policy_rollout_kernel", "kernel_ms": kms, "envs": B, "flops_per_env": fl["total"],
            "note": "fused rollout policy (v_mfma_f32_16x16x4_f32 tiles, 16 envs per workgroup); kernel_ms from "
                    "HIP events around a replayed hipGraph of 100 launches"}


class _IdentityComm:
    """A one-rank stand-in for torch.distributed: all_reduce is the identity (the per-rank C5 update
    below runs the data-parallel graphs with the collective taken out)."""

    @staticmethod
    def all_reduce(t, op=None, async_op=False):
        return None

    @staticmethod
    def get_world_size():
        return 1

    @staticmethod
    def get_backend():  # the updater captures its collectives for this stand-in as for RCCL
        return "identity"


def c5_rank_update(local, reps: int = 3) -> dict:
    """One rank's PPO update at BASELINE C5's per-rank shape on 8 GPUs (1024 envs x 256 steps, 4 epochs
    of 8,192-row minibatches = 128 minibatch steps) through PPOUpdater's data-parallel graphs with the
    all-reduce replaced by the identity (captured inside the update's graph, as the RCCL path captures
    it): the update's compute per rank (synthetic rollout data,
    random-init reference-size nets). The collective itself is measured at --gpus N > 1."""
    from mjx_amd import ppo
    from mjx_amd.config import reference_ppo_config
    dev = f"cuda:{local}"
    cfg = reference_ppo_config()
    cfg.minibatch_size = 8192
    g = torch.Generator().manual_seed(0)
    pol = ppo.GaussianPolicy(54, 21, cfg.policy_hidden_layer_specs, cfg.log_std_init, g).to(dev)
    val = ppo.ValueNet(54, cfg.value_hidden_layer_specs, g).to(dev)
    op, ov = ppo._adam(pol.parameters(), cfg.lr_policy), ppo._adam(val.parameters(), cfg.lr_value)
    up = ppo.PPOUpdater(pol, val, op, ov, cfg, _IdentityComm(), 1, use_graph=True)
    n = 1024 * 256
    gd = torch.Generator(device=dev).manual_seed(1)
    obs = torch.randn((n, 54), generator=gd, device=dev)
    act = torch.randn((n, 21), generator=gd, device=dev).clamp(-1, 1)
    logp, ret, adv = (torch.randn(n, generator=gd, device=dev) for _ in range(3))
    ts = []
    for r in range(reps + 2):
        idx = ppo.make_index_batches(n, cfg.minibatch_size, cfg.epochs, torch.Generator(device=dev).manual_seed(r), dev)
        sync(dev)
        t0 = time.perf_counter()
        up.run(obs, act, logp, ret, adv, idx)
        sync(dev)
        if r >= 2:
            ts.append(time.perf_counter() - t0)
    steps = int(idx.shape[0])
    out = {"ppo_c5_rank_update_ms": 1e3 * sorted(ts)[len(ts) // 2], "ppo_c5_rank_update_steps": steps,
           "ppo_c5_rank_update_twin": up.twin is not None,
           "ppo_c5_rank_update_note": "one rank of C5 on 8 GPUs: 1024 envs x 256 steps, 4 epochs x 32 minibatches "
                                      "of 8,192 rows, the data-parallel update as at N > 1 over RCCL (one graph per "
                                      "update, the collective captured inside) with an identity collective; "
                                      "median of 3 synced runs after 2 (capture)",
           "ppo_c5_rank_update_captured": bool(up.captured_last_run)}
    del up, pol, val, op, ov
    return out


def ppo_c3(args, local) -> dict:
    """C3: src/config.json PPO at 1024 envs on one GPU, throughput and return@iter (seed 42)."""
    tr = ppo_trainer(args, args.ppo_envs, None, 0, local, eval_envs=32)
    curve = tuple(i for i in PPO_CURVE_ITERS if i <= args.ppo_curve) if args.ppo_curve > 0 else ()
    t0 = time.perf_counter()
    res = ppo_leg(tr, args.ppo_iters, 2, None, f"cuda:{local}", curve)
    upd = update_roofline(tr, res)
    ev_it = res["next_iteration"] - 1
    eval_ret = tr.evaluate(ev_it) if curve else None
    out = {"ppo_c3_env_steps_per_s": res["env_steps_per_s"], "ppo_c3_ms_per_iter": res["ms_per_iter"],
           "ppo_c3_config": f"src/config.json: {args.ppo_envs} envs x 256 rollout x 4 epochs, minibatch 65536, "
                            f"seed 42; {res['iters']} timed iterations after 2 (graph capture)",
           "ppo_return_at_iter": {str(k): v for k, v in sorted(res["return_at_iter"].items())},
           "ppo_eval_return_at_iter": {str(ev_it): eval_ret} if eval_ret is not None else {},
           "ppo_curve_wall_s": time.perf_counter() - t0,
           "ppo_c3_phase_ms": res["phase_ms"], "ppo_update_roofline": upd,
           "ppo_update_tflops": upd.get("achieved"), "ppo_update_frac": upd.get("frac"),
           "ppo_policy_roofline": policy_roofline(tr, local)}
    from mjx_amd import tunable
    out["tuned_gemm_table"] = tunable.table_loaded()
    del tr
    free_gpu()
    out.update(c5_rank_update(local))
    free_gpu()
    return out


def apg_c4(args, local) -> dict:
    """C4: train_apg.py at 2048 envs x 128 horizon, CG 4/4, under the reference's solve derivative
    (unrolled: jax.grad through the iterations) and the implicit one; plus the replay VJP kernel's
    roofline from a reverse sweep over the last update's tape (HIP events around each launch)."""
    from mjx_amd import abi
    from mjx_amd import flops as flops_mod
    from mjx_amd import mjx
    from mjx_amd.apg import APGTrainer, HumanoidAPGEnv
    from mjx_amd.config import APGConfig, EnvConfig
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    from train_apg import apg_model
    out = {}
    dev = f"cuda:{local}"
    for vjp in ("unrolled", "implicit"):
        cfg = APGConfig()
        cfg.batch_size, cfg.horizon = args.apg_envs, args.apg_horizon
        m = apg_model(cfg, solver="cg")
        env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), cfg.batch_size, device=local, seed=cfg.seed)
        aenv = HumanoidAPGEnv(env, vjp)
        tr = APGTrainer(cfg, aenv, device=dev)
        tr.update(0)  # eager warm-up
        tr.update(1)  # captures the rollout + reverse sweep hipGraph
        sync(dev)
        t0 = time.perf_counter()
        res = [tr.update(i) for i in range(2, 2 + args.apg_updates)]
        sync(dev)
        wall = time.perf_counter() - t0
        key = "apg_c4" if vjp == "unrolled" else "apg_c4_implicit"
        out[f"{key}_env_steps_per_s"] = cfg.batch_size * cfg.horizon * len(res) / wall
        out[f"{key}_ms_per_update"] = wall / len(res) * 1e3
        out[f"{key}_returns"] = [r["return"] for r in res]
        out[f"{key}_nonfinite_envs"] = [r["nonfinite_envs"] for r in res]
        # the share of the batch whose cotangents overflowed and were cut from the gradient (unrolled
        # VJP under CG 4/4: DESIGN.md 3b), per timed update
        out[f"{key}_reverse_cut_frac"] = [r["reverse_nonfinite_envs"] / cfg.batch_size for r in res]
        if vjp == "implicit":  # the replay VJP kernel alone: one reverse sweep over the last update's tape
            B, H = cfg.batch_size, cfg.horizon
            act = torch.zeros((B, m.nu), device=dev)
            gq, gv = torch.zeros((B, m.nq), device=dev), torch.zeros((B, m.nv), device=dev)
            grew = torch.full((B,), -1.0 / B, device=dev)  # the reward's cotangent: every env runs the reverse
            nonf = torch.zeros(1, device=dev)
            gaux = torch.zeros((B, abi.AUX_DIM), device=dev)  # no per-call zero fill beside the kernel

            def sweep(events=None):
                for t in range(H - 1, -1, -1):
                    if events is not None:
                        events.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                        events[-1][0].record()
                    aenv.step_vjp_replay(t, act, gq, gv, None, grew, gaux, nonf)
                    if events is not None:
                        events[-1][1].record()
            sweep()  # warm-up
            sync(dev)
            # the H replay launches captured in one hipGraph, HIP events around its replay: the
            # launches run back to back as in the trainer's graph (per-launch event pairs around eager
            # launches also timed the gaps between them: 127 against rocprofv3's 101 us in round 3)
            g = torch.cuda.CUDAGraph()
            from mjx_amd.ppo import graph_capture
            with graph_capture(g):
                sweep()
            g.replay()
            sync(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            sync(dev)
            kms = e0.elapsed_time(e1) / H
            del g
            # the same H launches on the trainer's own workload: the last update's reward cotangents and
            # actions, the state cotangents chained step to step (the observation / policy terms the
            # trainer adds between launches left out), so the envs past termination take the kernel's
            # all-zero early exit as in training (the rocprofv3 average of the trainer)
            kms_tr = None
            if tr.last_reverse_inputs is not None:
                grew_all, acts = tr.last_reverse_inputs

                def sweep_tr():
                    q, v, ax = torch.zeros_like(gq), torch.zeros_like(gv), gaux
                    for t in range(H - 1, -1, -1):
                        q, v, _, _, ax = aenv.step_vjp_replay(t, acts[t], q, v, None, grew_all[t], ax, nonf)
                sweep_tr()
                sync(dev)
                g = torch.cuda.CUDAGraph()
                with graph_capture(g):
                    sweep_tr()
                g.replay()
                sync(dev)
                e0.record()
                g.replay()
                e1.record()
                sync(dev)
                kms_tr = e0.elapsed_time(e1) / H
                del g
            # the rollout's solver statistics (the same policy from fresh resets; CG reports no active-row
            # count, so the implicit Hessian is counted over all rows)
            env.data.set_option(0, 1)
            env.reset()
            acc = torch.zeros(3, dtype=torch.float64, device=dev)
            with torch.no_grad():
                for _ in range(H):
                    env.step(tr.policy(aenv.qpos_qvel()), auto_reset=False)
                    acc += env.data.get("stats")[:, :3].double().mean(0)
            s = (acc / H).cpu().numpy()
            fl = flops_mod.vjp_replay_flops(m, float(s[0]), float(s[1]), float(s[2]))
            tf = fl["total"] * B / (kms * 1e-3) / 1e12
            out["apg_vjp_roofline"] = {
                "bound": "valu", "achieved": tf, "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": tf / F32_PEAK_TFLOPS, "kernel": "vjp_kernel<mjl::Dims<27, 17, 22, 20, 4, 4>, true, 2, true>",
                "kernel_ms": kms, "launches_timed": H, "timing": "one captured sweep of H replay launches",
                "kernel_ms_every_env_active": kms, "kernel_ms_trainer_workload": kms_tr,
                "flops_per_env_step": fl["total"],
                "flops_by_stage": {k: v for k, v in fl.items() if k != "total"},
                "workload_mean_ncon_nefc_iter": [float(x) for x in s[:3]],
                "traffic": pmc_traffic(B, "vjp_bytes_per_launch")}
        del tr, aenv, env
        free_gpu()
    out["apg_c4_config"] = (f"train_apg.py: {args.apg_envs} envs x {args.apg_horizon} horizon, CG 4/4, hidden 32x2, "
                            f"lr 5e-5, clip 0.3; {args.apg_updates} timed updates after 2 (graph capture); "
                            f"apg_c4 = unrolled VJP (jax.grad semantics), apg_c4_implicit = implicit VJP; observation "
                            f"statistics: {'in-loss observations only (not the reference rule)' if APGConfig().rms_in_loss_only else 'every rollout observation (train_apg.py:290-292)'}")
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launch the N ranks as a child process (nothing here has touched the GPU yet) and pass
        # its status through; rank 0 of the child prints the JSON line
        import subprocess
        sys.exit(subprocess.run(launch_cmd(sys.argv[1:], args.gpus, free_port())).returncode)
    dist, rank, world, local = dist_setup(args)
    backend = dist.get_backend() if dist is not None else None

    if args.workload == "ppo":  # the PPO leg alone as the headline (C3 at N = 1, C5 at N > 1)
        tr = ppo_trainer(args, args.envs, dist, rank, local)
        res = ppo_leg(tr, args.steps, max(2, args.warmup), dist, f"cuda:{local}")
        line = {"metric": "humanoid PPO env-steps/sec (whole node)", "value": res["env_steps_per_s"],
                "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": max(2, args.warmup),
                "ms_per_step": res["ms_per_iter"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "f32", "data": "synthetic (env resets drawn on the device; random-init policy / value nets)",
                "config": {"workload": f"PPO src/config.json: {args.envs} envs per GPU x 256 rollout x 4 epochs, "
                                       f"global minibatch 65536", "envs_per_gpu": args.envs},
                "step": "one PPO iteration (rollout + GAE + updates), synced", "roofline": None, "cpu_baseline": None,
                "rehearsal": os.environ.get("MJL_BENCH_REHEARSAL") == "1", "build": build_info()}
        if dist is not None:
            line.update(c5_fields(res, world, backend, grad_numel(tr)))
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    line, (model, sys_) = speedtest(args, dist, world, local)
    legs = {}
    full = args.workload == "all"
    if world == 1:
        if full and not args.no_extras:
            legs.update(speedtest_extras(args, model, sys_, local))
        if full and not args.no_ppo:
            legs.update(ppo_c3(args, local))
        if full and not args.no_apg:
            legs.update(apg_c4(args, local))
    elif full and not args.no_ppo:  # C5 on every rank: the one collective of the path, timed
        tr = ppo_trainer(args, args.ppo_envs, dist, rank, local)
        res = ppo_leg(tr, args.ppo_iters, 2, dist, f"cuda:{local}")
        legs.update(c5_fields(res, world, backend, grad_numel(tr)))
        legs["ppo_c5_config"] = (f"src/config.json PPO: {args.ppo_envs} envs per rank x 256 rollout x 4 epochs, "
                                 f"global minibatch 65536 ({65536 // world} rows per rank); {res['iters']} timed "
                                 f"iterations after 2 (graph capture)")
        del tr
        free_gpu()
    if rank == 0:
        line["cpu_baseline"] = cpu_baseline(args.cpu_steps, args.envs) if world == 1 and not args.no_cpu else None
        if line["cpu_baseline"] is not None:
            line["cpu_speedtest_steps_per_s"] = line["cpu_baseline"]["speedtest"]["steps_per_s"]
        line.update(legs)
        if os.environ.get("MJL_BENCH_REHEARSAL") == "1":
            line["rehearsal"] = True
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""bench.py's launch contract on CPU: defaults per workload, the self-launch command for --gpus N,
and the refusal of a world size that disagrees with --gpus (--gpus was ignored)."""
import importlib.util
import json
import os
import socket

import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_defaults(bench):
    a = bench.parse([])
    assert (a.gpus, a.workload, a.steps, a.warmup, a.envs) == (1, "all", 50, 5, 2048)
    assert (a.ppo_envs, a.ppo_iters, a.apg_envs, a.apg_horizon) == (1024, 3, 2048, 128)  # C3 / C4
    p = bench.parse(["--workload", "ppo"])
    assert (p.steps, p.warmup, p.envs) == (3, 2, 1024)  # C5: 1024 envs per GPU, 8192 over 8


def test_self_launch_command(bench):
    cmd = bench.launch_cmd(["--gpus", "4", "--steps", "7"], 4, 29500)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"]
    assert os.path.samefile(cmd[cmd.index("--master-port") + 2], os.path.join(ROOT, "bench.py"))


def test_world_size_must_match_gpus(bench, monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit):
        bench.dist_setup(bench.parse(["--gpus", "1"]))
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit):
        bench.dist_setup(bench.parse(["--gpus", "8"]))


def test_cpu_baseline_protocol(bench):
    r = bench.cpu_baseline(50, speedtest_envs=64)
    assert r["kind"] == "port" and r["unit"] == "env-steps/s" and r["cores"] >= 1
    assert r["value"] == r["all_cores"]["ctrlU"] > 0 and set(r["single_thread"]) == {"ctrl0", "ctrlU"}
    assert r["host_cpus"] == os.cpu_count() and r["cpu_model"]
    assert 1 <= r["host_physical_cores"] <= r["host_cpus"] and 1 <= r["affinity_physical_cores"] <= r["affinity_cpus"]
    # the headline's own workload on the CPU: the speed-test states
    assert r["speedtest"]["envs"] == 64 and r["speedtest"]["steps_per_s"] > 0


def _load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _c5_worker(rank, port, out):
    """One rank of the N > 1 line's C5 leg over gloo: PPO with a CPU stand-in env, the per-minibatch
    all-reduce timed, the line's C5 keys built by bench.c5_fields."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=2)
    from test_ppo import PointEnv, small_cfg
    from mjx_amd import ppo
    bench = _load_bench()
    tr = ppo.PPOTrainer(small_cfg(), PointEnv(8, 100 + rank), None, device="cpu", dist=tdist)
    res = bench.ppo_leg(tr, 2, 1, tdist, "cpu")
    if rank == 0:
        line = bench.c5_fields(res, 2, tdist.get_backend(), bench.grad_numel(tr))
        with open(out, "w") as f:
            json.dump(line, f)
    tdist.destroy_process_group()


def test_c5_line_over_gloo_world_size_2(tmp_path):
    """the command the driver runs at N > 1 must time the one collective north_star
    names. Two gloo ranks run bench.ppo_leg and build the line's C5 keys."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "c5.json")
    mp.spawn(_c5_worker, args=(port, out), nprocs=2, join=True)
    line = json.load(open(out))
    for k in ("ppo_c5_env_steps_per_s", "ppo_c5_ms_per_iter", "allreduce_ms_per_minibatch", "rccl_ranks",
              "collective_ranks", "allreduces_per_iteration", "allreduce_bytes"):
        assert k in line, k
    assert line["collective_ranks"] == 2 and line["collective_backend"] == "gloo" and line["rccl_ranks"] == 0
    # small_cfg: 8 envs x 8 steps per rank, 16 rows per rank of each 32-row minibatch, 2 epochs
    assert line["allreduces_per_iteration"] == 2 * (8 * 8 // 16)
    assert line["ppo_c5_env_steps_per_s"] > 0 and line["allreduce_ms_per_minibatch"] > 0
    assert line["ppo_c5_global_envs"] == 16
    # which data-parallel path ran: one bucket (eager, the CPU stand-in nets take the
    # per-net path), no capture over gloo, so no fallback reason; the per-rank update list is filled
    # from the update-phase events on the GPU (none on the CPU)
    assert line["dp_buckets"] == 1 and line["dp_capture_fallback_reason"] is None
    assert line["allreduce_captured_in_graph"] is False and isinstance(line["ppo_c5_update_ms_per_rank"], list)

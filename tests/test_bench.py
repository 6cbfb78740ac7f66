"""bench.py's launch contract on CPU: defaults per workload, the self-launch command for --gpus N,
and the refusal of a world size that disagrees with --gpus (--gpus was ignored)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_defaults(bench):
    a = bench.parse([])
    assert (a.gpus, a.workload, a.steps, a.warmup, a.envs) == (1, "speedtest", 50, 5, 2048)
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
    r = bench.cpu_baseline(50)
    assert r["kind"] == "port" and r["unit"] == "env-steps/s" and r["cores"] >= 1
    assert r["value"] == r["all_cores"]["ctrlU"] > 0 and set(r["single_thread"]) == {"ctrl0", "ctrlU"}
    assert r["host_cpus"] == os.cpu_count() and r["cpu_model"]

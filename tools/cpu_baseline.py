"""BASELINE config C1 on the GPU box's host CPU, Plan B: MuJoCo is not importable
here, so the timed CPU path is this build's own serial C++ restatement (oracle/, fp64), labelled as
such. Protocol: 1 env x 10,000 steps from qpos0, ctrl = 0 and ctrl ~ U[-1,1] (seed 0), best of 3;
then one env per thread on `threads` host threads (the box's CPU share for one GPU is 16).
Prints one JSON line."""
import json
import os
import platform
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import mjx_amd  # noqa: E402
from oracle import Oracle  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def run(m, ctrl, steps):
    o = Oracle(m)
    s = o.new_state()
    t = time.perf_counter()
    o.rollout(s, ctrl[:steps])
    return time.perf_counter() - t


def main(steps=10000, threads=16):
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = min(threads, avail)
    out = {"kind": "port (oracle/ C++ restatement, fp64; MuJoCo not importable)", "cpu_model": cpu_model(),
           "os_cpu_count": os.cpu_count(), "affinity_cpus": avail, "threads": threads, "steps_per_env": steps}
    rng = np.random.default_rng(0)
    for name in ("humanoid_mjx", "humanoid"):
        m = mjx_amd.load_model(name)
        for cname, ctrl in (("ctrl0", np.zeros((steps, m.nu))), ("ctrlU", rng.uniform(-1, 1, (steps, m.nu)))):
            best = min(run(m, ctrl, steps) for _ in range(3))
            t = time.perf_counter()
            with ThreadPoolExecutor(threads) as ex:
                list(ex.map(lambda _: run(m, ctrl, steps), range(threads)))
            dt = time.perf_counter() - t
            out[f"{name}_{cname}"] = {"single_thread_steps_per_s": steps / best,
                                      "all_threads_steps_per_s": threads * steps / dt}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

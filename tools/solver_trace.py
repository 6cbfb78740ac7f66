"""Trace one env's truncated solves on the fp64 oracle (DESIGN.md "Truncated solves").

    python tools/solver_trace.py [cg|newton] ITER LS ENV FROM_STEP [--solver-qacc]

Runs the census controls of tests/test_solver_truncation.py (seeded resets, AR(1) smooth random
controls) for envs 0..ENV, and from step FROM_STEP of env ENV prints every solve: the warm-start
choice, each iteration's zoom line search beside a brute-force scan of alpha, the cost and scaled
gradient after each iteration, and the integrator's input next to the solver's qacc.
--solver-qacc feeds the integrator M qacc instead (the counterfactual)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mujoco-mjx-lab_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import mjx_amd  # noqa: E402
import oracle as O  # noqa: E402
from mjx_amd import abi, mjcf  # noqa: E402
from mjx_amd.config import reference_ppo_config  # noqa: E402
from mjx_amd.envs import obs_size, resolve_ids  # noqa: E402

solver, it, ls, pick, start = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
extra = O.DIAG_SOLVER_QACC if "--solver-qacc" in sys.argv else 0
m = mjx_amd.load_model("humanoid_mjx")
m.solver = mjcf.SOLVER_CG if solver == "cg" else mjcf.SOLVER_NEWTON
m.iterations, m.ls_iterations = it, ls
c = abi.env_config_c(resolve_ids(m, reference_ppo_config().env_config), m, obs_size(m.nq, m.nv))
o = O.Oracle(m)
rng = np.random.default_rng(0)
nd = m.nq - 7 + m.nv + 2
O.set_diag(extra)
for e in range(pick + 1):
    s, aux, _ = o.env_reset(c, rng.uniform(0, 1, nd))
    u = np.zeros(m.nu)
    for t in range(128):
        u = 0.9 * u + 0.45 * rng.uniform(-1, 1, m.nu)
        on = e == pick and t >= start
        O.set_diag(extra | (O.DIAG_TRACE if on else 0))
        if on:
            print(f"--- step {t}", file=sys.stderr, flush=True)
        s, aux, *_ = o.env_step(c, s, aux, np.clip(u, -1, 1))
        v = np.abs(np.array(s.qvel[:m.nv]))
        if on:
            print(f"step {t}: max|qvel| {v.max():.4g} at dof {v.argmax()}", file=sys.stderr, flush=True)
        if not np.isfinite(v.max()) or v.max() > 1e3:
            break
O.set_diag(0)

"""Diagnostic: per-phase cycle shares of the env-step VJP kernel from the MJL_TIMING build (run with
MJX355_LIB pointing at it). Slots: 0 start, 1 forward recompute (REPLAY=1: the tape-slot load) done,
2..13 after each reverse pass. REPLAY=1: the APG replay VJP over a recorded 2048 x 128 CG 4/4 tape
(mjl_env_step_vjp_replay, one slot), else the recomputing mjl_env_step_vjp after 20 random steps."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import _lib, mjx  # noqa: E402
from mjx_amd.config import EnvConfig  # noqa: E402
from mjx_amd.envs import HumanoidEnv, resolve_ids  # noqa: E402

names = ["forward recompute / slot load", "adj env + integrate", "adj solver rows", "adj contact jac",
         "adj collision", "adj geom frames", "adj forces", "adj rne", "adj mass", "adj crb", "adj cinert",
         "adj cdof", "adj kinematics"]
L = _lib.lib()
L.mjl_debug_set_stamps.argtypes = [C.c_void_p]
B = 2048
buf = torch.zeros((B, 48), dtype=torch.int64, device="cuda")  # the kernels' stamp stride is 48 per env
if os.environ.get("REPLAY") == "1":
    from mjx_amd.apg import APGTrainer, HumanoidAPGEnv
    from mjx_amd.config import APGConfig
    from train_apg import apg_model
    cfg = APGConfig()
    cfg.batch_size, cfg.horizon = B, 128
    ma = apg_model(cfg, solver="cg")
    env = HumanoidEnv(mjx.put_model(ma), resolve_ids(ma, EnvConfig()), B, seed=cfg.seed)
    aenv = HumanoidAPGEnv(env, os.environ.get("VJP", "implicit"))
    tr = APGTrainer(cfg, aenv, device="cuda", use_graph=False)
    tr.update(0)  # records the tape
    act = torch.zeros((B, ma.nu), device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    gq, gv = torch.randn((B, ma.nq), generator=g, device="cuda"), torch.randn((B, ma.nv), generator=g, device="cuda")
    grew = torch.full((B,), -1.0 / B, device="cuda")
    nonf = torch.zeros(1, device="cuda")
    gws = torch.zeros((B, ma.nv), device="cuda") if getattr(aenv, "vjp_carries_ws", False) else None
    t = int(os.environ.get("SLOT", "64"))
    aenv.step_vjp_replay(t, act, gq, gv, gws, grew, None, nonf)
    torch.cuda.synchronize()
    L.mjl_debug_set_stamps(C.c_void_p(buf.data_ptr()))
    aenv.step_vjp_replay(t, act, gq, gv, gws, grew, None, nonf)
else:
    m = mjx_amd.load_model("humanoid_mjx")
    if os.environ.get("SOLVER") == "cg44":  # train_apg.py's override
        from mjx_amd import mjcf
        m.solver, m.iterations, m.ls_iterations = mjcf.SOLVER_CG, 4, 4
    env = HumanoidEnv(mjx.put_model(m), resolve_ids(m, EnvConfig()), B, seed=3)
    if os.environ.get("VJP") == "unrolled":
        from mjx_amd import abi
        env.data.set_option(abi.OPT_VJP_UNROLLED, 1)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(20):
        env.step(torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1, auto_reset=False)
    act = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
    gq, gv, gr = torch.randn((B, m.nq), device="cuda"), torch.randn((B, m.nv), device="cuda"), torch.randn(B, device="cuda")
    for _ in range(2):
        env.step_vjp(act, gq, gv, gr)
    torch.cuda.synchronize()
    L.mjl_debug_set_stamps(C.c_void_p(buf.data_ptr()))
    env.step_vjp(act, gq, gv, gr)
torch.cuda.synchronize()
L.mjl_debug_set_stamps(C.c_void_p(0))
s = buf.cpu().numpy().astype(np.float64)
ok = s[:, 13] > 0  # envs that ran the reverse (all-zero cotangents return early)
d = np.diff(s[ok][:, :14], axis=1)
tot = d.sum(1)
print(f"VJP ({'replay' if os.environ.get('REPLAY') == '1' else 'recompute'}): envs timed {ok.sum()}; "
      f"mean cycles/env {tot.mean():.0f}; p50 / p99 / max {np.percentile(tot, 50):.0f} / "
      f"{np.percentile(tot, 99):.0f} / {tot.max():.0f}")
for i, n in enumerate(names):
    print(f"   {n:30s} {d[:, i].mean():9.0f}  {100 * d[:, i].mean() / tot.mean():5.1f}%")
subs = {20: "kin: scom + joint frames", 21: "kin: joint gather", 22: "kin: xipos + local transforms",
        23: "kin: tree pass reverse", 24: "kin: local transforms reverse", 25: "rne: bias + cfrc-bar",
        26: "rne: cvel/cacc recompute", 27: "rne: cfrc reverse", 28: "rne: tree reverse", 29: "rne: local terms",
        30: "mass: f + M-bar loops", 31: "mass: crb-bar"}
for i, n in subs.items():
    print(f"      {n:30s} {s[ok][:, i].mean():9.0f}")
if (s[ok][:, 14] > 0).all():
    print(f"      {'env: reward / obs adjoint':30s} {(s[ok][:, 14] - s[ok][:, 1]).mean():9.0f}")

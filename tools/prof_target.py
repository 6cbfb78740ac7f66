"""Minimal launch loops for rocprofv3 (kernel trace / counter passes), one kernel family per mode:
  speedtest     mjl_speedtest_step, B fresh speed-test states (the headline)
  envstep       mjl_env_step with in-place auto-reset, random actions, after 50 warm steps
  envstep_pool  the same with the trainer's reset pool (16 slots, refilled every 64 steps)
  envstep_nr    the same steps without auto-reset (the physics + env post only)
  vjp           mjl_env_step_vjp_replay over every slot of a 2048 x 128 CG 4/4 implicit APG tape
  policy        mjl_policy_fwd, the PPO rollout policy (obs 54 -> 256 x 3 -> 21) on B envs
  apgmlp        mjl_small_mlp_fwd + mjl_small_mlp_bwd_input, the APG policy (55 -> 32 x 2 -> 21) on B rows
  apgstep       the APG rollout's physics (CG 4/4 model) through mjl_env_step without reset, random
                actions, against the record kernel of the `vjp` mode (rows in LDS vs in global memory;
                PROF_FORCE_GLOBAL=1 keeps them in global memory as the record does)
  recab         the APG record and the env step without reset on the same states and actions
python tools/prof_target.py MODE [B] [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

import mjx_amd  # noqa: E402
from mjx_amd import mjx  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "speedtest"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
m = mjx_amd.load_model("humanoid_mjx")
sys_ = mjx.put_model(m)
if mode == "speedtest":
    d = mjx.make_data(sys_, B)
    vel = torch.linspace(0, 1, B, device="cuda")
    out = torch.empty_like(vel)
    for _ in range(n):
        mjx.speedtest_step(sys_, d, vel, out)
elif mode.startswith("envstep"):
    from mjx_amd.config import reference_ppo_config
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    env = HumanoidEnv(sys_, cfg, B, seed=1)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    act = torch.rand((B, m.nu), generator=g, device="cuda") * 2 - 1
    pool = mode == "envstep_pool"
    if pool:
        env.enable_reset_pool(16)
        npool = torch.tensor([16], dtype=torch.int32, device="cuda")
    for _ in range(50):
        env.step(act)
    for i in range(n):
        if pool and i % 64 == 0:
            env.fill_reset_pool(npool)
        env.step(act, auto_reset=mode != "envstep_nr")
elif mode == "vjp":
    from mjx_amd.apg import APGTrainer, HumanoidAPGEnv
    from mjx_amd.config import APGConfig, EnvConfig
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
    from train_apg import apg_model
    cfg = APGConfig()
    cfg.batch_size, cfg.horizon = B, 128
    ma = apg_model(cfg, solver="cg")
    env = HumanoidEnv(mjx.put_model(ma), resolve_ids(ma, EnvConfig()), B, seed=cfg.seed)
    aenv = HumanoidAPGEnv(env, "implicit")
    tr = APGTrainer(cfg, aenv, device="cuda", use_graph=False)
    tr.update(0)  # records the tape (eager)
    act = torch.zeros((B, ma.nu), device="cuda")
    gq, gv = torch.zeros((B, ma.nq), device="cuda"), torch.zeros((B, ma.nv), device="cuda")
    grew = torch.full((B,), -1.0 / B, device="cuda")
    nonf = torch.zeros(1, device="cuda")
    for _ in range(max(1, n // cfg.horizon)):
        for t in range(cfg.horizon - 1, -1, -1):
            aenv.step_vjp_replay(t, act, gq, gv, None, grew, None, nonf)
elif mode == "policy":
    from mjx_amd import ppo
    g = torch.Generator().manual_seed(0)
    pol = ppo.GaussianPolicy(54, 21, [(256, "tanh")] * 3, 0.0, g).cuda()
    gd = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn((B, 54), generator=gd, device="cuda")
    rms = ppo.RunningMeanStd(54, "cuda")
    eps = torch.randn((B, 21), generator=gd, device="cuda")
    dims, params = ppo.policy_fused_dims(pol), ppo.pack_policy_params(pol)
    act, lp = torch.empty((B, 21), device="cuda"), torch.empty(B, device="cuda")
    for _ in range(n):
        ppo.policy_fwd_native(x, rms.mean, rms.var, 10.0, params, dims, pol.log_std, eps, act, lp)
elif mode == "apgstep":
    from mjx_amd.config import APGConfig, EnvConfig
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
    from train_apg import apg_model
    cfg = APGConfig()
    ma = apg_model(cfg, solver="cg")
    env = HumanoidEnv(mjx.put_model(ma), resolve_ids(ma, EnvConfig()), B, seed=cfg.seed)
    if os.environ.get("PROF_FORCE_GLOBAL") == "1":  # rows in the global slab, as the record kernel keeps them
        from mjx_amd import abi
        env.data.set_option(abi.OPT_FORCE_GLOBAL_ROWS, 1)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for i in range(n):
        if i % 128 == 0:
            env.reset()
        act = (torch.rand((B, ma.nu), generator=g, device="cuda") * 2 - 1) * 0.3
        env.step(act, auto_reset=False)
elif mode == "recab":  # the record and the env step (no reset) on the same states and actions, alternating
    from mjx_amd.apg import HumanoidAPGEnv
    from mjx_amd.config import APGConfig, EnvConfig
    from mjx_amd.envs import HumanoidEnv, resolve_ids
    sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
    from train_apg import apg_model
    cfg = APGConfig()
    ma = apg_model(cfg, solver="cg")
    env = HumanoidEnv(mjx.put_model(ma), resolve_ids(ma, EnvConfig()), B, seed=cfg.seed)
    aenv = HumanoidAPGEnv(env, "implicit")
    aenv.enable_vjp_tape(128)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for i in range(n):
        act = (torch.rand((B, ma.nu), generator=g, device="cuda") * 2 - 1) * 0.3
        st = env.get_state()
        env.step(act, auto_reset=False)
        env.set_state(st)
        aenv.step_record(i % 128, act)
elif mode == "apgmlp":
    from mjx_amd import apg, ppo
    pol = ppo.APGPolicy(55, 21, 32, 2, None, torch.Generator().manual_seed(0)).cuda()
    nat = apg.NativeAPGPolicy(pol)
    gd = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn((B, 55), generator=gd, device="cuda")
    ga = torch.randn((B, 21), generator=gd, device="cuda")
    ys = [torch.empty((B, w), device="cuda") for w in nat.widths]
    for _ in range(n):
        nat.forward(x, ys)
        nat.backward_input(ga, ys)
torch.cuda.synchronize()
print("done", mode, B, n)

"""qpos-history dump of a policy rollout, for offline rendering (reference src/rendering.py:57-195).

The reference scans `duration / dt` env steps of a deterministic policy on one env, resetting to the
rollout's own initial state whenever the env is done, collects `qpos` after every step and renders
the history with mujoco.Renderer (every `1 / (fps dt)`-th frame). Rendering is out of scope here
(no mujoco / GL on the box); the history is written as an `.npz` that any MuJoCo install renders
offline with the reference's own loop (`mj_data.qpos[:] = qpos[i]; mj_forward; renderer.render()`):

    qpos [T, nq]   post-step (post-reset-merge) qpos, as the reference's scan returns it
    act  [T, nu]   the clipped actions that produced it (replayable through the env)
    dt, fps, stride, duration, model, camera_name
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import numpy as np
import torch


@torch.no_grad()
def rollout_qpos_history(env, policy_fn: Callable[[torch.Tensor], torch.Tensor], duration: float,
                         reset_keys: Optional[torch.Tensor] = None):
    """render_policy_rollout's scan (src/rendering.py:102-180) on a HumanoidEnv with B envs
    (B = 1 in the reference): action = clip(policy_fn(obs), -1, 1); step without the auto-reset;
    done envs go back to the rollout's initial state and obs. Returns (qpos [T, B, nq], act [T, B, nu])
    as numpy arrays. `reset_keys` [B, 2]: draw the initial state from jax.random keys
    (single_reset(key), src/rendering.py:91-93)."""
    dt = float(env.sys.m.timestep)
    steps = int(duration / dt)
    if reset_keys is not None:
        env.set_reset_keys(reset_keys.to(torch.int32).contiguous())
    obs0 = env.reset().clone()
    if reset_keys is not None:
        env.set_reset_keys(None)
    st0 = env.get_state().clone()
    B = env.num_envs
    qpos = torch.empty((steps, B, env.sys.nq), device=obs0.device)
    act = torch.empty((steps, B, env.act_dim), device=obs0.device)
    obs = obs0
    for t in range(steps):
        a = torch.clamp(policy_fn(obs), -1.0, 1.0)
        act[t] = a
        o, _, te, tr = env.step(a, auto_reset=False)
        done = torch.maximum(te, tr) > 0.5
        env.set_state(torch.where(done[:, None], st0, env.get_state()))
        obs = torch.where(done[:, None], obs0, o).clone()
        qpos[t] = env.data.get("qpos")
    return qpos.cpu().numpy(), act.cpu().numpy()


def save_qpos_history(path: str, qpos: np.ndarray, act: np.ndarray, dt: float, fps: int = 60,
                      model: str = "", camera_name: str = "side_view") -> str:
    """Write the history (one env: [T, nq]) next to where the reference writes its video
    (training_dir/videos/<prefix>_<step+1:06d>.npz instead of .mp4, training_utils.py:191-195)."""
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    stride = max(1, int(1.0 / (fps * dt)))
    np.savez(path, qpos=qpos, act=act, dt=dt, fps=fps, stride=stride, duration=qpos.shape[0] * dt,
             model=model, camera_name=camera_name)
    return path


def load_qpos_history(path: str) -> dict:
    """Read a dump back (plain arrays, no pickle)."""
    with np.load(path, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}

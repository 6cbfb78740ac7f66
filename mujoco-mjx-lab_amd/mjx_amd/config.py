"""Configuration objects read with the same keys as the reference.

Field names and defaults follow reference `src/config.py` (EnvConfig :29-66, APGConfig :69-86,
PPOConfig :89-172). `PPOConfig.from_json` honours the same JSON layout as reference
`src/config.json` ("env", "ppo", "symmetry.flip_params" sections; unknown keys ignored, as in
`src/config.py:146-170`). `reference_ppo_config()` reproduces the values of `src/config.json`
without needing the file (the GPU box has no copy of the reference).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field, fields
from typing import List, Optional, Tuple

_RIGHT_ACT = [3, 4, 5, 6, 7, 8, 15, 16, 17]
_LEFT_ACT = [9, 10, 11, 12, 13, 14, 18, 19, 20]
_RIGHT_OBS = [7, 8, 9, 10, 11, 12, 19, 20, 21, 34, 35, 36, 37, 38, 39, 46, 47, 48]
_LEFT_OBS = [13, 14, 15, 16, 17, 18, 22, 23, 24, 40, 41, 42, 43, 44, 45, 49, 50, 51]


@dataclass
class EnvConfig:
    progress_weight: float = 1.0
    electricity_cost: float = 0.026
    stall_torque_cost: float = 0.0000023
    joints_at_limit_cost: float = 5.0
    posture_penalty_weight: float = 0.60
    tall_height_threshold: float = 0.7
    tall_bonus_weight: float = 0.0
    target_threshold: float = 0.15
    target_dist: float = 2.0
    stop_frames: int = 1
    stance_time_reward_weight: float = 0.0
    random_joint_noise: float = 0.01
    random_vel_noise: float = 0.01
    initial_velocity_max: float = 0.5
    terminate_height: float = 0.7
    terminate_reward: float = 0.0
    max_episode_steps: int = 1000
    random_flip: bool = False
    joint_limit_force_threshold: float = 6.5
    pelvis_body_id: int = -1
    head_body_id: int = -1
    touch_sensor_right_id: int = -1
    touch_sensor_left_id: int = -1
    flip_action_right: List[int] = field(default_factory=lambda: list(_RIGHT_ACT))
    flip_action_left: List[int] = field(default_factory=lambda: list(_LEFT_ACT))
    flip_action_sign: List[int] = field(default_factory=lambda: [0, 2])
    flip_obs_right: List[int] = field(default_factory=lambda: list(_RIGHT_OBS))
    flip_obs_left: List[int] = field(default_factory=lambda: list(_LEFT_OBS))
    flip_obs_sign: List[int] = field(default_factory=lambda: [1, 3, 4, 6, 26, 28, 30, 31, 33, 52])


@dataclass
class BaseConfig:
    xml_path: str = "models/humanoid_mjx.xml"
    lighten_solver: bool = False
    seed: int = 42
    checkpoint_every: int = 50
    log_interval: int = 10
    eval_interval: int = 50
    results_dir: str = "results"
    save_video: bool = False  # a qpos-history .npz per eval for offline rendering (mjx_amd/rendering.py)
    render_fps: int = 60
    render_duration: float = 6.0
    camera_name: str = "side_view"


@dataclass
class APGConfig(BaseConfig):
    lighten_solver: bool = True
    hidden_size: int = 32
    hidden_depth: int = 2
    batch_size: int = 8
    horizon: int = 24
    gamma: float = 0.99
    lr: float = 5e-5
    total_steps: int = 8000
    normalize_observations: bool = True
    grad_clip: float = 0.3           # optax.clip_by_global_norm(0.3), train_apg.py:142-146
    obs_warmup_steps: int = 100      # train_apg.py:256,262
    rms_update_every: int = 10       # train_apg.py:290-292
    # not in the reference: an env whose max |qvel| passes this bound is treated like a non-finite one
    # (dropped from the loss from that step on). Truncated solves (CG 4/4) diverge for some envs under
    # MJX's integrator rules (DESIGN.md "Truncated solves"); the reference's loss turns NaN/huge there.
    diverge_qvel: float = 1e3
    # off = the reference (train_apg.py:290-292 feeds every rollout observation to the statistics). On
    # (opt-in, train_apg.py --rms-in-loss-only; not the reference's normalisation, parity unpinned): only
    # the observations that enter the loss -- of envs not yet terminated, diverged or non-finite -- update
    # them. A fallen env keeps stepping to the horizon; under CG 4/4 some of those diverge (|qvel| ~1e13)
    # and, included, their variance swamps the statistics: when normalisation starts at update 100 every
    # policy input collapses to ~const and the return drops from ~-130 to ~-416 (DESIGN.md "APG C4").
    rms_in_loss_only: bool = False
    # not in the reference (opt-in, train_apg.py --rms-freeze-after N): no observation-statistics updates
    # after update N. At C4 the statistics' drift under a fixed policy is what undoes the learning after
    # normalisation starts: frozen after update 100 the return rises -82 -> -56 over updates 100-300
    # where the drifting statistics take it -101 -> -120 (same resets, DESIGN.md "APG at C4").
    rms_freeze_after: Optional[int] = None


@dataclass
class PPOConfig(BaseConfig):
    lighten_solver: bool = False
    env_config: EnvConfig = field(default_factory=EnvConfig)
    policy_hidden_layer_specs: List[Tuple[int, str]] = field(
        default_factory=lambda: [(256, "tanh"), (256, "tanh"), (256, "tanh")])
    value_hidden_layer_specs: List[Tuple[int, str]] = field(
        default_factory=lambda: [(256, "tanh"), (256, "tanh"), (256, "tanh")])
    num_envs: int = 2048
    rollout_length: int = 128
    gamma: float = 0.999
    lam: float = 0.95
    lr_policy: float = 3e-4
    lr_value: float = 1e-3
    clip_eps: float = 0.2
    ent_coef: float = 0.01
    vf_coef: float = 0.5
    epochs: int = 4
    minibatch_size: int = 1024
    log_std_init: float = 0.0
    total_iterations: int = 1000

    @property
    def total_steps(self) -> int:
        return self.total_iterations

    @classmethod
    def from_dict(cls, data: dict) -> "PPOConfig":
        cfg = cls()
        names = {f.name for f in fields(cfg)}
        for k, v in data.get("ppo", {}).items():
            if k in names:
                setattr(cfg, k, v)
        env_names = {f.name for f in fields(cfg.env_config)}
        for k, v in data.get("env", {}).items():
            if k in env_names:
                setattr(cfg.env_config, k, v)
        fp = data.get("symmetry", {}).get("flip_params", {})
        if "action_index_info" in fp:
            a = fp["action_index_info"]
            cfg.env_config.flip_action_right = list(a["right"])
            cfg.env_config.flip_action_left = list(a["left"])
            cfg.env_config.flip_action_sign = list(a["negative_sign"])
        if "observation_index_info" in fp:
            o = fp["observation_index_info"]
            cfg.env_config.flip_obs_right = list(o["right"])
            cfg.env_config.flip_obs_left = list(o["left"])
            cfg.env_config.flip_obs_sign = list(o["negative_sign"])
        return cfg

    @classmethod
    def from_json(cls, path: str) -> "PPOConfig":
        if not os.path.exists(path):
            return cls()
        with open(path) as f:
            return cls.from_dict(json.load(f))


def reference_ppo_config() -> PPOConfig:
    """The hyper-parameters of reference src/config.json (env :2-22, ppo :110-131)."""
    return PPOConfig.from_dict({
        "env": {"progress_weight": 1.0, "electricity_cost": 0.026, "stall_torque_cost": 0.0000023,
                "joints_at_limit_cost": 0.0, "posture_penalty_weight": 0.0, "tall_height_threshold": 0.7,
                "tall_bonus_weight": 0.0, "target_threshold": 0.15, "target_dist": 2.0, "stop_frames": 1,
                "stance_time_reward_weight": 0.0, "random_joint_noise": 0.01, "random_vel_noise": 0.01,
                "initial_velocity_max": 0.5, "terminate_height": 0.7, "terminate_reward": 0.0,
                "max_episode_steps": 1000, "random_flip": True, "joint_limit_force_threshold": 0.0},
        "ppo": {"lr_policy": 0.0003, "lr_value": 0.0003, "gamma": 0.99, "lam": 0.95, "clip_eps": 0.2,
                "ent_coef": 0.01, "num_envs": 2048, "rollout_length": 256, "minibatch_size": 65536,
                "epochs": 4, "total_iterations": 1000, "log_std_init": 0.0, "log_interval": 10,
                "eval_interval": 100, "checkpoint_every": 100, "seed": 42},
    })

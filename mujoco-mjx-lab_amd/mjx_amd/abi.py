"""ctypes mirrors of the C ABI structs in include/mjx355.h and conversion from compiled models.

The struct layouts here must match `mjlModelDesc` / `mjlEnvConfig` field for field; tests
check `sizeof` against the library (`tests/test_abi.py`).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

MAXBODY, MAXJNT, MAXQ, MAXV, MAXGEOM, MAXSITE, MAXU = 32, 32, 48, 32, 32, 8, 32
MAXTENDON, MAXTENWRAP, MAXPAIR, MAXSENSOR, MAXOBS = 4, 4, 256, 4, 64
AUX_DIM = 9

OPT_STORE_DERIVED = 0
OPT_FORCE_GLOBAL_ROWS = 1
OPT_RESET_POOL = 3  # slots per env of the reset pool (mjl_env_fill_reset_pool)
OPT_VJP_TAPE = 4  # slots of the APG VJP tape (mjl_env_step_record / mjl_env_step_vjp_replay)
OPT_VJP_UNROLLED = 2  # step VJPs differentiate the solver iterations as executed (jax.grad semantics)

FIELD = {
    "qpos": 0, "qvel": 1, "qacc_warmstart": 2, "time": 3, "ctrl": 4, "qacc": 5, "xpos": 6,
    "xquat": 7, "qfrc_actuator": 8, "sensordata": 9, "aux": 10, "stats": 11, "qfrc_bias": 12,
    "qfrc_passive": 13, "qfrc_constraint": 14, "qacc_smooth": 15,
}

i32, f64, f32 = C.c_int32, C.c_double, C.c_float


def _a(t, *dims):
    for d in reversed(dims):
        t = t * d
    return t


class ModelDesc(C.Structure):
    _fields_ = [
        ("nq", i32), ("nv", i32), ("nu", i32), ("nbody", i32), ("njnt", i32), ("ngeom", i32),
        ("nsite", i32), ("ntendon", i32), ("npair", i32), ("nsensor", i32), ("nsensordata", i32),
        ("iterations", i32), ("ls_iterations", i32), ("solver", i32), ("integrator", i32), ("eulerdamp", i32),
        ("timestep", f64), ("gravity", _a(f64, 3)), ("impratio", f64), ("tolerance", f64),
        ("ls_tolerance", f64), ("meaninertia", f64),
        ("body_parentid", _a(i32, MAXBODY)), ("body_rootid", _a(i32, MAXBODY)), ("body_weldid", _a(i32, MAXBODY)),
        ("body_jntadr", _a(i32, MAXBODY)), ("body_jntnum", _a(i32, MAXBODY)),
        ("body_dofadr", _a(i32, MAXBODY)), ("body_dofnum", _a(i32, MAXBODY)),
        ("body_subtree_end", _a(i32, MAXBODY)), ("body_level", _a(i32, MAXBODY)),
        ("body_pos", _a(f64, MAXBODY, 3)), ("body_quat", _a(f64, MAXBODY, 4)), ("body_ipos", _a(f64, MAXBODY, 3)),
        ("body_inertia", _a(f64, MAXBODY, 6)),
        ("body_mass", _a(f64, MAXBODY)), ("body_invweight0", _a(f64, MAXBODY, 2)),
        ("jnt_type", _a(i32, MAXJNT)), ("jnt_qposadr", _a(i32, MAXJNT)), ("jnt_dofadr", _a(i32, MAXJNT)),
        ("jnt_bodyid", _a(i32, MAXJNT)), ("jnt_limited", _a(i32, MAXJNT)),
        ("jnt_pos", _a(f64, MAXJNT, 3)), ("jnt_axis", _a(f64, MAXJNT, 3)), ("jnt_range", _a(f64, MAXJNT, 2)),
        ("jnt_stiffness", _a(f64, MAXJNT)), ("jnt_margin", _a(f64, MAXJNT)),
        ("jnt_solref", _a(f64, MAXJNT, 2)), ("jnt_solimp", _a(f64, MAXJNT, 5)),
        ("dof_bodyid", _a(i32, MAXV)), ("dof_jntid", _a(i32, MAXV)), ("dof_parentid", _a(i32, MAXV)),
        ("dof_damping", _a(f64, MAXV)), ("dof_armature", _a(f64, MAXV)), ("dof_invweight0", _a(f64, MAXV)),
        ("qpos0", _a(f64, MAXQ)), ("qpos_spring", _a(f64, MAXQ)),
        ("geom_type", _a(i32, MAXGEOM)), ("geom_bodyid", _a(i32, MAXGEOM)),
        ("geom_pos", _a(f64, MAXGEOM, 3)), ("geom_quat", _a(f64, MAXGEOM, 4)), ("geom_size", _a(f64, MAXGEOM, 3)),
        ("pair_geom1", _a(i32, MAXPAIR)), ("pair_geom2", _a(i32, MAXPAIR)), ("pair_kind", _a(i32, MAXPAIR)),
        ("pair_condim", _a(i32, MAXPAIR)),
        ("pair_friction", _a(f64, MAXPAIR, 5)), ("pair_solref", _a(f64, MAXPAIR, 2)),
        ("pair_solimp", _a(f64, MAXPAIR, 5)),
        ("pair_margin", _a(f64, MAXPAIR)), ("pair_gap", _a(f64, MAXPAIR)),
        ("site_type", _a(i32, MAXSITE)), ("site_bodyid", _a(i32, MAXSITE)),
        ("site_pos", _a(f64, MAXSITE, 3)), ("site_quat", _a(f64, MAXSITE, 4)), ("site_size", _a(f64, MAXSITE, 3)),
        ("actuator_trnid", _a(i32, MAXU)), ("actuator_ctrllimited", _a(i32, MAXU)),
        ("actuator_gear", _a(f64, MAXU)), ("actuator_ctrlrange", _a(f64, MAXU, 2)),
        ("tendon_num", _a(i32, MAXTENDON)), ("tendon_jnt", _a(i32, MAXTENDON, MAXTENWRAP)),
        ("tendon_limited", _a(i32, MAXTENDON)),
        ("tendon_coef", _a(f64, MAXTENDON, MAXTENWRAP)), ("tendon_range", _a(f64, MAXTENDON, 2)),
        ("tendon_margin", _a(f64, MAXTENDON)), ("tendon_solref", _a(f64, MAXTENDON, 2)),
        ("tendon_solimp", _a(f64, MAXTENDON, 5)), ("tendon_invweight0", _a(f64, MAXTENDON)),
        ("sensor_type", _a(i32, MAXSENSOR)), ("sensor_objid", _a(i32, MAXSENSOR)), ("sensor_adr", _a(i32, MAXSENSOR)),
    ]


class EnvConfigC(C.Structure):
    _fields_ = [
        ("progress_weight", f32), ("electricity_cost", f32), ("stall_torque_cost", f32),
        ("posture_penalty_weight", f32), ("tall_height_threshold", f32), ("tall_bonus_weight", f32),
        ("target_threshold", f32), ("target_dist", f32), ("stance_time_reward_weight", f32),
        ("random_joint_noise", f32), ("random_vel_noise", f32), ("initial_velocity_max", f32),
        ("terminate_height", f32), ("terminate_reward", f32),
        ("stop_frames", i32), ("max_episode_steps", i32), ("random_flip", i32),
        ("pelvis_body_id", i32), ("head_body_id", i32), ("touch_sensor_right_id", i32),
        ("touch_sensor_left_id", i32), ("obs_dim", i32),
        ("act_perm", _a(i32, MAXU)), ("act_sign", _a(f32, MAXU)),
        ("obs_perm", _a(i32, MAXOBS)), ("obs_sign", _a(f32, MAXOBS)),
    ]


_CAP = {"body": MAXBODY, "jnt": MAXJNT, "dof": MAXV, "geom": MAXGEOM, "pair": MAXPAIR, "site": MAXSITE,
        "actuator": MAXU, "tendon": MAXTENDON, "sensor": MAXSENSOR}


class UnsupportedModel(ValueError):
    pass


def model_desc(m) -> ModelDesc:
    """Pack a CompiledModel into the C descriptor (range-checked against the capacities)."""
    if m.nbody > MAXBODY or m.njnt > MAXJNT or m.nv > MAXV or m.nq > MAXQ or m.ngeom > MAXGEOM \
            or m.npair > MAXPAIR or m.nsite > MAXSITE or m.nu > MAXU or m.ntendon > MAXTENDON \
            or m.nsensor > MAXSENSOR:
        raise UnsupportedModel("model exceeds kernel capacities (see include/mjx355.h MJL_MAX*)")
    d = ModelDesc()
    for k in ("nq", "nv", "nu", "nbody", "njnt", "ngeom", "nsite", "ntendon", "npair", "nsensor",
              "nsensordata", "iterations", "ls_iterations", "solver", "integrator", "eulerdamp"):
        setattr(d, k, int(getattr(m, k)))
    for k in ("timestep", "impratio", "tolerance", "ls_tolerance", "meaninertia"):
        setattr(d, k, float(getattr(m, k)))
    for i in range(3):
        d.gravity[i] = float(m.gravity[i])
    names = [f for f, _ in ModelDesc._fields_]
    for name in names:
        if name in m.arrays:
            _fill(getattr(d, name), m.arrays[name])
    return d


def _fill(carr, arr):
    arr = np.asarray(arr)
    if arr.ndim == 1:
        for i, v in enumerate(arr):
            carr[i] = v.item()
    elif arr.ndim == 2:
        if arr.shape[1] > len(carr[0]):
            raise UnsupportedModel("array exceeds capacity")
        for i in range(arr.shape[0]):
            row = carr[i]
            for j in range(arr.shape[1]):
                row[j] = arr[i, j].item()


def desc_size() -> int:
    return C.sizeof(ModelDesc)


def env_config_c(cfg, m, obs_dim: int) -> EnvConfigC:
    """EnvConfig (src/config.py:29-66) -> C struct, building the flip tables the way
    create_env_functions does (reference src/envs.py:48-74)."""
    c = EnvConfigC()
    for k in ("progress_weight", "electricity_cost", "stall_torque_cost", "posture_penalty_weight",
              "tall_height_threshold", "tall_bonus_weight", "target_threshold", "target_dist",
              "stance_time_reward_weight", "random_joint_noise", "random_vel_noise", "initial_velocity_max",
              "terminate_height", "terminate_reward"):
        setattr(c, k, float(getattr(cfg, k)))
    c.stop_frames = int(cfg.stop_frames)
    c.max_episode_steps = int(cfg.max_episode_steps)
    c.random_flip = int(bool(cfg.random_flip))
    c.pelvis_body_id = int(cfg.pelvis_body_id)
    c.head_body_id = int(cfg.head_body_id)
    c.touch_sensor_right_id = int(cfg.touch_sensor_right_id)
    c.touch_sensor_left_id = int(cfg.touch_sensor_left_id)
    c.obs_dim = int(obs_dim)
    act_perm, act_sign, obs_perm, obs_sign = flip_tables(cfg, m.nu, obs_dim)
    for i in range(m.nu):
        c.act_perm[i] = int(act_perm[i])
        c.act_sign[i] = float(act_sign[i])
    for i in range(obs_dim):
        c.obs_perm[i] = int(obs_perm[i])
        c.obs_sign[i] = float(obs_sign[i])
    return c


def flip_tables(cfg, nu: int, obs_dim: int):
    """act_perm/act_sign/obs_perm/obs_sign exactly as reference src/envs.py:48-74."""
    act_perm = np.arange(nu)
    act_sign = np.ones(nu, np.float32)
    obs_perm = np.arange(obs_dim)
    obs_sign = np.ones(obs_dim, np.float32)
    if cfg.random_flip:
        r, l = np.array(cfg.flip_action_right), np.array(cfg.flip_action_left)
        act_perm[r] = l
        act_perm[l] = r
        act_sign[np.array(cfg.flip_action_sign)] = -1.0
        ro, lo = np.array(cfg.flip_obs_right), np.array(cfg.flip_obs_left)
        obs_perm[ro] = lo
        obs_perm[lo] = ro
        obs_sign[np.array(cfg.flip_obs_sign)] = -1.0
    return act_perm, act_sign, obs_perm, obs_sign

"""Env wrapper semantics on the oracle (src/envs.py restated): obs layout, flip, reward terms."""
import numpy as np
import pytest

import mjx_amd
from mjx_amd import abi
from mjx_amd.config import EnvConfig, reference_ppo_config
from mjx_amd.envs import obs_size, resolve_ids
from oracle import Oracle, state_arrays


@pytest.fixture(scope="module")
def env():
    m = mjx_amd.load_model("humanoid_mjx")
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    return m, cfg, abi.env_config_c(cfg, m, obs_size(m.nq, m.nv)), Oracle(m)


def test_dims(env):
    m, cfg, c, _ = env
    assert obs_size(m.nq, m.nv) == 54 and abi.AUX_DIM == 9
    assert (cfg.pelvis_body_id, cfg.head_body_id, cfg.touch_sensor_right_id, cfg.touch_sensor_left_id) == (4, 2, 0, 1)


def test_reset_layout(env):
    m, cfg, c, o = env
    nd = m.nq - 7 + m.nv + 2
    u = np.full(nd, 0.5)
    u[m.nq - 7 + m.nv] = 0.9      # no flip
    u[-1] = 1.0                   # speed = initial_velocity_max
    s, aux, obs = o.env_reset(c, u)
    a = state_arrays(m, s)
    np.testing.assert_allclose(a["qpos"], m.qpos0, atol=1e-12)      # zero noise at u = 0.5
    assert a["qvel"][0] == pytest.approx(cfg.initial_velocity_max) and a["qvel"][1] == 0
    pelvis = a["xpos"][4]
    assert aux[0] == 0 and aux[1] == pytest.approx(pelvis[0] + 2.0) and aux[2] == pytest.approx(pelvis[1])
    assert aux[4] == 0 and aux[6] == 0 and aux[8] == 0
    dist = max(np.hypot(aux[1] - pelvis[0], aux[2] - pelvis[1]), np.hypot(aux[1] - a["xpos"][2][0], aux[2] - a["xpos"][2][1]))
    assert aux[7] == pytest.approx(-dist / m.timestep)
    assert obs[0] == pytest.approx(pelvis[2])
    np.testing.assert_allclose(obs[4:25], a["qpos"][7:], atol=1e-12)
    np.testing.assert_allclose(obs[31:52], a["qvel"][6:], atol=1e-12)


def test_flip_obs_is_permuted(env):
    m, cfg, c, o = env
    nd = m.nq - 7 + m.nv + 2
    u = np.random.default_rng(0).uniform(0, 1, nd)
    u[m.nq - 7 + m.nv] = 0.9
    _, aux0, obs0 = o.env_reset(c, u)
    u[m.nq - 7 + m.nv] = 0.1
    _, aux1, obs1 = o.env_reset(c, u)
    assert aux0[0] == 0 and aux1[0] == 1
    _, _, op, osg = abi.flip_tables(cfg, m.nu, 54)
    np.testing.assert_allclose(obs1, obs0[op] * osg, atol=1e-12)


def test_step_reward_terms(env):
    m, cfg, c, o = env
    nd = m.nq - 7 + m.nv + 2
    u = np.full(nd, 0.5)
    u[m.nq - 7 + m.nv] = 0.9
    s, aux, obs = o.env_reset(c, u)
    act = np.zeros(m.nu)
    s, aux2, obs2, r, te, tr = o.env_step(c, s, aux, act)
    a = state_arrays(m, s)
    # zero action: no actuator force -> no energy term; posture/tall/stance weights are 0 in config.json
    dist = max(np.hypot(aux[1] - a["xpos"][4][0], aux[2] - a["xpos"][4][1]),
               np.hypot(aux[1] - a["xpos"][2][0], aux[2] - a["xpos"][2][1]))
    assert r == pytest.approx((-dist / m.timestep - aux[7]) * cfg.progress_weight, rel=1e-9, abs=1e-9)
    assert te == 0 and tr == 0 and aux2[8] == 1


def test_default_envconfig_matches_reference_defaults():
    e = EnvConfig()
    assert (e.electricity_cost, e.stall_torque_cost, e.target_dist, e.max_episode_steps) == (0.026, 0.0000023, 2.0, 1000)
    r = reference_ppo_config()
    assert (r.num_envs, r.rollout_length, r.minibatch_size, r.epochs, r.gamma, r.lam) == (2048, 256, 65536, 4, 0.99, 0.95)
    assert r.env_config.random_flip is True and r.env_config.posture_penalty_weight == 0.0

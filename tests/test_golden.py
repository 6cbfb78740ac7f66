"""Golden fixtures (tests/golden/, made by tools/make_golden.py from the fp64 oracle).

Parity against MJX itself is unpinned (no jax / mujoco anywhere here): these vectors
pin the CPU restatement against drift (CPU tests, exact to rounding) and hand the HIP path fixed
inputs with known fp64 answers (GPU tests, tolerances as in test_gpu_parity.py).
"""
import os

import numpy as np
import pytest

import mjx_amd
from mjx_amd import abi
from mjx_amd.config import reference_ppo_config
from mjx_amd.envs import obs_size, resolve_ids
from oracle import Oracle, state_arrays

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MODELS = ["humanoid_mjx", "humanoid"]


def _load(name):
    return dict(np.load(os.path.join(GOLD, name)))


@pytest.mark.parametrize("name", MODELS)
def test_oracle_reproduces_physics_fixture(name):
    m = mjx_amd.load_model(name)
    g = _load(f"{name}_physics.npz")
    o = Oracle(m)
    for i in range(len(g["qpos"])):
        ins = (g["qpos"][i], g["qvel"][i], g["qacc_warmstart"][i], g["ctrl"][i])
        a = state_arrays(m, o.forward(o.new_state(*ins)))
        assert (a["ncon"], a["nefc"]) == (g["f_ncon"][i], g["f_nefc"][i])
        for k in ["xpos", "qacc", "qfrc_bias", "qfrc_constraint", "sensordata"]:
            np.testing.assert_allclose(a[k], g["f_" + k][i], atol=1e-9, err_msg=k)
        b = state_arrays(m, o.step(o.new_state(*ins)))
        np.testing.assert_allclose(b["qpos"], g["s_qpos"][i], atol=1e-10)
        np.testing.assert_allclose(b["qvel"], g["s_qvel"][i], atol=1e-8)


@pytest.mark.parametrize("name", MODELS)
def test_oracle_reproduces_speedtest_fixture(name):
    g = _load(f"{name}_speedtest.npz")
    np.testing.assert_allclose(Oracle(mjx_amd.load_model(name)).speedtest(g["vel"]), g["qpos0_out"], atol=1e-12)


def test_oracle_reproduces_env_fixture():
    m = mjx_amd.load_model("humanoid_mjx")
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    c = abi.env_config_c(cfg, m, obs_size(m.nq, m.nv))
    g = _load("humanoid_mjx_env.npz")
    o = Oracle(m)
    for i in range(len(g["u"])):
        s, aux, obs = o.env_reset(c, g["u"][i])
        np.testing.assert_allclose(obs, g["reset_obs"][i], atol=1e-10)
        for t in range(g["actions"].shape[1]):
            s, aux, ob, r, te, tr = o.env_step(c, s, aux, g["actions"][i, t])
            np.testing.assert_allclose(ob, g["obs"][i, t], atol=1e-8)
            assert r == pytest.approx(g["rew"][i, t], abs=1e-8)
            assert (te, tr) == (g["term"][i, t], g["trunc"][i, t])


# ---------------------------------------------------------------- HIP path against the fixtures
@pytest.mark.gpu
@pytest.mark.parametrize("name", MODELS)
def test_hip_matches_physics_fixture(name):
    import torch
    from mjx_amd import mjx
    m = mjx_amd.load_model(name)
    g = _load(f"{name}_physics.npz")
    sys_ = mjx.put_model(m)
    B = len(g["qpos"])
    t = lambda k: torch.tensor(g[k], dtype=torch.float32)
    d = mjx.make_data(sys_, B)
    for k in ["qpos", "qvel", "qacc_warmstart", "ctrl"]:
        d.set(k, t(k))
    mjx.forward(sys_, d)
    st = d.get("stats").cpu().numpy()
    np.testing.assert_array_equal(st[:, 0], g["f_ncon"])
    np.testing.assert_array_equal(st[:, 1], g["f_nefc"])
    for k, rel in [("xpos", 2e-5), ("qfrc_bias", 2e-5), ("qfrc_actuator", 2e-5), ("qacc", 2e-3),
                   ("qfrc_constraint", 2e-3), ("sensordata", 2e-3)]:
        got = d.get(k).cpu().numpy().reshape(B, -1)
        ref = g["f_" + k].reshape(B, -1)
        for i in range(B):
            assert np.abs(got[i] - ref[i]).max() <= rel * (1 + np.abs(ref[i]).max()), (k, i)
    d2 = mjx.make_data(sys_, B)
    for k in ["qpos", "qvel", "qacc_warmstart", "ctrl"]:
        d2.set(k, t(k))
    mjx.step(sys_, d2)
    np.testing.assert_allclose(d2.get("qpos").cpu().numpy(), g["s_qpos"], atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", MODELS)
def test_hip_matches_speedtest_fixture(name):
    import torch
    from mjx_amd import mjx
    g = _load(f"{name}_speedtest.npz")
    sys_ = mjx.put_model(mjx_amd.load_model(name))
    d = mjx.make_data(sys_, len(g["vel"]))
    out = mjx.speedtest_step(sys_, d, torch.tensor(g["vel"], dtype=torch.float32, device="cuda"))
    np.testing.assert_allclose(out.cpu().numpy(), g["qpos0_out"], atol=1e-6)


@pytest.mark.gpu
def test_hip_matches_env_fixture():
    import torch
    from mjx_amd import mjx
    from mjx_amd.envs import HumanoidEnv
    m = mjx_amd.load_model("humanoid_mjx")
    cfg = resolve_ids(m, reference_ppo_config().env_config)
    g = _load("humanoid_mjx_env.npz")
    B = len(g["u"])
    env = HumanoidEnv(mjx.put_model(m), cfg, B, seed=3)
    obs = env.reset(noise=torch.tensor(g["u"], dtype=torch.float32)).cpu().numpy()
    np.testing.assert_allclose(obs, g["reset_obs"], atol=2e-4, rtol=1e-4)
    for t in range(g["actions"].shape[1]):
        o, r, te, tr = (x.cpu().numpy() for x in env.step(torch.tensor(g["actions"][:, t], dtype=torch.float32),
                                                          auto_reset=False))
        ref = g["obs"][:, t]
        assert np.all(np.abs(o - ref).max(1) <= 5e-3 * (1 + np.abs(ref).max(1)))
        np.testing.assert_allclose(r, g["rew"][:, t], atol=5e-3 * (1 + np.abs(g["rew"][:, t]).max()))
        np.testing.assert_array_equal(te, g["term"][:, t])
        np.testing.assert_array_equal(tr, g["trunc"][:, t])

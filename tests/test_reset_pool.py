"""Reset pool (mjl_env_fill_reset_pool): auto-resets computed in bulk before the steps that merge
them (train_ppo.py:147-161 merge_if_done; the reset itself is src/envs.py:115-202). A finished env
merges its next unused slot, which is bit for bit the reset mjl_env_reset draws from the slot's
counter; once its slots are used up it resets in place from the step's counter, as without a pool."""
import dataclasses

import pytest
import torch

import mjx_amd
from mjx_amd import mjx
from mjx_amd._lib import MjlError, check, lib
from mjx_amd.config import reference_ppo_config
from mjx_amd.envs import HumanoidEnv, resolve_ids
from mjx_amd.mjx import _ptr, _stream

pytestmark = pytest.mark.gpu

STATE = ("qpos", "qvel", "qacc_warmstart", "ctrl", "time", "aux", "xpos", "xquat", "sensordata", "qacc",
         "qfrc_actuator", "qfrc_bias", "qfrc_passive", "qfrc_constraint", "qacc_smooth")
DOMAIN = 1 << 63  # the pool's counter domain (include/mjx355.h)


def slot_counter(c0, j):
    """The RNG counter of pool slot j filled at counter c0: the slot index in bits 48..55."""
    return ((c0 + (j << 48)) % (1 << 64)) ^ DOMAIN


def _envs(B, max_steps, seed=5):
    m = mjx_amd.load_model("humanoid_mjx")
    cfg = resolve_ids(m, dataclasses.replace(reference_ppo_config().env_config, max_episode_steps=max_steps))
    return m, [HumanoidEnv(mjx.put_model(m), cfg, B, seed=seed, store_derived=True) for _ in range(2)]


def _reset_at(env, counter):
    check(lib().mjl_env_reset(env.data.handle, None, env.seed, counter, None, _ptr(env.obs), _stream()))
    return env.obs.clone()


def test_pooled_resets_equal_slot_draws():
    """Every env truncates at steps 3, 6, 9 (max_episode_steps 3, zero actions: no falls that early):
    with 2 pooled slots the first two resets are slots 0 and 1, the third is the in-place reset of
    the step's counter; each compared bit for bit (obs and every state / derived field) with
    mjl_env_reset at the same counter on a second batch."""
    B = 64
    m, (env, ref) = _envs(B, max_steps=3)
    env.enable_reset_pool(4)
    env.reset()
    c0 = env.counter
    n = torch.tensor([2], dtype=torch.int32, device="cuda")
    env.fill_reset_pool(n)
    act = torch.zeros((B, m.nu), device="cuda")
    for t in range(1, 10):
        obs, rew, term, trunc = (x.clone() for x in env.step(act))
        if t % 3:
            assert float(trunc.sum()) == 0
            continue
        assert bool(torch.all(trunc == 1)) and float(term.sum()) == 0
        want = _reset_at(ref, slot_counter(c0, t // 3 - 1) if t < 9 else env.counter)
        assert torch.equal(obs, want), f"step {t}: obs"
        for f in STATE:
            assert torch.equal(env.data.get(f), ref.data.get(f)), f"step {t}: {f}"
        assert torch.equal(env.data.get("stats")[:, :3], ref.data.get("stats")[:, :3]), f"step {t}: stats"


def test_pool_fill_is_clamped_and_refilled():
    """n above the capacity fills every slot; a refill restarts every env at slot 0."""
    B = 16
    m, (env, ref) = _envs(B, max_steps=1)
    env.enable_reset_pool(2)
    env.reset()
    act = torch.zeros((B, m.nu), device="cuda")
    for rnd in range(2):
        c0 = env.counter
        env.fill_reset_pool(torch.tensor([100], dtype=torch.int32, device="cuda"))
        for j in range(3):  # every step finishes (max_episode_steps 1): slots 0, 1, then in place
            obs = env.step(act)[0].clone()
            want = _reset_at(ref, slot_counter(c0, j) if j < 2 else env.counter)
            assert torch.equal(obs, want), f"round {rnd} step {j}"


def test_pool_preconditions():
    m, (env, _) = _envs(4, max_steps=1000)
    n = torch.tensor([1], dtype=torch.int32, device="cuda")
    with pytest.raises(MjlError, match="RESET_POOL"):
        env.fill_reset_pool(n)
    env.enable_reset_pool(2)
    env.set_reset_keys(torch.zeros((4, 2), dtype=torch.int32, device="cuda"))
    with pytest.raises(MjlError, match="not pooled"):
        env.fill_reset_pool(n)
    with pytest.raises(MjlError):
        env.data.set_option(3, 65)


def test_consecutive_fills_never_share_a_draw():
    """with the slot index added to the counter, slot j + T of one fill and slot j of the
    next fill (counter + T, here T = 1 < the slot count) drew the same reset; with the slot in the
    high bits every slot of both fills is a distinct draw."""
    B = 8
    m, (env, ref) = _envs(B, max_steps=1000)
    env.enable_reset_pool(4)
    env.reset()
    c0 = env.counter
    seen = []
    for c in (c0, c0 + 1):
        for j in range(4):
            seen.append(_reset_at(ref, slot_counter(c, j)))
    for a in range(len(seen)):
        for b in range(a + 1, len(seen)):
            assert not torch.equal(seen[a], seen[b]), (a, b)

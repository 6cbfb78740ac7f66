"""Batched humanoid walker env on the device (reference src/envs.py, train_ppo.py auto-reset).

The reference builds pure functions `single_reset`/`single_step` and vmaps them
(`create_env_functions`, src/envs.py:26-497); PPO then computes a reset for *every* env on
*every* step and merges it with `where(done, reset, step)` over the whole mjx.Data pytree
(train_ppo.py:149-161). Here one native launch does step + reward + obs and, for the envs that
finished, the reset, in place (`mjl_env_step(auto_reset=1)`); the merged state, obs, reward and
done flags are exactly those of the reference's merge.
"""
from __future__ import annotations

import ctypes as C
from typing import NamedTuple, Optional, Tuple

import torch

from . import abi
from ._lib import MjlError, check, lib
from .config import EnvConfig
from .mjx import Data, Model, _ptr, _stream, make_data


def obs_size(nq: int, nv: int) -> int:
    """1 (height) + 3 (rpy) + (nq-7) joints + nv velocities + 2 target features (src/envs.py:54-56)."""
    return 1 + 3 + (nq - 7) + nv + 2


def resolve_ids(m, cfg: EnvConfig) -> EnvConfig:
    """Body / sensor id lookup done by reference load_model_and_create_env (training_utils.py:84-89)."""
    cfg.pelvis_body_id = m.name2id("body", "pelvis")
    cfg.head_body_id = m.name2id("body", "head")
    cfg.touch_sensor_right_id = m.name2id("sensor", "touch_foot_right")
    cfg.touch_sensor_left_id = m.name2id("sensor", "touch_foot_left")
    if min(cfg.pelvis_body_id, cfg.head_body_id, cfg.touch_sensor_right_id, cfg.touch_sensor_left_id) < 0:
        raise MjlError("model lacks pelvis/head bodies or touch_foot_* sensors")
    return cfg


class HumanoidEnv:
    """`num_envs` walker envs resident on one GPU. State lives in `self.data` (native batch)."""

    def __init__(self, sys: Model, cfg: EnvConfig, num_envs: int, device: int = 0, seed: int = 0,
                 store_derived: bool = False):
        self.sys = sys
        self.cfg = cfg
        self.num_envs = int(num_envs)
        self.obs_dim = obs_size(sys.nq, sys.nv)
        self.act_dim = sys.nu
        self.data: Data = make_data(sys, self.num_envs, device)
        self.data.set_option(abi.OPT_STORE_DERIVED, int(store_derived))
        self._cfg_c = abi.env_config_c(cfg, sys.m, self.obs_dim)
        check(lib().mjl_env_config(self.data.handle, C.byref(self._cfg_c)))
        dev = self.data.device
        self.obs = torch.zeros((self.num_envs, self.obs_dim), dtype=torch.float32, device=dev)
        self.rew = torch.zeros(self.num_envs, dtype=torch.float32, device=dev)
        self.term = torch.zeros(self.num_envs, dtype=torch.float32, device=dev)
        self.trunc = torch.zeros(self.num_envs, dtype=torch.float32, device=dev)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.counter = 0
        # device RNG counter base (0 in eager use): a hipGraph-captured rollout passes counters
        # 1..T and the trainer moves the base before each replay (mjl_batch_set_counter_base)
        self.ctr_base = torch.zeros(1, dtype=torch.int64, device=dev)
        check(lib().mjl_batch_set_counter_base(self.data.handle, C.c_void_p(self.ctr_base.data_ptr())))

    def set_reset_keys(self, keys: Optional[torch.Tensor], mode: int = 1):
        """Draw resets (reset() and the auto-reset of step()) from per-env jax.random keys
        [num_envs, 2] (int32/uint32 bits, device; read at execution time, so update in place), as
        single_reset(key) does (src/envs.py:116-147); None returns to the (seed, counter) stream."""
        if keys is not None:
            if keys.shape != (self.num_envs, 2) or keys.dtype not in (torch.int32, torch.uint32) or not keys.is_cuda \
                    or not keys.is_contiguous():
                raise MjlError("reset keys must be a contiguous [num_envs, 2] int32 CUDA tensor")
        self._keys = keys  # keep the buffer alive while the library points at it
        check(lib().mjl_env_set_reset_keys(self.data.handle, None if keys is None else C.c_void_p(keys.data_ptr()),
                                           int(mode)))

    def _next_counter(self) -> int:
        self.counter += 1
        return self.counter

    def reset(self, mask: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None,
              counter: Optional[int] = None) -> torch.Tensor:
        """v_reset (src/envs.py:115-202,494) on all envs, or on envs with mask > 0.5.
        `noise` [num_envs, nq-7+nv+2] of uniforms replaces the on-device RNG (parity tests).
        `counter` (graph capture) is the RNG counter relative to `ctr_base`; default: the next one."""
        mk = None if mask is None else mask.to(self.obs.device, torch.float32).contiguous()
        nz = None if noise is None else noise.to(self.obs.device, torch.float32).contiguous()
        check(lib().mjl_env_reset(self.data.handle, _ptr(mk), self.seed,
                                  self._next_counter() if counter is None else int(counter), _ptr(nz),
                                  _ptr(self.obs), _stream()))
        return self.obs

    def enable_reset_pool(self, slots: int = 16):
        """Allocate `slots` pooled resets per env (MJL_OPT_RESET_POOL); outside stream capture."""
        self.data.set_option(abi.OPT_RESET_POOL, int(slots))
        self.pool_slots = int(slots)

    def fill_reset_pool(self, n: torch.Tensor, counter: Optional[int] = None):
        """Compute min(n, slots) resets per env in bulk (mjl_env_fill_reset_pool; n: device int32 [1],
        read at execution time); the next auto-resets of step() merge them in order. `counter`:
        the draw's counter (relative to ctr_base under graph capture); default the current counter,
        which the pool's own counter domain keeps apart from the steps' draws."""
        check(lib().mjl_env_fill_reset_pool(self.data.handle, C.c_void_p(n.data_ptr()), self.seed,
                                            self.counter if counter is None else int(counter), _stream()))

    def step(self, act: torch.Tensor, auto_reset: bool = True,
             out: Optional[Tuple[torch.Tensor, ...]] = None, counter: Optional[int] = None) -> Tuple[torch.Tensor, ...]:
        """v_step (src/envs.py:333-495) fused with merge_if_done (train_ppo.py:147-161).
        Returns (obs, reward, terminated, truncated); obs is post-reset for finished envs.
        `counter` (graph capture) is the RNG counter relative to `ctr_base`; default: the next one."""
        act = act.to(self.obs.device, torch.float32).contiguous()
        if act.shape != (self.num_envs, self.act_dim):
            raise MjlError(f"action must have shape {(self.num_envs, self.act_dim)}")
        obs, rew, term, trunc = out if out is not None else (self.obs, self.rew, self.term, self.trunc)
        check(lib().mjl_env_step(self.data.handle, _ptr(act), _ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc),
                                 int(auto_reset), self.seed, self._next_counter() if counter is None else int(counter),
                                 _stream()))
        return obs, rew, term, trunc

    def step_vjp(self, act: torch.Tensor, g_qpos: torch.Tensor, g_qvel: torch.Tensor, g_rew: torch.Tensor,
                 g_aux: Optional[torch.Tensor] = None, nonfinite: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, ...]:
        """VJP of one env step (src/envs.py:333-492, no reset merge) at the current state and aux:
        cotangents of (qpos', qvel', reward, aux') -> (qpos, qvel, action, aux). State unchanged.
        With `nonfinite` (a device float counter) an env whose cotangents come out non-finite gets
        zero outputs and is counted there."""
        dev, B = self.obs.device, self.num_envs
        f = lambda x, *shape: x.to(dev, torch.float32).reshape(B, *shape).contiguous()  # noqa: E731
        act = f(act, self.act_dim)
        gq, gv, gr = f(g_qpos, self.sys.nq), f(g_qvel, self.sys.nv), f(g_rew)
        ga = torch.zeros((B, abi.AUX_DIM), device=dev) if g_aux is None else f(g_aux, abi.AUX_DIM)
        oq, ov = torch.empty_like(gq), torch.empty_like(gv)
        oa, oaux = torch.empty_like(act), torch.empty_like(ga)
        check(lib().mjl_env_step_vjp_guarded(self.data.handle, _ptr(act), _ptr(gq), _ptr(gv), _ptr(gr), _ptr(ga),
                                             _ptr(oq), _ptr(ov), _ptr(oa), _ptr(oaux), _ptr(nonfinite), _stream()))
        return oq, ov, oa, oaux

    def step_vjp_full(self, act: torch.Tensor, g_qpos: torch.Tensor, g_qvel: torch.Tensor, g_ws: torch.Tensor,
                      g_rew: torch.Tensor, g_aux: Optional[torch.Tensor] = None,
                      nonfinite: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, ...]:
        """step_vjp plus the carried warm start (mjl_env_step_vjp_full): g_ws is the cotangent of the
        output qacc_warmstart; returns (qpos, qvel, qacc_warmstart, action, aux) cotangents. The
        warm-start cotangent is nonzero only with the unrolled VJP (jax.grad through the Data carry)."""
        dev, B = self.obs.device, self.num_envs
        f = lambda x, *shape: x.to(dev, torch.float32).reshape(B, *shape).contiguous()  # noqa: E731
        act = f(act, self.act_dim)
        gq, gv, gw, gr = f(g_qpos, self.sys.nq), f(g_qvel, self.sys.nv), f(g_ws, self.sys.nv), f(g_rew)
        ga = torch.zeros((B, abi.AUX_DIM), device=dev) if g_aux is None else f(g_aux, abi.AUX_DIM)
        oq, ov, ow = torch.empty_like(gq), torch.empty_like(gv), torch.empty_like(gw)
        oa, oaux = torch.empty_like(act), torch.empty_like(ga)
        check(lib().mjl_env_step_vjp_full(self.data.handle, _ptr(act), _ptr(gq), _ptr(gv), _ptr(gw), _ptr(gr),
                                          _ptr(ga), _ptr(oq), _ptr(ov), _ptr(ow), _ptr(oa), _ptr(oaux),
                                          _ptr(nonfinite), _stream()))
        return oq, ov, ow, oa, oaux

    @property
    def state_size(self) -> int:
        return int(lib().mjl_state_size(self.data.handle))

    def get_state(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The persistent per-env state as packed rows [num_envs, state_size] = [qpos | qvel |
        qacc_warmstart | aux | time] (one launch)."""
        if out is None:
            out = torch.empty((self.num_envs, self.state_size), dtype=torch.float32, device=self.obs.device)
        check(lib().mjl_get_state(self.data.handle, _ptr(out), _stream()))
        return out

    def set_state(self, src: torch.Tensor, ws_src: Optional[torch.Tensor] = None):
        """Restore packed rows (get_state layout); qacc_warmstart from ws_src's rows if given."""
        check(lib().mjl_set_state(self.data.handle, _ptr(src.contiguous()), _ptr(ws_src), _stream()))

    @property
    def aux(self) -> torch.Tensor:
        return self.data.get("aux")


class EnvState(NamedTuple):
    """The `(mjx.Data, aux)` pair v_reset / v_step pass around (src/envs.py:200,490). `data` is the
    device-resident batch, updated in place by v_step; `aux` [B, 9] is a view of its aux rows."""
    data: Data
    aux: torch.Tensor


def create_env_functions(sys: Model, cfg: EnvConfig, q0=None, nq: Optional[int] = None, nv: Optional[int] = None,
                         device: int = 0, key_mode: int = 1):
    """Reference `create_env_functions(sys, cfg, q0, nq, nv)` (src/envs.py:26,494-497): returns
    `(single_reset, single_step, v_reset, v_step)` with the reference's argument meaning.

    * `v_reset(keys [B, 2] uint32/int32)` -> `(EnvState, obs [B, obs_dim])`: every env reset from its
      jax.random key exactly as `single_reset(key)` draws it (src/envs.py:115-202; `mjl_env_set_reset_keys`);
    * `v_step(state, action [B, nu])` -> `(EnvState, obs, reward, terminated, truncated)` (floats
      {0, 1}), no reset merge (src/envs.py:333-492; train_ppo.py merges, here `HumanoidEnv.step`
      does it in the same launch);
    * `single_reset(key [2])` / `single_step(state, action [nu])`: the same on a one-env batch.

    Not functional: the returned state aliases the batch, which v_step advances in place (the
    library owns the device state; keeping old states would mean copying the pytree every step, the
    cost the fused step avoids). One batch per B is built on first use. `q0` must be the model's
    qpos0 (the reset base; the kernel takes it from the model), `nq` / `nv` the model's sizes.
    The trainers use `HumanoidEnv` directly (step with the fused auto-reset)."""
    import numpy as np
    if nq is not None and nq != sys.nq or nv is not None and nv != sys.nv:
        raise MjlError(f"nq/nv ({nq}, {nv}) do not match the model ({sys.nq}, {sys.nv})")
    if q0 is not None and not np.allclose(np.asarray(q0, np.float64), np.asarray(sys.m.qpos0, np.float64), atol=1e-6):
        raise MjlError("q0 must equal the model's qpos0 (the reset base of the native env)")
    envs = {}

    def _env(B: int) -> HumanoidEnv:
        if B not in envs:
            envs[B] = HumanoidEnv(sys, cfg, B, device=device)
        return envs[B]

    def v_reset(keys: torch.Tensor):
        keys = torch.as_tensor(keys)
        if keys.dim() != 2 or keys.shape[1] != 2:
            raise MjlError("keys must have shape [B, 2]")
        env = _env(keys.shape[0])
        k = keys.to(torch.int64).to(torch.int32).to(env.obs.device).contiguous()
        env.set_reset_keys(k, key_mode)
        obs = env.reset().clone()
        env.set_reset_keys(None)
        return EnvState(env.data, env.aux), obs

    def v_step(state: EnvState, action: torch.Tensor):
        env = next((e for e in envs.values() if e.data is state.data), None)
        if env is None:
            raise MjlError("state does not come from this v_reset")
        obs, rew, term, trunc = env.step(action, auto_reset=False)
        return EnvState(env.data, env.aux), obs.clone(), rew.clone(), term.clone(), trunc.clone()

    def single_reset(key: torch.Tensor):
        st, obs = v_reset(torch.as_tensor(key).reshape(1, 2))
        return st, obs[0]

    def single_step(state: EnvState, action: torch.Tensor):
        st, obs, rew, term, trunc = v_step(state, torch.as_tensor(action).reshape(1, -1))
        return st, obs[0], rew[0], term[0], trunc[0]

    return single_reset, single_step, v_reset, v_step

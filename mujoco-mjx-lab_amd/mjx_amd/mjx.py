"""mjx-shaped front end over the native library (the reference calls `mujoco.mjx`).

    reference                                   here
    mujoco.MjModel.from_xml_path(path)          mjcf.load_model(path)       (host compile)
    mjx.put_model(m)            training_utils.py:105      put_model(m)    -> Model (constants)
    mjx.make_data(sys) (vmapped)   envs.py:110             make_data(sys, nenv, device) -> Data
    mjx.forward(sys, d)            envs.py:112             forward(sys, d, mask=None)
    mjx.step(sys, d)               envs.py:345             step(sys, d, ctrl=None)

Differences forced by a batched, device-resident design: `Data` is a handle to state owned by the
library (one row per env, all envs in one HBM slab), `forward`/`step` update it in place and
return it, and fields are read/written as torch tensors on the batch's GPU.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import abi, mjcf
from ._lib import MjlError, check, lib


def _stream() -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
        raise MjlError("device buffers must be contiguous float32 CUDA tensors")
    return C.c_void_p(t.data_ptr())


class Model:
    """Device-ready model (mjx.Model analog). Holds the compiled constants and the C handle."""

    def __init__(self, compiled: mjcf.CompiledModel):
        self.m = compiled
        self.desc = abi.model_desc(compiled)
        h = C.c_void_p()
        check(lib().mjl_model_create(C.byref(self.desc), C.byref(h)))
        self._h = h
        self.nq, self.nv, self.nu, self.nbody = compiled.nq, compiled.nv, compiled.nu, compiled.nbody
        self.nsensordata = compiled.nsensordata
        self.timestep = compiled.timestep

    @property
    def handle(self):
        return self._h

    @property
    def nefc_max(self) -> int:
        return lib().mjl_model_nefc_max(self._h)

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().mjl_model_destroy(self._h)
                self._h = None
        except Exception:
            pass


_FIELD_DIM = {
    "qpos": lambda m: m.nq, "qvel": lambda m: m.nv, "qacc_warmstart": lambda m: m.nv, "time": lambda m: 1,
    "ctrl": lambda m: m.nu, "qacc": lambda m: m.nv, "xpos": lambda m: m.nbody * 3, "xquat": lambda m: m.nbody * 4,
    "qfrc_actuator": lambda m: m.nv, "sensordata": lambda m: max(1, m.nsensordata), "aux": lambda m: abi.AUX_DIM,
    "stats": lambda m: 4, "qfrc_bias": lambda m: m.nv, "qfrc_passive": lambda m: m.nv,
    "qfrc_constraint": lambda m: m.nv, "qacc_smooth": lambda m: m.nv,
}


class Data:
    """Batched simulation state (mjx.Data with a leading env axis), owned by the library in HBM."""

    def __init__(self, model: Model, nenv: int, device: int = 0):
        if not torch.cuda.is_available():
            raise MjlError("mjx355 needs a GPU (torch.cuda.is_available() is False)")
        self.model = model
        self.nenv = int(nenv)
        self.device = torch.device("cuda", device)
        h = C.c_void_p()
        check(lib().mjl_batch_create(model.handle, self.nenv, int(device), C.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def set_option(self, option: int, value: int):
        check(lib().mjl_batch_set_option(self._h, option, int(value)))

    def get(self, field: str) -> torch.Tensor:
        dim = _FIELD_DIM[field](self.model)
        out = torch.empty((self.nenv, dim), dtype=torch.float32, device=self.device)
        check(lib().mjl_get(self._h, abi.FIELD[field], _ptr(out), _stream()))
        if field == "xpos":
            return out.view(self.nenv, self.model.nbody, 3)
        if field == "xquat":
            return out.view(self.nenv, self.model.nbody, 4)
        if field == "time":
            return out.view(self.nenv)
        return out

    def set(self, field: str, value: torch.Tensor, mask: Optional[torch.Tensor] = None):
        dim = _FIELD_DIM[field](self.model)
        v = value.to(device=self.device, dtype=torch.float32).reshape(self.nenv, dim).contiguous()
        mk = None if mask is None else mask.to(device=self.device, dtype=torch.float32).contiguous()
        check(lib().mjl_set(self._h, abi.FIELD[field], _ptr(v), _ptr(mk), _stream()))

    def __getattr__(self, name):
        if name in _FIELD_DIM:
            return self.get(name)
        raise AttributeError(name)

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().mjl_batch_destroy(self._h)
                self._h = None
        except Exception:
            pass


def put_model(m: mjcf.CompiledModel) -> Model:
    return Model(m)


def make_data(sys: Model, nenv: int = 1, device: int = 0) -> Data:
    """Fresh batched data: qpos = qpos0, everything else zero (mjx.make_data per env)."""
    return Data(sys, nenv, device)


def forward(sys: Model, d: Data, mask: Optional[torch.Tensor] = None) -> Data:
    check(lib().mjl_forward(d.handle, _ptr(mask), _stream()))
    return d


def step(sys: Model, d: Data, ctrl: Optional[torch.Tensor] = None) -> Data:
    if ctrl is not None:
        ctrl = ctrl.to(device=d.device, dtype=torch.float32).contiguous()
        if ctrl.shape != (d.nenv, sys.nu):
            raise MjlError(f"ctrl must have shape {(d.nenv, sys.nu)}")
    check(lib().mjl_step(d.handle, _ptr(ctrl), _stream()))
    return d


def speedtest_step(sys: Model, d: Data, vel: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """mjx_humanoid_speed_test.py:48-57 step(vel): fresh data, qvel[0]=vel, one step -> qpos[0]."""
    if vel.shape != (d.nenv,):
        raise MjlError("vel must have shape (nenv,)")
    out = torch.empty_like(vel) if out is None else out
    check(lib().mjl_speedtest_step(d.handle, _ptr(vel), _ptr(out), _stream()))
    return out


def step_vjp(sys: Model, d: Data, g_qpos: torch.Tensor, g_qvel: torch.Tensor):
    """Reverse-mode derivative of one mjx.step at the batch's current state (not modified):
    cotangents of (qpos', qvel') -> cotangents of (qpos, qvel, ctrl). See include/mjx355.h."""
    dev = d.device
    gq = g_qpos.to(dev, torch.float32).reshape(d.nenv, sys.nq).contiguous()
    gv = g_qvel.to(dev, torch.float32).reshape(d.nenv, sys.nv).contiguous()
    oq = torch.empty_like(gq)
    ov = torch.empty_like(gv)
    oc = torch.empty((d.nenv, sys.nu), dtype=torch.float32, device=dev)
    check(lib().mjl_step_vjp(d.handle, _ptr(gq), _ptr(gv), _ptr(oq), _ptr(ov), _ptr(oc), _stream()))
    return oq, ov, oc


def step_vjp_full(sys: Model, d: Data, g_qpos: torch.Tensor, g_qvel: torch.Tensor, g_qacc_ws: torch.Tensor):
    """step_vjp with the carried warm start (mjl_step_vjp_full): cotangents of (qpos', qvel',
    qacc_warmstart') -> (qpos, qvel, qacc_warmstart, ctrl)."""
    dev = d.device
    gq = g_qpos.to(dev, torch.float32).reshape(d.nenv, sys.nq).contiguous()
    gv = g_qvel.to(dev, torch.float32).reshape(d.nenv, sys.nv).contiguous()
    gw = g_qacc_ws.to(dev, torch.float32).reshape(d.nenv, sys.nv).contiguous()
    oq, ov, ow = torch.empty_like(gq), torch.empty_like(gv), torch.empty_like(gw)
    oc = torch.empty((d.nenv, sys.nu), dtype=torch.float32, device=dev)
    check(lib().mjl_step_vjp_full(d.handle, _ptr(gq), _ptr(gv), _ptr(gw), _ptr(oq), _ptr(ov), _ptr(ow), _ptr(oc),
                                  _stream()))
    return oq, ov, ow, oc

"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/_build/liboracle.so (the serial CPU restatement in physics.hpp/env.hpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product package (mujoco-mjx-lab_amd/mjx_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.join(os.path.dirname(_HERE), "mujoco-mjx-lab_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from mjx_amd import abi  # noqa: E402  (struct layouts only)

MAXCON, MAXEFC = 512, 2048
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

f64, i32 = C.c_double, C.c_int32


def _a(t, *dims):
    for d in reversed(dims):
        t = t * d
    return t


class OrcState(C.Structure):
    _fields_ = [
        ("qpos", _a(f64, abi.MAXQ)), ("qvel", _a(f64, abi.MAXV)), ("qacc_warmstart", _a(f64, abi.MAXV)),
        ("ctrl", _a(f64, abi.MAXU)), ("time", f64),
        ("qacc", _a(f64, abi.MAXV)), ("qacc_smooth", _a(f64, abi.MAXV)), ("qfrc_bias", _a(f64, abi.MAXV)),
        ("qfrc_passive", _a(f64, abi.MAXV)), ("qfrc_actuator", _a(f64, abi.MAXV)),
        ("qfrc_constraint", _a(f64, abi.MAXV)),
        ("xpos", _a(f64, abi.MAXBODY, 3)), ("xquat", _a(f64, abi.MAXBODY, 4)), ("xipos", _a(f64, abi.MAXBODY, 3)),
        ("subtree_com", _a(f64, abi.MAXBODY, 3)), ("cvel", _a(f64, abi.MAXBODY, 6)),
        ("cinert", _a(f64, abi.MAXBODY, 10)), ("cdof", _a(f64, abi.MAXV, 6)),
        ("M", _a(f64, abi.MAXV, abi.MAXV)), ("sensordata", _a(f64, abi.MAXSENSOR)),
        ("ncon", i32), ("nefc", i32), ("niter", i32), ("pad", i32),
        ("con_dist", _a(f64, MAXCON)), ("con_pos", _a(f64, MAXCON, 3)), ("con_frame", _a(f64, MAXCON, 9)),
        ("con_geom", _a(i32, MAXCON, 2)),
        ("efc_force", _a(f64, MAXEFC)), ("efc_D", _a(f64, MAXEFC)), ("efc_aref", _a(f64, MAXEFC)),
        ("efc_pos", _a(f64, MAXEFC)), ("efc_type", _a(i32, MAXEFC)),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.orc_run.argtypes = [P(abi.ModelDesc), P(OrcState), C.c_int, C.c_int, C.c_int]
        L.orc_env_reset.argtypes = [P(abi.ModelDesc), P(abi.EnvConfigC), P(OrcState), P(f64), P(f64), P(f64), C.c_int]
        L.orc_env_step.argtypes = [P(abi.ModelDesc), P(abi.EnvConfigC), P(OrcState), P(f64), P(f64), P(f64), P(f64),
                                   C.c_int]
        L.orc_speedtest.argtypes = [P(abi.ModelDesc), P(f64), C.c_int, P(f64), C.c_int]
        L.orc_rollout.argtypes = [P(abi.ModelDesc), P(OrcState), P(f64), C.c_int, C.c_int]
        L.orc_step_jacobian.argtypes = [P(abi.ModelDesc), P(OrcState), P(f64)]
        L.orc_env_step_jacobian.argtypes = [P(abi.ModelDesc), P(abi.EnvConfigC), P(OrcState), P(f64), P(f64), P(f64)]
        L.orc_step_jacobian_ws.argtypes = [P(abi.ModelDesc), P(OrcState), P(f64)]
        L.orc_env_step_jacobian_ws.argtypes = [P(abi.ModelDesc), P(abi.EnvConfigC), P(OrcState), P(f64), P(f64),
                                               P(f64)]
        L.orc_set_diag.argtypes = [C.c_int]
        L.orc_take_cost_log.argtypes = [P(f64), C.c_int]
        L.orc_take_cost_log.restype = C.c_int
        assert L.orc_state_size() == C.sizeof(OrcState), "OrcState layout mismatch"
        assert L.orc_desc_size() == C.sizeof(abi.ModelDesc), "ModelDesc layout mismatch"
        assert L.orc_envcfg_size() == C.sizeof(abi.EnvConfigC), "EnvConfig layout mismatch"
        _lib = L
    return _lib


DIAG_TRACE, DIAG_SOLVER_QACC, DIAG_COST_LOG = 1, 2, 4  # physics.hpp kDiag*


def set_diag(flags: int) -> None:
    """Truncated-solve diagnostics (physics.hpp kDiag*); 0 restores the restated algorithm."""
    lib().orc_set_diag(int(flags))


def take_cost_log() -> list:
    """Per solve since the last call: [cost at the start, after iteration 1, ...] (needs DIAG_COST_LOG)."""
    buf = np.zeros(1 << 20)
    n = lib().orc_take_cost_log(_dp(buf), buf.size)
    out, cur = [], None
    for x in buf[:n]:
        if np.isnan(x):
            cur = []
            out.append(cur)
        else:
            cur.append(float(x))
    return out


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(f64))


class Oracle:
    """Single-env CPU reference. `use_float` runs the float32 instantiation of the same code."""

    def __init__(self, model, use_float: bool = False):
        self.m = model
        self.desc = abi.model_desc(model)
        self.use_float = int(use_float)
        self.L = lib()

    def new_state(self, qpos=None, qvel=None, qacc_warmstart=None, ctrl=None, time=0.0) -> OrcState:
        s = OrcState()
        m = self.m
        q = m.qpos0 if qpos is None else qpos
        for i in range(m.nq):
            s.qpos[i] = float(q[i])
        for i in range(m.nv):
            s.qvel[i] = 0.0 if qvel is None else float(qvel[i])
            s.qacc_warmstart[i] = 0.0 if qacc_warmstart is None else float(qacc_warmstart[i])
        for i in range(m.nu):
            s.ctrl[i] = 0.0 if ctrl is None else float(ctrl[i])
        s.time = float(time)
        return s

    def forward(self, s: OrcState) -> OrcState:
        self.L.orc_run(C.byref(self.desc), C.byref(s), 0, 1, self.use_float)
        return s

    def step(self, s: OrcState, nstep: int = 1) -> OrcState:
        self.L.orc_run(C.byref(self.desc), C.byref(s), 1, nstep, self.use_float)
        return s

    def speedtest(self, vel: np.ndarray) -> np.ndarray:
        vel = np.ascontiguousarray(vel, np.float64)
        out = np.zeros_like(vel)
        self.L.orc_speedtest(C.byref(self.desc), _dp(vel), vel.size, _dp(out), self.use_float)
        return out

    def rollout(self, s: OrcState, ctrl: np.ndarray) -> OrcState:
        ctrl = np.ascontiguousarray(ctrl, np.float64)
        self.L.orc_rollout(C.byref(self.desc), C.byref(s), _dp(ctrl), ctrl.shape[0], self.use_float)
        return s

    def env_reset(self, envcfg, u: np.ndarray):
        s = OrcState()
        aux = np.zeros(abi.AUX_DIM)
        obs = np.zeros(abi.MAXOBS)
        u = np.ascontiguousarray(u, np.float64)
        self.L.orc_env_reset(C.byref(self.desc), C.byref(envcfg), C.byref(s), _dp(aux), _dp(u), _dp(obs),
                             self.use_float)
        return s, aux, obs[:envcfg.obs_dim].copy()

    def env_step(self, envcfg, s: OrcState, aux: np.ndarray, action: np.ndarray):
        aux = np.ascontiguousarray(aux, np.float64).copy()
        act = np.ascontiguousarray(action, np.float64)
        obs = np.zeros(abi.MAXOBS)
        rtt = np.zeros(3)
        self.L.orc_env_step(C.byref(self.desc), C.byref(envcfg), C.byref(s), _dp(aux), _dp(act), _dp(obs), _dp(rtt),
                            self.use_float)
        return s, aux, obs[:envcfg.obs_dim].copy(), rtt[0], rtt[1], rtt[2]


    def step_jacobian(self, s: OrcState) -> np.ndarray:
        """Exact d(qpos', qvel')/d(qpos, qvel, ctrl) of one step (forward-mode dual numbers)."""
        m = self.m
        jac = np.zeros((m.nq + m.nv, m.nq + m.nv + m.nu))
        assert self.L.orc_step_jacobian(C.byref(self.desc), C.byref(s), _dp(jac)) == 0
        return jac

    def env_step_jacobian(self, envcfg, s: OrcState, aux: np.ndarray, action: np.ndarray) -> np.ndarray:
        """Exact d(qpos', qvel', reward, aux')/d(qpos, qvel, action, aux) of one env step."""
        m = self.m
        rows, cols = m.nq + m.nv + 1 + abi.AUX_DIM, m.nq + m.nv + m.nu + abi.AUX_DIM
        jac = np.zeros((rows, cols))
        aux = np.ascontiguousarray(aux, np.float64)
        act = np.ascontiguousarray(action, np.float64)
        assert self.L.orc_env_step_jacobian(C.byref(self.desc), C.byref(envcfg), C.byref(s), _dp(aux), _dp(act),
                                            _dp(jac)) == 0
        return jac

    def step_jacobian_ws(self, s: OrcState) -> np.ndarray:
        """d(qpos', qvel', qacc_warmstart')/d(qpos, qvel, qacc_warmstart, ctrl): the carried warm start
        as state (what jax.grad through the Data carry differentiates)."""
        m = self.m
        jac = np.zeros((m.nq + 2 * m.nv, m.nq + 2 * m.nv + m.nu))
        assert self.L.orc_step_jacobian_ws(C.byref(self.desc), C.byref(s), _dp(jac)) == 0
        return jac

    def env_step_jacobian_ws(self, envcfg, s: OrcState, aux: np.ndarray, action: np.ndarray) -> np.ndarray:
        """d(qpos', qvel', qacc_warmstart', reward, aux')/d(qpos, qvel, qacc_warmstart, action, aux)."""
        m = self.m
        rows, cols = m.nq + 2 * m.nv + 1 + abi.AUX_DIM, m.nq + 2 * m.nv + m.nu + abi.AUX_DIM
        jac = np.zeros((rows, cols))
        aux = np.ascontiguousarray(aux, np.float64)
        act = np.ascontiguousarray(action, np.float64)
        assert self.L.orc_env_step_jacobian_ws(C.byref(self.desc), C.byref(envcfg), C.byref(s), _dp(aux), _dp(act),
                                               _dp(jac)) == 0
        return jac


def state_arrays(m, s: OrcState) -> dict:
    """Copy the interesting fields of an OrcState into numpy arrays."""
    nv, nq, nb = m.nv, m.nq, m.nbody
    g = lambda name, *shape: np.array(getattr(s, name))[tuple(slice(0, k) for k in shape)]
    return {
        "qpos": g("qpos", nq), "qvel": g("qvel", nv), "qacc_warmstart": g("qacc_warmstart", nv), "time": s.time,
        "qacc": g("qacc", nv), "qacc_smooth": g("qacc_smooth", nv), "qfrc_bias": g("qfrc_bias", nv),
        "qfrc_passive": g("qfrc_passive", nv), "qfrc_actuator": g("qfrc_actuator", nv),
        "qfrc_constraint": g("qfrc_constraint", nv), "xpos": g("xpos", nb, 3), "xquat": g("xquat", nb, 4),
        "xipos": g("xipos", nb, 3), "subtree_com": g("subtree_com", nb, 3), "cvel": g("cvel", nb, 6),
        "cdof": g("cdof", nv, 6), "M": g("M", nv, nv), "sensordata": g("sensordata", m.nsensordata),
        "ncon": s.ncon, "nefc": s.nefc, "niter": s.niter,
        "con_dist": g("con_dist", s.ncon), "con_pos": g("con_pos", s.ncon, 3), "con_frame": g("con_frame", s.ncon, 9),
        "con_geom": g("con_geom", s.ncon, 2), "efc_force": g("efc_force", s.nefc), "efc_type": g("efc_type", s.nefc),
    }

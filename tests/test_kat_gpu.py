"""Closed-form known answers on the HIP path (libmjx355.so), independent of the CPU oracle's code.

The oracle versions of these KATs are in tests/test_oracle_kat.py; here the same closed forms
check the fp32 kernel directly, so a misreading shared by kernel and oracle cannot pass both
(parity unpinned). The expected values come from the MJCF compiler's numpy forward
kinematics / mass matrix (mjx_amd/mjcf.py `_fk_and_mass`, `body_jacobian`) and MuJoCo's documented
soft-constraint model, never from the oracle. Tolerances are fp32 ones, stated per test.
"""
import numpy as np
import pytest
import torch

import mjx_amd
from mjx_amd import mjcf, mjx
from test_oracle_kat import _mj_impedance, _root

pytestmark = pytest.mark.gpu


def _data(sys_, qpos, qvel=None, ctrl=None):
    qpos = np.atleast_2d(qpos)
    d = mjx.make_data(sys_, qpos.shape[0])
    d.set("qpos", torch.tensor(qpos, dtype=torch.float32))
    if qvel is not None:
        d.set("qvel", torch.tensor(np.atleast_2d(qvel), dtype=torch.float32))
    if ctrl is not None:
        d.set("ctrl", torch.tensor(np.atleast_2d(ctrl), dtype=torch.float32))
    return d


@pytest.mark.parametrize("name", ["humanoid_mjx", "humanoid"])
def test_gravity_bias_kat_on_gpu(name):
    """qvel = 0: qfrc_bias = sum_b -J_b(xipos_b)^T m_b g from numpy body Jacobians, and its vertical
    root entry carries the total weight; xpos equals the numpy forward kinematics.
    Tolerance: 2e-5 * (1 + max|expected|) (fp32 kernel, fp64 closed form)."""
    m = mjx_amd.load_model(name)
    sys_ = mjx.put_model(m)
    rng = np.random.default_rng(1)
    qs = []
    for _ in range(6):
        q = m.qpos0.copy()
        q[7:] += rng.uniform(-0.5, 0.5, m.nq - 7)
        q[3:7] = rng.normal(size=4)
        q[3:7] /= np.linalg.norm(q[3:7])
        qs.append(np.float32(q).astype(np.float64))
    d = _data(sys_, np.array(qs))
    mjx.forward(sys_, d)
    bias = d.get("qfrc_bias").cpu().numpy().astype(np.float64)
    xpos = d.get("xpos").cpu().numpy().astype(np.float64).reshape(len(qs), m.nbody, 3)
    for i, q in enumerate(qs):
        kin = mjcf._fk_and_mass(m, q)
        expect = np.zeros(m.nv)
        for b in range(1, m.nbody):
            jp, _ = mjcf.body_jacobian(m, kin, b, kin["xipos"][b])
            expect -= jp.T @ (m.body_mass[b] * m.gravity)
        np.testing.assert_allclose(bias[i], expect, atol=2e-5 * (1 + np.abs(expect).max()))
        assert bias[i][2] == pytest.approx(m.body_mass.sum() * 9.81, rel=1e-5)
        np.testing.assert_allclose(xpos[i], kin["xpos"], atol=2e-5)


def test_solver_optimality_on_gpu():
    """At the solver's answer the gradient of the Gauss + constraint cost vanishes:
    M (qacc - qacc_smooth) = qfrc_constraint, with M the numpy mass matrix of the compiler (not the
    kernel's). Keyframes plus random velocities / controls on humanoid_mjx (Newton 10/20).
    Tolerance: 2e-3 * (1 + max|M (qacc - qacc_smooth)|) (fp32 solve, tolerance-terminated)."""
    m = mjx_amd.load_model("humanoid_mjx")
    sys_ = mjx.put_model(m)
    rng = np.random.default_rng(2)
    n = m.nkey
    q = np.float32(m.key_qpos[:n]).astype(np.float64)
    v = np.float32(rng.uniform(-0.5, 0.5, (n, m.nv))).astype(np.float64)
    c = np.float32(rng.uniform(-1, 1, (n, m.nu))).astype(np.float64)
    d = _data(sys_, q, v, c)
    mjx.forward(sys_, d)
    qacc, qsm, qfc = (d.get(f).cpu().numpy().astype(np.float64) for f in ("qacc", "qacc_smooth", "qfrc_constraint"))
    nefc = d.get("stats").cpu().numpy()[:, 1]
    assert (nefc > 0).sum() >= 3
    for i in range(n):
        M = mjcf._fk_and_mass(m, q[i])["M"]
        lhs = M @ (qacc[i] - qsm[i])
        np.testing.assert_allclose(lhs, qfc[i], atol=2e-3 * (1 + np.abs(lhs).max()))


def test_pendulum_energy_on_gpu():
    """An undamped, unsprung hinge pendulum under implicitfast (dt 1 ms) conserves m g z + 1/2 qd M qd
    over 1000 steps to 3e-3 of the initial energy (numpy FK for z and M)."""
    m = mjcf.compile_xml_string("""<mujoco><option timestep="0.001" integrator="implicitfast"/><worldbody>
      <body pos="0 0 1"><joint type="hinge" axis="0 1 0"/><geom type="capsule" fromto="0 0 0 0.5 0 0" size="0.02"/>
      </body></worldbody></mujoco>""")
    sys_ = mjx.put_model(m)
    v0 = np.array([[0.0], [0.5], [-1.0], [2.0]])
    d = _data(sys_, np.zeros((4, 1)), v0)

    def energy(q, v):
        kin = mjcf._fk_and_mass(m, q)
        return m.body_mass[1] * 9.81 * kin["xipos"][1][2] + 0.5 * v @ kin["M"] @ v
    e0 = [energy(np.zeros(1), v0[i]) for i in range(4)]
    for _ in range(1000):
        mjx.step(sys_, d)
    q, v = (d.get(f).cpu().numpy().astype(np.float64) for f in ("qpos", "qvel"))
    assert np.abs(q).max() > 0.5                       # it swung
    for i in range(4):
        assert abs(energy(q[i], v[i]) - e0[i]) < 3e-3 * abs(e0[i])


@pytest.mark.parametrize("solimp", [(0.9, 0.95, 0.001, 0.5, 2.0), (0.0, 0.99, 0.01, 0.5, 2.0)])
def test_joint_limit_equilibrium_kat_on_gpu(solimp):
    """A rod on a hinge held by gravity against its upper limit comes to rest where the soft limit
    force balances the gravity torque (MuJoCo's soft-constraint model, diagApprox = 1/I; the closed
    form of tests/test_oracle_kat.py). Tolerance rtol 2e-3 (fp32 resolution of a ~1e-3 rad depth)."""
    si = " ".join(map(str, solimp))
    m = mjcf.compile_xml_string(f"""<mujoco><option timestep="0.002"/><worldbody><body>
      <joint type="hinge" axis="0 1 0" limited="true" range="-30 30" solimplimit="{si}"/>
      <geom type="capsule" fromto="0 0 0 0.5 0 0" size="0.02"/></body></worldbody></mujoco>""")
    sys_ = mjx.put_model(m)
    d = _data(sys_, np.zeros((2, 1)), np.array([[0.0], [1.0]]))
    for _ in range(6000):
        mjx.step(sys_, d)
    q, v = (d.get(f).cpu().numpy().astype(np.float64) for f in ("qpos", "qvel"))
    assert np.abs(v).max() < 1e-4
    kin = mjcf._fk_and_mass(m, np.zeros(1))
    inertia, mass = kin["M"][0, 0], m.body_mass[1]
    c = float(np.linalg.norm(kin["xipos"][1]))
    k = 1.0 / (solimp[1] ** 2 * 0.02 ** 2)
    tau = lambda p: mass * 9.81 * c * np.cos(np.deg2rad(30.0) - p)  # noqa: E731
    want = _root(lambda p: p * k * _mj_impedance(solimp, p) ** 2 * inertia + tau(p) * (1.0 - _mj_impedance(solimp, p)),
                 -0.5, 0.0)
    np.testing.assert_allclose(np.deg2rad(30.0) - q[:, 0], want, rtol=2e-3)


def test_sphere_rests_on_plane_on_gpu():
    """A sphere dropped on a plane (condim 3, pyramidal friction; no horizontal velocity, which it would
    keep rolling with) comes to rest at its radius (soft
    penetration < 2 mm) and the contact carries its weight: qfrc_constraint_z = m g (rel 1e-3)."""
    m = mjcf.compile_xml_string("""<mujoco><option timestep="0.005"/><worldbody><geom type="plane" size="0 0 1"/>
      <body pos="0 0 0.3"><freejoint/><geom type="sphere" size="0.1"/></body></worldbody></mujoco>""")
    sys_ = mjx.put_model(m)
    q0 = np.tile(m.qpos0, (3, 1))
    q0[:, 0] = [0.0, 0.5, -1.0]
    d = _data(sys_, q0, np.array([[0, 0, 0, 0, 0, 0], [0, 0, -0.5, 0, 0, 0], [0, 0, 0.5, 0, 0, 0.0]]))
    for _ in range(600):
        mjx.step(sys_, d)
    mjx.forward(sys_, d)
    q, v, f = (d.get(x).cpu().numpy().astype(np.float64) for x in ("qpos", "qvel", "qfrc_constraint"))
    assert np.abs(q[:, 2] - 0.1).max() < 2e-3
    assert np.abs(v).max() < 1e-3
    np.testing.assert_allclose(f[:, 2], m.body_mass[1] * 9.81, rtol=1e-3)

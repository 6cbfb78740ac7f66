"""Pinning the CPU oracle (parity unpinned against MJX itself): analytic known
answers, invariants, and agreement with the compiler's independent numpy forward pass."""
import numpy as np
import pytest

import mjx_amd
from mjx_amd import mjcf
from oracle import Oracle, state_arrays

SPHERE_XML = """<mujoco><worldbody><body><freejoint/><geom size=".15" mass="1" type="sphere"/></body></worldbody></mujoco>"""


@pytest.fixture(scope="module")
def hm():
    return mjx_amd.load_model("humanoid_mjx")


def test_sphere_speedtest_kat():
    """SPHERE row of the speed test (mjx_humanoid_speed_test.py:29-40,50-55): no floor, Euler,
    dt = 0.002: qpos[0] = v*dt, qpos[2] = -g*dt^2 (semi-implicit Euler)."""
    m = mjcf.compile_xml_string(SPHERE_XML.replace(' mass="1"', ""))
    o = Oracle(m)
    vel = np.linspace(0.0, 1.0, 11)
    np.testing.assert_allclose(o.speedtest(vel), vel * 0.002, rtol=0, atol=1e-15)
    s = o.new_state(qvel=np.array([0.3, -0.2, 0.0, 0, 0, 0]))
    o.step(s)
    a = state_arrays(m, s)
    np.testing.assert_allclose(a["qpos"][:3], [0.3 * 0.002, -0.2 * 0.002, -9.81 * 0.002 ** 2], atol=1e-15)


def test_gravity_bias_kat(hm):
    """qvel = 0: qfrc_bias = sum_b -J_b(xipos)^T m_b g (numpy Jacobians from the compiler)."""
    rng = np.random.default_rng(1)
    o = Oracle(hm)
    for _ in range(3):
        q = hm.qpos0.copy()
        q[7:] += rng.uniform(-0.5, 0.5, hm.nq - 7)
        q[3:7] = rng.normal(size=4)
        q[3:7] /= np.linalg.norm(q[3:7])
        s = o.forward(o.new_state(q))
        a = state_arrays(hm, s)
        kin = mjcf._fk_and_mass(hm, q)
        g = hm.gravity
        expect = np.zeros(hm.nv)
        for b in range(1, hm.nbody):
            jp, _ = mjcf.body_jacobian(hm, kin, b, kin["xipos"][b])
            expect -= jp.T @ (hm.body_mass[b] * g)
        np.testing.assert_allclose(a["qfrc_bias"], expect, atol=1e-9)
        assert a["qfrc_bias"][2] == pytest.approx(hm.body_mass.sum() * 9.81)
        np.testing.assert_allclose(a["M"], kin["M"], atol=1e-10)
        np.testing.assert_allclose(a["xpos"], kin["xpos"], atol=1e-12)


def test_solver_optimality(hm):
    """At the Newton solution: M (qacc - qacc_smooth) = qfrc_constraint, pyramid forces >= 0."""
    rng = np.random.default_rng(2)
    o = Oracle(hm)
    checked = 0
    for k in range(hm.nkey):
        s = o.forward(o.new_state(hm.key_qpos[k], rng.uniform(-0.5, 0.5, hm.nv), ctrl=rng.uniform(-1, 1, hm.nu)))
        a = state_arrays(hm, s)
        if a["nefc"] == 0:
            continue
        lhs = a["M"] @ (a["qacc"] - a["qacc_smooth"])
        np.testing.assert_allclose(lhs, a["qfrc_constraint"], atol=1e-6 * (1 + np.abs(lhs).max()))
        assert np.all(a["efc_force"] >= 0)
        assert a["niter"] <= hm.iterations
        checked += 1
    assert checked >= 3


def test_sphere_rests_on_plane():
    xml = """<mujoco><option timestep="0.005"/><worldbody><geom type="plane" size="0 0 1"/>
      <body pos="0 0 0.3"><freejoint/><geom type="sphere" size="0.1"/></body></worldbody></mujoco>"""
    m = mjcf.compile_xml_string(xml)
    o = Oracle(m)
    s = o.new_state()
    o.step(s, 600)
    a = state_arrays(m, s)
    assert abs(a["qpos"][2] - 0.1) < 2e-3          # resting on the plane, small soft penetration
    assert np.abs(a["qvel"]).max() < 1e-3           # at rest
    o.forward(s)
    a = state_arrays(m, s)
    mass = m.body_mass[1]
    fz = a["qfrc_constraint"][2]
    assert fz == pytest.approx(mass * 9.81, rel=1e-3)  # contact carries the weight


def test_pendulum_energy():
    xml = """<mujoco><option timestep="0.001" integrator="implicitfast"/><worldbody>
      <body pos="0 0 1"><joint type="hinge" axis="0 1 0"/><geom type="capsule" fromto="0 0 0 0.5 0 0" size="0.02"/>
      </body></worldbody></mujoco>"""
    m = mjcf.compile_xml_string(xml)
    o = Oracle(m)
    s = o.new_state()
    I = None

    def energy(st):
        a = state_arrays(m, st)
        kin = mjcf._fk_and_mass(m, a["qpos"])
        pe = m.body_mass[1] * 9.81 * kin["xipos"][1][2]
        ke = 0.5 * a["qvel"] @ kin["M"] @ a["qvel"]
        return pe + ke
    e0 = energy(s)
    o.step(s, 1000)
    assert abs(energy(s) - e0) < 2e-3 * abs(e0)
    del I


def test_free_fall_com(hm):
    """In the air (no contacts) the COM follows the discrete semi-implicit particle law."""
    o = Oracle(hm)
    q = hm.qpos0.copy()
    q[2] = 20.0
    rng = np.random.default_rng(3)
    v = rng.uniform(-0.2, 0.2, hm.nv)
    v[:3] = [0.5, -0.3, 1.0]
    s = o.forward(o.new_state(q, v))
    c0 = state_arrays(hm, s)["subtree_com"][1].copy()
    n = 100
    o.step(s, n)
    o.forward(s)
    a = state_arrays(hm, s)
    assert a["ncon"] == 0
    dt = hm.timestep
    # com velocity is not qvel[:3] (limbs move) -> only the vertical gravity drop is checked loosely
    drop = c0[2] - a["subtree_com"][1][2]
    expect = 9.81 * dt * dt * n * (n + 1) / 2 - n * dt * 1.0
    assert abs(drop - expect) < 0.05


def test_float_oracle_agrees(hm):
    rng = np.random.default_rng(4)
    od, of = Oracle(hm), Oracle(hm, use_float=True)
    for k in range(hm.nkey):
        args = (np.float32(hm.key_qpos[k]), np.float32(rng.uniform(-0.5, 0.5, hm.nv)))
        c = np.float32(rng.uniform(-1, 1, hm.nu))
        a = state_arrays(hm, od.forward(od.new_state(*args, ctrl=c)))
        b = state_arrays(hm, of.forward(of.new_state(*args, ctrl=c)))
        assert a["ncon"] == b["ncon"] and a["nefc"] == b["nefc"]
        scale = 1 + np.abs(a["qacc"]).max()
        assert np.abs(a["qacc"] - b["qacc"]).max() < 1e-3 * scale


def _mj_impedance(solimp, x):
    """MuJoCo's impedance d(x) (documentation, Computation > Soft constraints; engine_core_constraint.c
    getimpedance): x = |pos - margin| / width, y(x) a two-piece power sigmoid with midpoint `mid`."""
    d0, dmax, width, mid, power = solimp
    d0, dmax = min(max(d0, 1e-4), 0.9999), min(max(dmax, 1e-4), 0.9999)  # mjMINIMP / mjMAXIMP
    r = abs(x) / width
    if r >= 1.0:
        return dmax
    y = r ** power / mid ** (power - 1) if r <= mid else 1.0 - (1.0 - r) ** power / (1.0 - mid) ** (power - 1)
    return d0 + y * (dmax - d0)


@pytest.mark.parametrize("solref,solimp", [((0.02, 1.0), (0.9, 0.95, 0.001, 0.5, 2.0)),       # MuJoCo defaults
                                           ((0.015, 1.0), (0.9, 0.99, 0.003, 0.5, 2.0)),      # humanoid_mjx bodies
                                           ((0.03, 0.7), (0.8, 0.99, 0.01, 0.3, 3.0))])
def test_contact_equilibrium_penetration_kat(solref, solimp):
    """A frictionless sphere at rest on a plane sinks to where the soft-contact force carries its
    weight. From MuJoCo's documented model (independent of the oracle's code): at rest a = 0, so
    m g = D aref with D = 1/R, R = (1 - d)/d * diagApprox (diagApprox = 1/m for a free sphere) and
    aref = -k d pos, k = 1/(dmax^2 tc^2 dr^2) => pos k d^2 = -g (1 - d), d = d(pos). The oracle's
    steady state must sit on that root."""
    sr, si = " ".join(map(str, solref)), " ".join(map(str, solimp))
    # both geoms carry the parameters (MuJoCo mixes the pair's solref / solimp by solmix)
    xml = f"""<mujoco><option timestep="0.002"/><worldbody>
      <geom type="plane" size="0 0 1" condim="1" solref="{sr}" solimp="{si}"/>
      <body pos="0 0 0.101"><freejoint/><geom type="sphere" size="0.1" condim="1" solref="{sr}" solimp="{si}"/>
      </body></worldbody></mujoco>"""
    m = mjcf.compile_xml_string(xml)
    o = Oracle(m)
    s = o.new_state()
    o.step(s, 4000)
    a = state_arrays(m, s)
    assert np.abs(a["qvel"]).max() < 1e-7
    pen = a["qpos"][2] - 0.1
    tc, dr = max(solref[0], 2 * 0.002), solref[1]   # refsafe: timeconst >= 2 dt
    k = 1.0 / (solimp[1] ** 2 * tc ** 2 * dr ** 2)
    f = lambda p: p * k * _mj_impedance(solimp, p) ** 2 + 9.81 * (1.0 - _mj_impedance(solimp, p))  # noqa: E731
    lo, hi = -0.05, 0.0                              # f(lo) < 0 < f(0): bisection
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        lo, hi = (mid, hi) if f(mid) < 0 else (lo, mid)
    assert pen == pytest.approx(0.5 * (lo + hi), rel=1e-6, abs=1e-12)


def _root(f, lo, hi):
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        lo, hi = (mid, hi) if f(mid) < 0 else (lo, mid)
    return 0.5 * (lo + hi)


def test_contact_parameter_mixing_kat():
    """Different solref / solimp on the two geoms: MuJoCo mixes them by solmix weights (default 1
    each, so the plain mean); the resting penetration is the closed-form root for the mean."""
    a_ref, a_imp = (0.02, 1.0), (0.9, 0.95, 0.001, 0.5, 2.0)
    b_ref, b_imp = (0.015, 1.0), (0.9, 0.99, 0.003, 0.5, 2.0)
    xml = f"""<mujoco><option timestep="0.002"/><worldbody>
      <geom type="plane" size="0 0 1" condim="1" solref="{' '.join(map(str, a_ref))}" solimp="{' '.join(map(str, a_imp))}"/>
      <body pos="0 0 0.101"><freejoint/><geom type="sphere" size="0.1" condim="1" solref="{' '.join(map(str, b_ref))}"
      solimp="{' '.join(map(str, b_imp))}"/></body></worldbody></mujoco>"""
    m = mjcf.compile_xml_string(xml)
    o = Oracle(m)
    s = o.new_state()
    o.step(s, 4000)
    pen = state_arrays(m, s)["qpos"][2] - 0.1
    sr = [(x + y) / 2 for x, y in zip(a_ref, b_ref)]
    si = [(x + y) / 2 for x, y in zip(a_imp, b_imp)]
    k = 1.0 / (si[1] ** 2 * sr[0] ** 2 * sr[1] ** 2)
    want = _root(lambda p: p * k * _mj_impedance(si, p) ** 2 + 9.81 * (1.0 - _mj_impedance(si, p)), -0.05, 0.0)
    assert pen == pytest.approx(want, rel=1e-6)


@pytest.mark.parametrize("solimp", [(0.9, 0.95, 0.001, 0.5, 2.0), (0.0, 0.99, 0.01, 0.5, 2.0)])  # default; humanoid
def test_joint_limit_equilibrium_kat(solimp):
    """A rod on a hinge, pulled by gravity against its upper limit: at rest the limit force f = tau
    (gravity torque m g c cos(q)) and f = -k d(pos)^2 pos I / (1 - d), pos = q_max - q (MuJoCo's soft
    constraint model with diagApprox = dof_invweight0 = 1/I for one hinge)."""
    si = " ".join(map(str, solimp))
    xml = f"""<mujoco><option timestep="0.002"/><worldbody><body>
      <joint type="hinge" axis="0 1 0" limited="true" range="-30 30" solimplimit="{si}"/>
      <geom type="capsule" fromto="0 0 0 0.5 0 0" size="0.02"/></body></worldbody></mujoco>"""
    m = mjcf.compile_xml_string(xml)
    o = Oracle(m)
    s = o.new_state()
    o.step(s, 6000)
    a = state_arrays(m, s)
    assert abs(a["qvel"][0]) < 1e-8
    pos = np.deg2rad(30.0) - a["qpos"][0]
    kin = mjcf._fk_and_mass(m, np.zeros(1))
    inertia, mass = kin["M"][0, 0], m.body_mass[1]
    c = float(np.linalg.norm(kin["xipos"][1]))
    k = 1.0 / (solimp[1] ** 2 * 0.02 ** 2)
    tau = lambda p: mass * 9.81 * c * np.cos(np.deg2rad(30.0) - p)  # noqa: E731
    want = _root(lambda p: p * k * _mj_impedance(solimp, p) ** 2 * inertia + tau(p) * (1.0 - _mj_impedance(solimp, p)),
                 -0.5, 0.0)
    assert pos == pytest.approx(want, rel=1e-6)

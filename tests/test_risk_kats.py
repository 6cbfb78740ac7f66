"""Independent pins for the parity risk register's open rows, written from
closed-form mechanics and MuJoCo's documented models -- not from the oracle's or the kernel's code --
and checked on the CPU oracle here and on the HIP kernel in the `gpu` twins.

* R5 (diagApprox of a contact on a body deep in a kinematic chain): a free root, three hinges about
  the vertical axis, the last body a sphere resting on a frictionless plane. At rest the soft contact
  carries the whole weight W: pos k d(pos)^2 + W diagApprox (1 - d(pos)) = 0 (MuJoCo "Computation >
  Soft constraints": f = -D aref, D = 1/R, R = (1 - d)/d diagApprox, aref = -k d pos), with
  diagApprox = body_invweight0[sphere][0] = trace(J M^-1 J')/3 over the sphere body's COM Jacobian at
  qpos0 (mj_setConst). Here J and M come from finite differences of the compiler's forward kinematics
  (M = sum_b m_b Jv'Jv + Jw' I_b Jw: the kinetic energy), independent of its cdof / CRB code. The
  sphere's COM sits above the root's, so the free joint's rotations enter J: the mean-diagonal
  approximation differs from 1/W_mass (what the vertical direction alone would give) and from
  1/m_sphere, and the test tells them apart.
* R3 (capsule-capsule contact frame): a long capsule lying across two static capsule rails, gravity
  tilted along the free capsule's axis so it slides along itself (no rolling). The pair's normal is
  +z and MJX's frame is make_frame(n): t1 = +y, t2 = n x t1. With the capsule along y (a frame axis)
  the pyramidal friction bound is mu f_n: a = g (sin - mu cos); along (x + y)/sqrt2 (the frame's
  diagonal) it is mu f_n / sqrt2: a = g (sin - mu / sqrt2 cos). A different tangent choice would swap
  (or blend) the two.
* R1 (near-parallel capsules): two capsules 3 degrees apart give MJX's single contact at the segments'
  closest points (the lines' common perpendicular) -- MuJoCo C's mjc_CapsuleCapsule would emit two for
  (near-)parallel segments -- at the midpoint of the overlap along the normal. MJX's +1e-6 in the
  segment-parameter denominator (1 - (d_a . d_b)^2 = sin^2 phi here) moves the points by at most
  1e-6 / sin^2 phi of their distance from the segment midpoint; the tolerances allow for exactly that.
"""
import numpy as np
import pytest

from mjx_amd import mjcf
from oracle import Oracle, state_arrays
from test_oracle_kat import _mj_impedance, _root

G, DT = 9.81, 0.002

# ---- R5 -------------------------------------------------------------------------------------------
SOLREF, SOLIMP = (0.015, 1.0), (0.9, 0.99, 0.003, 0.5, 2.0)   # the humanoid_mjx bodies' contact params
R5_RAD, R5_RISE = 0.25, 0.12   # the sphere's radius, its centre above the root's origin
R5_Z0 = R5_RAD - R5_RISE       # root height with the sphere just touching the plane


def _r5_model():
    sr, si = " ".join(map(str, SOLREF)), " ".join(map(str, SOLIMP))
    return mjcf.compile_xml_string(f"""<mujoco><option timestep="{DT}"/><worldbody>
      <geom type="plane" size="0 0 1" condim="1" solref="{sr}" solimp="{si}"/>
      <body pos="0 0 {R5_Z0}"><freejoint/>
        <geom type="sphere" size="0.06" mass="8" contype="0" conaffinity="0"/>
        <body pos="0 0 0.05"><joint type="hinge" axis="0 0 1"/>
          <geom type="capsule" fromto="-0.12 0 0 0.12 0 0" size="0.03" contype="0" conaffinity="0"/>
          <body pos="0 0 0.04"><joint type="hinge" axis="0 0 1"/>
            <geom type="capsule" fromto="0 -0.1 0 0 0.1 0" size="0.025" contype="0" conaffinity="0"/>
            <body pos="0 0 {R5_RISE - 0.09}"><joint type="hinge" axis="0 0 1"/>
              <geom type="sphere" size="{R5_RAD}" mass="2" condim="1" solref="{sr}" solimp="{si}"/>
            </body></body></body></body></worldbody></mujoco>""")


def _quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def _perturb(m, q, i, eps):
    """qpos moved by eps along velocity coordinate i (free joint: world translation, local rotation)."""
    q = q.copy()
    if i < 3:
        q[i] += eps
    elif i < 6:
        ax = np.zeros(3)
        ax[i - 3] = 1.0
        dq = np.concatenate([[np.cos(eps / 2)], np.sin(eps / 2) * ax])
        q[3:7] = _quat_mul(q[3:7], dq)
    else:
        q[i + 1] += eps  # hinges: qpos index = dof index + 1 after the free joint's 7
    return q


def _fd_jacobians(m, q, eps=1e-6):
    """Per body: COM linear and world angular Jacobians (3 x nv) by central differences of FK."""
    k0 = mjcf._fk_and_mass(m, q)
    nb, nv = m.nbody, m.nv
    Jv, Jw = np.zeros((nb, 3, nv)), np.zeros((nb, 3, nv))
    for i in range(nv):
        kp, km = mjcf._fk_and_mass(m, _perturb(m, q, i, eps)), mjcf._fk_and_mass(m, _perturb(m, q, i, -eps))
        Jv[:, :, i] = (kp["xipos"] - km["xipos"]) / (2 * eps)
        for b in range(nb):
            W = (kp["xmat"][b] - km["xmat"][b]) / (2 * eps) @ k0["xmat"][b].T  # [w]x
            Jw[b, :, i] = [W[2, 1], W[0, 2], W[1, 0]]
    return k0, Jv, Jw


def _fd_mass_matrix(m, k0, Jv, Jw):
    M = np.diag(m.arrays["dof_armature"]).astype(np.float64)
    for b in range(1, m.nbody):
        t = m.arrays["body_inertia"][b]
        Ib = np.array([[t[0], t[3], t[4]], [t[3], t[1], t[5]], [t[4], t[5], t[2]]])
        Iw = k0["xmat"][b] @ Ib @ k0["xmat"][b].T
        M += m.body_mass[b] * Jv[b].T @ Jv[b] + Jw[b].T @ Iw @ Jw[b]
    return M


def _r5_expected_depth(m):
    q0 = m.qpos0.copy()
    k0, Jv, Jw = _fd_jacobians(m, q0)
    M = _fd_mass_matrix(m, k0, Jv, Jw)
    np.testing.assert_allclose(M, k0["M"], atol=1e-7)  # the compiler's CRB M agrees (sanity)
    b = m.nbody - 1
    diag = float(np.trace(Jv[b] @ np.linalg.solve(M, Jv[b].T)) / 3.0)
    W = float(m.body_mass.sum()) * G
    k = 1.0 / (SOLIMP[1] ** 2 * SOLREF[0] ** 2 * SOLREF[1] ** 2)

    def depth(dg):
        return _root(lambda p: p * k * _mj_impedance(SOLIMP, p) ** 2 + W * dg * (1.0 - _mj_impedance(SOLIMP, p)),
                     -0.05, 0.0)
    alt = [depth(1.0 / float(m.body_mass.sum())), depth(1.0 / float(m.body_mass[b]))]
    return depth(diag), alt, diag


def _r5_sphere_bottom(m, qpos):
    return mjcf._fk_and_mass(m, qpos)["xipos"][m.nbody - 1][2] - R5_RAD


def test_r5_deep_chain_contact_depth_oracle():
    m = _r5_model()
    want, alt, diag = _r5_expected_depth(m)
    assert diag > 1.2 / m.body_mass.sum()      # the root's rotations do enter the approximation
    for a in alt:                               # and the alternatives are far apart at this tolerance
        assert abs(a - want) > 0.05 * abs(want)
    o = Oracle(m)
    s = o.new_state()
    o.step(s, 4000)
    a = state_arrays(m, s)
    assert np.abs(a["qvel"]).max() < 1e-6
    assert _r5_sphere_bottom(m, a["qpos"]) == pytest.approx(want, rel=1e-5)


@pytest.mark.gpu
def test_r5_deep_chain_contact_depth_on_gpu():
    from mjx_amd import mjx
    m = _r5_model()
    want, _, _ = _r5_expected_depth(m)
    sys_ = mjx.put_model(m)
    d = mjx.make_data(sys_, 4)
    for _ in range(4000):
        mjx.step(sys_, d)
    q = d.get("qpos").cpu().numpy().astype(np.float64)
    got = np.array([_r5_sphere_bottom(m, qi) for qi in q])
    np.testing.assert_allclose(got, want, rtol=2e-3)


# ---- R3 -------------------------------------------------------------------------------------------
R3_MU, R3_THETA = 0.5, 30.0


def _r3_xml(diag):
    w = np.array([1.0, 1.0, 0.0]) / np.sqrt(2.0) if diag else np.array([0.0, 1.0, 0.0])  # free capsule axis
    u = np.array([w[1], -w[0], 0.0])                                                      # rail axis
    th = np.deg2rad(R3_THETA)
    g = G * np.sin(th) * w + np.array([0.0, 0.0, -G * np.cos(th)])
    fr = f'friction="{R3_MU} 0.005 0.0001"'
    rails = ""
    for off in (-0.8, 0.8):
        a, b = off * w - 0.3 * u, off * w + 0.3 * u
        rails += (f'<geom type="capsule" fromto="{a[0]:.17g} {a[1]:.17g} 0 {b[0]:.17g} {b[1]:.17g} 0" size="0.03" '
                  f'condim="3" {fr}/>')
    e = 1.6 * w
    return f"""<mujoco><option timestep="{DT}" gravity="{g[0]:.17g} {g[1]:.17g} {g[2]:.17g}"/><worldbody>{rails}
      <body pos="0 0 {0.03 + 0.04 - 0.0005}"><freejoint/>
      <geom type="capsule" fromto="{-e[0]:.17g} {-e[1]:.17g} 0 {e[0]:.17g} {e[1]:.17g} 0" size="0.04" condim="3" {fr}/>
      </body></worldbody></mujoco>""", w


def _r3_accel(diag, run):
    """Least-squares slope of the velocity along the free capsule's axis over steps [50, 450) (the
    contacts hop on the pyramid rows and the capsule pitches slightly on the rails, so the velocity
    is a noisy ramp): it slides < 0.7 m, its COM stays between the rails (+-0.8 m along its axis) and
    its 1.6 m half-length lies over both."""
    xml, w = _r3_xml(diag)
    m = mjcf.compile_xml_string(xml)
    v = run(m, w, 50, 450)
    t = np.arange(len(v)) * DT
    return np.polyfit(t, v, 1)[0], m  # (per env when v is [steps, envs])


def _oracle_run(m, w, s0, s1):
    o = Oracle(m)
    s = o.new_state()
    o.step(s, s0)
    vs = []
    for _ in range(s1 - s0):
        a = state_arrays(m, s)
        for c in range(a["ncon"]):  # (a sliding body hops on the pyramid rows: 0-2 contacts at a time)
            np.testing.assert_allclose(np.abs(a["con_frame"][c][:3]), [0, 0, 1], atol=1e-2)
            np.testing.assert_allclose(np.abs(a["con_frame"][c][3:6]), [0, 1, 0], atol=1e-2)  # make_frame(+-z): t1 = y
        vs.append(a["qvel"][:3] @ w)
        o.step(s)
    return np.array(vs)


def _r3_expect(diag):
    th = np.deg2rad(R3_THETA)
    mu = R3_MU / np.sqrt(2.0) if diag else R3_MU
    return G * (np.sin(th) - mu * np.cos(th))


@pytest.mark.parametrize("diag", [False, True])
def test_r3_capsule_capsule_pyramid_frame_oracle(diag):
    a, _ = _r3_accel(diag, _oracle_run)
    a = float(a)
    assert a == pytest.approx(_r3_expect(diag), rel=0.03)
    assert abs(a - _r3_expect(not diag)) > 0.5  # tells the two frames apart


@pytest.mark.gpu
def test_r3_capsule_capsule_pyramid_frame_on_gpu():
    import torch
    from mjx_amd import mjx

    def run(m, w, s0, s1):
        sys_ = mjx.put_model(m)
        d = mjx.make_data(sys_, 2)
        for _ in range(s0):
            mjx.step(sys_, d)
        vs = []
        for _ in range(s1 - s0):
            vs.append(d.get("qvel")[:, :3].clone())
            mjx.step(sys_, d)
        torch.cuda.synchronize()
        return np.stack([x.cpu().numpy().astype(np.float64) @ w for x in vs])  # [steps, envs]
    for diag in (False, True):
        a, _ = _r3_accel(diag, run)
        np.testing.assert_allclose(a, _r3_expect(diag), rtol=0.03)


# ---- R1 -------------------------------------------------------------------------------------------
R1_PHI = np.deg2rad(3.0)
R1_RA, R1_RB, R1_HA, R1_HB = 0.05, 0.04, 0.5, 0.3
R1_DIR = np.array([np.cos(R1_PHI), np.sin(R1_PHI), 0.0])


def _r1_model():
    d = R1_DIR * R1_HB
    return mjcf.compile_xml_string(f"""<mujoco><option gravity="0 0 0"/><worldbody>
      <geom type="capsule" fromto="-{R1_HA} 0 0 {R1_HA} 0 0" size="{R1_RA}" condim="1"/>
      <body><freejoint/><geom type="capsule" fromto="{-d[0]:.17g} {-d[1]:.17g} 0 {d[0]:.17g} {d[1]:.17g} 0"
      size="{R1_RB}" condim="1"/></body></worldbody></mujoco>""")


def _r1_expect(body):
    """Closest points of the x-axis segment and the free one through `body` along R1_DIR (both in
    horizontal planes: the common perpendicular is vertical, at the lines' crossing in projection)."""
    t = -body[1] / R1_DIR[1]
    pb = body + t * R1_DIR
    pa = np.array([pb[0], 0.0, 0.0])
    assert abs(t) < R1_HB and abs(pa[0]) < R1_HA
    n = (pb - pa) / np.linalg.norm(pb - pa)
    dist = np.linalg.norm(pb - pa) - R1_RA - R1_RB
    return dist, n, pa + n * (R1_RA + 0.5 * dist), abs(t)


R1_BODIES = [np.array([0.1, 0.006, 0.088]), np.array([-0.15, -0.004, 0.0885])]


def _r1_qpos(m, body):
    q = m.qpos0.copy()
    q[:3] = body
    q[3:7] = [1, 0, 0, 0]
    return q


def test_r1_near_parallel_capsules_one_contact_oracle():
    m = _r1_model()
    o = Oracle(m)
    for body in R1_BODIES:
        dist, n, pos, t = _r1_expect(body)
        assert -0.01 < dist < 0
        tol = 1e-6 / np.sin(R1_PHI) ** 2 * (t + 0.2) + 1e-6   # MJX's regularisation bound (module doc)
        a = state_arrays(m, o.forward(o.new_state(_r1_qpos(m, body))))
        assert a["ncon"] == 1
        assert a["con_dist"][0] == pytest.approx(dist, abs=1e-6)
        np.testing.assert_allclose(np.abs(a["con_frame"][0][:3]), np.abs(n), atol=tol * np.sin(R1_PHI) / 0.08 + 1e-6)
        np.testing.assert_allclose(a["con_pos"][0], pos, atol=tol)


@pytest.mark.gpu
def test_r1_near_parallel_capsules_one_contact_on_gpu():
    import torch
    from mjx_amd import mjx
    m = _r1_model()
    sys_ = mjx.put_model(m)
    d = mjx.make_data(sys_, len(R1_BODIES))
    d.set("qpos", torch.tensor(np.array([_r1_qpos(m, b) for b in R1_BODIES]), dtype=torch.float32))
    mjx.forward(sys_, d)
    st = d.get("stats").cpu().numpy()
    qf = d.get("qfrc_constraint").cpu().numpy().astype(np.float64)
    for i, body in enumerate(R1_BODIES):
        dist, n, pos, t = _r1_expect(body)
        assert st[i][0] == 1
        f = qf[i]
        np.testing.assert_allclose(f[:3] / np.linalg.norm(f[:3]), n, atol=2e-4)
        # torque (pos - origin) x F: the force acts at the closed-form point (to 2e-4 m + the bound)
        lever = 2e-4 + 1e-6 / np.sin(R1_PHI) ** 2 * (t + 0.2)
        np.testing.assert_allclose(f[3:6], np.cross(pos - body, f[:3]), atol=lever * np.linalg.norm(f[:3]))


# ---- R6 -------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_r6_fp32_activation_outliers_bounded():
    """R6 (the kernel's fp32 solver exits and fp32 contact activation): 50 steps of 2048 humanoid_mjx
    envs from env resets (falling, landing, contacts coming and going) under random controls, each
    step re-synced: the oracle (fp64, MJX's exact solver loop) steps every env from the GPU's own
    fp32 state, and an env-step is an outlier when its contact / row counts differ from the oracle's
    or its next qpos / qvel leaves the parity tolerance (qpos 1e-4, qvel 1e-2 (1 + max|qvel|)). Such
    an env is one whose contact sits at its activation distance, decided differently in fp32 and
    fp64, or whose solver exit lands elsewhere. Ceiling: 0.15 % of the env-steps (measured in
    round 2 at 2048 x 3: 0.05 %); every other env-step within the tolerance by construction."""
    import torch
    from mjx_amd import mjx
    from test_gpu_parity import _env
    B, T = 2048, 50
    m, env, _ = _env(B)
    sys_ = env.sys
    nd = m.nq - 7 + m.nv + 2
    rng = np.random.default_rng(11)
    env.reset(noise=torch.tensor(rng.uniform(0, 1, (B, nd)).astype(np.float32)))
    d = env.data
    d.set_option(0, 1)  # store derived fields: the stats row carries (ncon, nefc)
    orc = Oracle(m)
    outliers = np.zeros(T, int)
    for t in range(T):
        ctrl = rng.uniform(-1, 1, (B, m.nu)).astype(np.float32)
        q0, v0, w0 = (d.get(f).cpu().numpy().astype(np.float64) for f in ("qpos", "qvel", "qacc_warmstart"))
        mjx.step(sys_, d, torch.tensor(ctrl, device="cuda"))
        q1, v1 = d.get("qpos").cpu().numpy(), d.get("qvel").cpu().numpy()
        st = d.get("stats").cpu().numpy()
        for i in range(B):
            s = orc.new_state(q0[i], v0[i], w0[i], ctrl=ctrl[i].astype(np.float64))
            orc.step(s)
            a = state_arrays(m, s)
            bad = (int(st[i][0]), int(st[i][1])) != (a["ncon"], a["nefc"])
            bad |= np.abs(q1[i] - a["qpos"]).max() > 1e-4
            bad |= np.abs(v1[i] - a["qvel"]).max() > 1e-2 * (1 + np.abs(a["qvel"]).max())
            outliers[t] += bool(bad)
    total = int(outliers.sum())
    print(f"R6: {total} outlier env-steps of {B * T} ({100.0 * total / (B * T):.3f} %), per step {outliers.tolist()}")
    assert total <= 0.0015 * B * T

"""Contact known-answer tests, written from closed-form mechanics and MuJoCo's documented contact
model, independent of the oracle's and the kernel's code (VERDICT r1 "independent pins").

* Pyramidal friction (condim 3, MuJoCo's default cone): a plane contact's force is a non-negative
  combination of the edges n +- mu t1, n +- mu t2, with (t1, t2) the contact frame's tangents, so the
  friction along a tangent axis is bounded by mu f_n and along the diagonal (t1 + t2)/sqrt2 by
  mu f_n / sqrt2 (the diamond inscribed in the elliptic cone). MJX's plane-sphere frame is
  `math.make_frame(n)`: for n = +z, t1 = +y, t2 = n x t1 = -x; its plane-capsule frame puts t1 along
  the capsule axis projected on the plane.
  - A capsule lying on an incline along the slope cannot roll (two contacts): it sticks for
    tan(theta) < mu and slides with a = g (sin(theta) - mu cos(theta)) above.
  - A sphere rolls without slipping for tan(theta) < 7/2 mu: a = 5/7 g sin(theta) (solid sphere,
    I = 2/5 m r^2); below that mu it slides: a = g (sin(theta) - mu_eff cos(theta)), mu_eff = mu along
    a frame axis and mu / sqrt2 along the frame diagonal.
  The incline is a tilted gravity vector over the z-up floor (same dynamics, and the floor keeps
  the frame the test names). A sliding body hops on MuJoCo's pyramid rows (each edge row's
  reference acceleration -b J v carries -/+ b mu v_t: an edge row pushes the body off the plane in
  proportion to the slip speed), and the contact comes and goes; the friction impulse is still mu
  times the normal impulse whenever the contact is on, so the slope-direction velocity gained over
  a window is the closed form's, which the tests compare.
* Capsule-capsule and capsule-sphere geometry: the closest points of two segments / a point and a
  segment in closed form give the contact distance, normal (from the first geom to the second) and
  position (the midpoint of the overlap, MJX `_sphere_sphere` on the closest points). MJX regularises
  the segment-parameter denominators with +1e-6 (`math.closest_segment_point`,
  `closest_segment_to_segment_points`), which moves the points by <= 1e-6 of a segment length; the
  tolerances below allow for that.

Each physics KAT runs on the CPU oracle here and on the HIP kernel in the `gpu` twin, which reads
the contact through what the C ABI exposes: the active contact count and qfrc_constraint, whose
free-joint part is (F, (p - body origin) x F) for a single frictionless contact at p with force F
along the normal.
"""
import numpy as np
import pytest

from mjx_amd import mjcf
from oracle import Oracle, state_arrays

G = 9.81
DT = 0.002


def _incline_xml(theta_deg, mu, body_geom, diag=False):
    th = np.deg2rad(theta_deg)
    d = np.array([1.0, 1.0, 0.0]) / np.sqrt(2.0) if diag else np.array([1.0, 0.0, 0.0])
    g = G * np.sin(th) * d + np.array([0.0, 0.0, -G * np.cos(th)])
    fr = f'friction="{mu} 0.005 0.0001"'
    return f"""<mujoco><option timestep="{DT}" gravity="{g[0]:.17g} {g[1]:.17g} {g[2]:.17g}"/><worldbody>
      <geom type="plane" size="0 0 1" condim="3" {fr}/>
      <body pos="0 0 0.0995"><freejoint/>{body_geom.format(fr=fr)}</body></worldbody></mujoco>""", d


SPHERE = '<geom type="sphere" size="0.1" {fr}/>'
CAPSULE_X = '<geom type="capsule" fromto="-0.2 0 0 0.2 0 0" size="0.1" {fr}/>'


def _slope_accel(theta_deg, mu, body_geom, diag=False, settle=500, nstep=1500):
    """Mean slope-direction acceleration of the oracle over steps [settle, nstep), and the final
    slope-direction speed."""
    xml, d = _incline_xml(theta_deg, mu, body_geom, diag)
    m = mjcf.compile_xml_string(xml)
    o = Oracle(m)
    s = o.new_state()
    o.step(s, settle)
    v0 = state_arrays(m, s)["qvel"][:3] @ d
    o.step(s, nstep - settle)
    v1 = state_arrays(m, s)["qvel"][:3] @ d
    return (v1 - v0) / ((nstep - settle) * DT), v1


def _slide(theta_deg, mu):
    th = np.deg2rad(theta_deg)
    return G * (np.sin(th) - mu * np.cos(th))


def test_plane_contact_frames_are_mjx_make_frame():
    """The frames the friction KATs assume: plane-sphere t1 = +y (make_frame(+z)), plane-capsule t1
    along the capsule axis."""
    for geom, t1 in ((SPHERE, [0, 1, 0]), (CAPSULE_X, [1, 0, 0]),
                     (CAPSULE_X.replace("-0.2 0 0 0.2 0 0", "0 -0.2 0 0 0.2 0"), [0, 1, 0])):
        xml, _ = _incline_xml(0.0, 1.0, geom)
        m = mjcf.compile_xml_string(xml)
        o = Oracle(m)
        a = state_arrays(m, o.forward(o.new_state()))
        assert a["ncon"] >= 1
        for c in range(a["ncon"]):
            f = a["con_frame"][c].reshape(3, 3)
            np.testing.assert_allclose(f[0], [0, 0, 1], atol=1e-12)
            np.testing.assert_allclose(np.abs(f[1]), np.abs(t1), atol=1e-12)
            np.testing.assert_allclose(f[2], np.cross(f[0], f[1]), atol=1e-12)


@pytest.mark.parametrize("theta,slides", [(22.0, False), (26.5, False), (27.0, True), (35.0, True)])
def test_capsule_stick_slip_threshold(theta, slides):
    """mu = 0.5, tan(theta*) = mu at theta* = 26.565 deg. Below: the capsule sticks (soft-contact
    creep below 1 cm/s, no sustained acceleration); above: a = g (sin - mu cos)."""
    a, v = _slope_accel(theta, 0.5, CAPSULE_X)
    if slides:   # the hopping contact averages out to 3 % (5e-3 m/s^2 absolute just past the threshold)
        assert a == pytest.approx(_slide(theta, 0.5), rel=0.03, abs=5e-3)
    else:
        assert abs(v) < 0.01 and abs(a) < 1e-3


def test_sphere_rolls_without_slipping():
    """mu = 1 > 2/7 tan(30 deg): rolling, a = 5/7 g sin(theta)."""
    a, _ = _slope_accel(30.0, 1.0, SPHERE)
    assert a == pytest.approx(5.0 / 7.0 * G * np.sin(np.deg2rad(30.0)), rel=5e-3)


@pytest.mark.parametrize("diag", [False, True])
def test_sphere_slides_on_pyramid(diag):
    """mu = 0.1 < 2/7 tan(30 deg): sliding; the friction bound is mu f_n along the frame axis x and
    mu f_n / sqrt2 along the diagonal (pyramidal cone, not the elliptic cone's mu f_n)."""
    a, _ = _slope_accel(30.0, 0.1, SPHERE, diag=diag)
    mu_eff = 0.1 / np.sqrt(2.0) if diag else 0.1
    assert a == pytest.approx(_slide(30.0, mu_eff), rel=5e-3)
    assert abs(a - _slide(30.0, 0.1 if diag else 0.1 / np.sqrt(2.0))) > 0.1   # tells the two apart


# ---- capsule-capsule / capsule-sphere contact geometry ----------------------------------------

PHI = np.deg2rad(30.0)
RA, RB, RS = 0.05, 0.04, 0.06          # static capsule, free capsule, free sphere radii
HALF_A, HALF_B = 0.5, 0.3
DIR_B = np.array([0.0, np.cos(PHI), np.sin(PHI)])


def _cc_model():
    d = DIR_B * HALF_B
    return mjcf.compile_xml_string(f"""<mujoco><option gravity="0 0 0"/><worldbody>
      <geom type="capsule" fromto="-{HALF_A} 0 0 {HALF_A} 0 0" size="{RA}" condim="1"/>
      <body><freejoint/><geom type="capsule" fromto="{-d[0]} {-d[1]:.17g} {-d[2]:.17g} {d[0]} {d[1]:.17g} {d[2]:.17g}"
      size="{RB}" condim="1"/></body></worldbody></mujoco>""")


def _cs_model():
    return mjcf.compile_xml_string(f"""<mujoco><option gravity="0 0 0"/><worldbody>
      <geom type="capsule" fromto="-{HALF_A} 0 0 {HALF_A} 0 0" size="{RA}" condim="1"/>
      <body><freejoint/><geom type="sphere" size="{RS}" condim="1"/></body></worldbody></mujoco>""")


def _seg_closest(a0, a1, p):
    ab = a1 - a0
    t = np.clip((p - a0) @ ab / (ab @ ab), 0.0, 1.0)
    return a0 + t * ab


def _cc_closed_form(body):
    """Closest points of the static segment (x axis, |x| <= HALF_A) and the free one (body +-
    HALF_B DIR_B), for the two configurations used: lines' common perpendicular inside both
    segments, or an endpoint pair."""
    b0, b1 = body - HALF_B * DIR_B, body + HALF_B * DIR_B
    a0, a1 = np.array([-HALF_A, 0, 0.0]), np.array([HALF_A, 0, 0.0])
    # interior: point on B closest to the x axis (minimise y(t)^2 + z(t)^2), then its x on A
    t = -(body[1] * DIR_B[1] + body[2] * DIR_B[2])
    if abs(t) <= HALF_B and abs(body[0]) <= HALF_A:
        pb = body + t * DIR_B
        pa = np.array([pb[0], 0.0, 0.0])
    else:                                   # endpoint pair: the closer of the two clamped projections
        cands = [(_seg_closest(a0, a1, e), e) for e in (b0, b1)] + [(e, _seg_closest(b0, b1, e)) for e in (a0, a1)]
        pa, pb = min(cands, key=lambda c: np.linalg.norm(c[1] - c[0]))
    return pa, pb, RA, RB


def _cs_closed_form(body):
    pa = _seg_closest(np.array([-HALF_A, 0, 0.0]), np.array([HALF_A, 0, 0.0]), body)
    return pa, body.copy(), RA, RS


def _expect(pa, pb, ra, rb):
    n = (pb - pa) / np.linalg.norm(pb - pa)
    dist = np.linalg.norm(pb - pa) - ra - rb
    return dist, n, pa + n * (ra + 0.5 * dist)


# free-body origins: penetrating by a few mm (checked), and the same pose shifted to +1e-4 clear
CC_BODIES = [np.array([0.1, 0.0, 0.088 / np.cos(PHI)]),                 # interior, common perpendicular
             np.array([-0.2, 0.03, 0.085 / np.cos(PHI) + 0.03 * np.tan(PHI)]),  # interior, offset in y
             np.array([0.55, 0.0, 0.06]) + HALF_B * DIR_B]               # B's lower end over A's end
CS_BODIES = [np.array([0.2, 0.03, 0.1]), np.array([0.55, 0.02, 0.05])]


def _clear(body, closed_form, eps=1e-4):
    """Move the body along the contact normal until the closed-form distance is +eps."""
    dist, n, _ = _expect(*closed_form(body))
    out = body + n * (eps - dist)
    d2, _, _ = _expect(*closed_form(out))
    assert d2 == pytest.approx(eps, abs=1e-9)
    return out


def _qpos(m, body):
    q = m.qpos0.copy()
    q[:3] = body
    q[3:7] = [1, 0, 0, 0]
    return q


@pytest.mark.parametrize("kind", ["capsule_capsule", "capsule_sphere"])
def test_segment_contact_geometry_closed_form(kind):
    m, bodies, cf = (_cc_model(), CC_BODIES, _cc_closed_form) if kind == "capsule_capsule" else \
        (_cs_model(), CS_BODIES, _cs_closed_form)
    # MuJoCo orders a pair's geoms by type (sphere 2 < capsule 3) and the frame normal points from
    # geom1 to geom2: capsule-capsule keeps (static, free), capsule-sphere becomes (sphere, static)
    geoms, sign = ((0, 1), 1.0) if kind == "capsule_capsule" else ((1, 0), -1.0)
    o = Oracle(m)
    for body in bodies:
        dist, n, pos = _expect(*cf(body))
        assert -0.05 < dist < 0
        a = state_arrays(m, o.forward(o.new_state(_qpos(m, body))))
        assert a["ncon"] == 1 and tuple(a["con_geom"][0]) == geoms
        assert a["con_dist"][0] == pytest.approx(dist, abs=1e-6)
        np.testing.assert_allclose(a["con_frame"][0][:3], sign * n, atol=1e-5)
        np.testing.assert_allclose(a["con_pos"][0], pos, atol=1e-6)
        # the free body is pushed out along n, with torque (pos - origin) x F
        f = a["qfrc_constraint"]
        assert f[:3] @ n > 0
        np.testing.assert_allclose(f[:3] / np.linalg.norm(f[:3]), n, atol=1e-5)
        np.testing.assert_allclose(f[3:6], np.cross(pos - body, f[:3]), atol=1e-6 * np.linalg.norm(f[:3]))
        a = state_arrays(m, o.forward(o.new_state(_qpos(m, _clear(body, cf)))))
        assert a["ncon"] == 0 or a["con_dist"][0] > 0


# ---- the same KATs on the HIP kernel ---------------------------------------------------------

def _gpu_rollout_slope_accel(theta_deg, mu, body_geom, diag=False, settle=500, nstep=1500):
    import torch
    from mjx_amd import mjx
    xml, d = _incline_xml(theta_deg, mu, body_geom, diag)
    m = mjcf.compile_xml_string(xml)
    sys_ = mjx.put_model(m)
    data = mjx.make_data(sys_, 2)
    for _ in range(settle):
        mjx.step(sys_, data)
    v0 = data.get("qvel").cpu().numpy()[:, :3].astype(np.float64) @ d
    for _ in range(nstep - settle):
        mjx.step(sys_, data)
    torch.cuda.synchronize()
    v1 = data.get("qvel").cpu().numpy()[:, :3].astype(np.float64) @ d
    return (v1 - v0) / ((nstep - settle) * DT), v1


@pytest.mark.gpu
def test_friction_kats_on_gpu():
    """The incline KATs above through libmjx355.so (fp32): same closed forms, same tolerances."""
    for theta, slides in ((26.5, False), (27.0, True), (35.0, True)):
        a, v = _gpu_rollout_slope_accel(theta, 0.5, CAPSULE_X)
        if slides:
            np.testing.assert_allclose(a, _slide(theta, 0.5), rtol=0.03, atol=5e-3)
        else:
            assert np.all(np.abs(v) < 0.01) and np.all(np.abs(a) < 1e-3)
    a, _ = _gpu_rollout_slope_accel(30.0, 1.0, SPHERE)
    np.testing.assert_allclose(a, 5.0 / 7.0 * G * 0.5, rtol=5e-3)
    for diag in (False, True):
        a, _ = _gpu_rollout_slope_accel(30.0, 0.1, SPHERE, diag=diag)
        np.testing.assert_allclose(a, _slide(30.0, 0.1 / np.sqrt(2.0) if diag else 0.1), rtol=5e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["capsule_capsule", "capsule_sphere"])
def test_segment_contact_geometry_on_gpu(kind):
    """Contact count switches at the closed-form distance (-/+1e-4 around touching), and the force on
    the free body is along the closed-form normal with the torque of the closed-form position."""
    import torch
    from mjx_amd import mjx
    m, bodies, cf = (_cc_model(), CC_BODIES, _cc_closed_form) if kind == "capsule_capsule" else \
        (_cs_model(), CS_BODIES, _cs_closed_form)
    poses = []
    for body in bodies:
        poses += [body, _clear(body, cf, eps=1e-4), _clear(body, cf, eps=-1e-4)]
    sys_ = mjx.put_model(m)
    d = mjx.make_data(sys_, len(poses))
    d.set("qpos", torch.tensor(np.array([_qpos(m, b) for b in poses]), dtype=torch.float32))
    mjx.forward(sys_, d)
    st = d.get("stats").cpu().numpy()
    qf = d.get("qfrc_constraint").cpu().numpy().astype(np.float64)
    for i, body in enumerate(poses):
        dist, n, pos = _expect(*cf(body))
        assert st[i][0] == (1 if dist < 0 else 0), f"pose {i}: dist {dist:.2e}, ncon {st[i][0]}"
        if dist < -1e-3:
            f = qf[i]
            np.testing.assert_allclose(f[:3] / np.linalg.norm(f[:3]), n, atol=2e-4)
            np.testing.assert_allclose(f[3:6], np.cross(pos - body, f[:3]), atol=2e-4 * np.linalg.norm(f[:3]))

"""MJCF compiler KATs (CPU). The compiled constants feed both the product and the oracle, so they
are pinned here by independent closed forms and the structural facts of SURVEY.md §4/§8."""
import math
import os

import numpy as np
import pytest

import mjx_amd
from mjx_amd import mjcf

REF_MODELS = "/root/reference/models"


@pytest.fixture(scope="module", params=["humanoid_mjx", "humanoid"])
def model(request):
    return mjx_amd.load_model(request.param)


def test_sizes(model):
    assert (model.nq, model.nv, model.nu, model.nbody, model.njnt, model.ngeom) == (28, 27, 21, 17, 22, 20)
    assert model.ntendon == 2 and model.nsensor == 2 and model.nkey == 5
    assert model.name2id("body", "pelvis") == 4 and model.name2id("body", "head") == 2


def test_pair_counts():
    m1 = mjx_amd.load_model("humanoid_mjx")
    m2 = mjx_amd.load_model("humanoid")
    assert m1.npair == 108  # 108 candidate pairs after contype/conaffinity masks
    kinds = np.bincount(m1.pair_kind, minlength=5)
    assert kinds[mjcf.COL_PLANE_CAPSULE] == 8 and kinds[mjcf.COL_CAPSULE_CAPSULE] == 76
    assert kinds[mjcf.COL_SPHERE_CAPSULE] == 24
    # humanoid.xml: all-collide masks; weld (head->torso, hand->forearm) and parent filtering apply
    assert m2.npair == 159
    assert sum(mjcf.COL_NCON[k] for k in m1.pair_kind) == 116


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference models not mounted")
def test_humanoid_xml_pair_filter_by_mujoco_rules():
    """humanoid.xml's 159 candidate pairs, derived here from the XML's body tree (xml.etree, not the
    compiler) by MuJoCo's documented filter (Modeling > Contact > Selection): of C(20,2) = 190 geom
    pairs drop (1) pairs inside one weld body (a body without joints is welded to its parent: head
    to torso, hands to lower arms) — 3 same-body + 4 same-weld; (2) parent-child weld bodies
    ("filterparent": weld(b1) == weld(parent(weld(b2))) or vice versa) — 17 direct parent-child +
    the 5 below that only the weld makes parent-child; (3) the two <exclude> pairs; contype/
    conaffinity are the defaults (1/1) and keep everything else: 190 - 7 - 22 - 2 = 159. SURVEY.md
    §8's 164 omitted the 5 weld-parent pairs."""
    import xml.etree.ElementTree as ET
    root = ET.parse(os.path.join(REF_MODELS, "humanoid.xml")).getroot()
    parent, has_joint, geoms = {"world": None}, {"world": False}, []

    def walk(el, body):
        for ch in el:
            if ch.tag == "body":
                name = ch.get("name")
                parent[name] = body
                has_joint[name] = any(c.tag in ("joint", "freejoint") for c in ch)
                walk(ch, name)
            elif ch.tag == "geom":
                geoms.append((ch.get("name"), body))
    walk(root.find("worldbody"), "world")
    weld = lambda b: b if b == "world" or has_joint[b] else weld(parent[b])  # noqa: E731
    excl = {frozenset((e.get("body1"), e.get("body2"))) for e in root.find("contact") if e.tag == "exclude"}
    assert len(geoms) == 20 and len(excl) == 2
    kept, weld_parent = set(), set()
    for i in range(20):
        for j in range(i + 1, 20):
            (g1, b1), (g2, b2) = geoms[i], geoms[j]
            w1, w2 = weld(b1), weld(b2)
            if w1 == w2:
                continue
            if w1 != "world" and w2 != "world" and (w1 == weld(parent[w2]) or w2 == weld(parent[w1])):
                if parent[b1] != b2 and parent[b2] != b1:
                    weld_parent.add(frozenset((b1, b2)))
                continue
            if frozenset((b1, b2)) in excl:
                continue
            kept.add(frozenset((g1, g2)))
    assert weld_parent == {frozenset(p) for p in (("head", "waist_lower"), ("head", "upper_arm_right"),
                                                  ("head", "upper_arm_left"), ("upper_arm_right", "hand_right"),
                                                  ("upper_arm_left", "hand_left"))}
    assert len(kept) == 159
    m = mjx_amd.load_model("humanoid")
    gn = m.names["geom"]
    assert {frozenset((gn[a], gn[b])) for a, b in zip(m.pair_geom1, m.pair_geom2)} == kept


def _capsule(r, h, rho=1000.0):
    mc = rho * math.pi * r * r * h
    ms = rho * 4.0 / 3.0 * math.pi * r ** 3
    return mc + ms


def test_masses_closed_form():
    m = mjx_amd.load_model("humanoid_mjx")
    # torso body holds the torso + waist_upper capsules; head is its own (welded) body
    assert m.body_mass[1] == pytest.approx(_capsule(0.07, 0.14) + _capsule(0.06, 0.12), rel=1e-12)
    assert m.body_mass[2] == pytest.approx(1000 * 4 / 3 * math.pi * 0.09 ** 3, rel=1e-12)
    shin = _capsule(0.049, 0.3)
    assert m.body_mass[m.name2id("body", "shin_right")] == pytest.approx(shin, rel=1e-12)
    assert m.body_mass.sum() == pytest.approx(40.84402122, rel=1e-8)


def test_inertia_spd_and_qpos0(model):
    for b in range(1, model.nbody):
        t = model.body_inertia[b]
        I = np.array([[t[0], t[3], t[4]], [t[3], t[1], t[5]], [t[4], t[5], t[2]]])
        ev = np.linalg.eigvalsh(I)
        assert ev.min() > 0
        assert ev[0] + ev[1] >= ev[2] * (1 - 1e-9)  # triangle inequality of principal moments
    q0 = model.qpos0
    assert q0[2] == pytest.approx(1.282) and list(q0[3:7]) == [1, 0, 0, 0] and np.all(q0[7:] == 0)


def test_joint_ranges_radians(model):
    j = model.name2id("joint", "knee_right")
    assert model.jnt_range[j] == pytest.approx(np.deg2rad([-160, 2]))
    assert model.jnt_limited[j] == 1


def test_contact_mixing():
    m = mjx_amd.load_model("humanoid_mjx")
    floor = m.name2id("geom", "floor")
    p = [i for i in range(m.npair) if m.pair_geom1[i] == floor][0]
    assert m.pair_condim[p] == 3
    assert m.pair_solref[p] == pytest.approx([0.0175, 1.0])
    assert m.pair_solimp[p][:3] == pytest.approx([0.9, 0.97, 0.002])
    assert m.pair_friction[p][0] == pytest.approx(1.0)


def test_invweight_and_meaninertia(model):
    assert np.all(model.body_invweight0[1:] > 0)
    kin = mjcf._fk_and_mass(model, model.qpos0)
    M = kin["M"]
    assert np.allclose(M, M.T) and np.linalg.eigvalsh(M).min() > 0
    assert model.meaninertia == pytest.approx(np.trace(M) / model.nv)


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference models not mounted")
def test_assets_match_fresh_compile():
    for name in mjx_amd.BUILTIN_MODELS:
        fresh = mjcf.compile_xml(os.path.join(REF_MODELS, name + ".xml"))
        asset = mjx_amd.load_model(name)
        assert asset.source_sha256 == fresh.source_sha256
        for k, v in fresh.arrays.items():
            np.testing.assert_array_equal(asset.arrays[k], v, err_msg=k)


def test_unsupported_rejected():
    xml = """<mujoco><worldbody><body><freejoint/><geom type="box" size=".1 .1 .1"/></body></worldbody></mujoco>"""
    with pytest.raises(mjcf.MJCFError):
        mjcf.compile_xml_string(xml)
    xml2 = """<mujoco><option solver="PGS"/><worldbody/></mujoco>"""
    with pytest.raises(mjcf.MJCFError):
        mjcf.compile_xml_string(xml2)


def test_flip_tables_involution():
    from mjx_amd import abi
    from mjx_amd.config import reference_ppo_config
    cfg = reference_ppo_config().env_config
    ap, asg, op, osg = abi.flip_tables(cfg, 21, 54)
    assert np.array_equal(ap[ap], np.arange(21)) and np.array_equal(op[op], np.arange(54))
    # flipping twice is the identity on values (sign of a permuted entry is consistent)
    x = np.random.default_rng(0).normal(size=54)
    y = x[op] * osg
    z = y[op] * osg
    assert np.allclose(z, x)


def test_explicit_geom_mass_sets_density():
    """mjx_humanoid_speed_test.py:29-40's SPHERE model gives its geom mass="1": MuJoCo then takes
    density = mass / volume (mjCGeom::SetInertia), so body mass 1 and inertia 2/5 m r^2."""
    from mjx_amd import mjcf
    m = mjcf.compile_xml_string("<mujoco><worldbody><body><freejoint/><geom size='.15' mass='1' type='sphere'/>"
                                "</body></worldbody></mujoco>")
    assert m.body_mass[1] == pytest.approx(1.0, rel=1e-12)
    assert m.body_inertia[1][:3] == pytest.approx([0.4 * 0.15 ** 2] * 3, rel=1e-12)


def test_geom_mass_on_worldbody_plane_is_ignored():
    """a worldbody plane with a mass attribute (legal MJCF, MuJoCo ignores it) compiles; a
    zero-volume geom with an explicit mass is a clear compile error, not a ZeroDivisionError."""
    from mjx_amd import mjcf
    m = mjcf.compile_xml_string("<mujoco><worldbody><geom type='plane' size='5 5 .1' mass='3'/>"
                                "<body><freejoint/><geom size='.15' mass='1' type='sphere'/></body></worldbody>"
                                "</mujoco>")
    assert m.body_mass[1] == pytest.approx(1.0, rel=1e-12)
    with pytest.raises(mjcf.MJCFError, match="zero volume"):
        mjcf.compile_xml_string("<mujoco><worldbody><body><freejoint/><geom size='0' mass='1' type='sphere'/>"
                                "</body></worldbody></mujoco>")

"""The maintainer-side MjModel -> descriptor path (mjx_amd/mjmodel.py; VERDICT r2 item 9: the reference
holds a mujoco.MjModel, src/training_utils.py:80,105, and INTEGRATION.md promised a descriptor filled
from its fields).

`mujoco` is not importable here, so the filler runs on an MjModel-shaped view of this
package's compiler output — MuJoCo's attribute names and layouts (principal inertia + body_iquat,
[nu, 2] trnid, [nu, 6] gear, wrap arrays, exclude_signature, opt / stat) — and must reproduce the
descriptor the compiler itself produces, field for field. The same check against a real MjModel runs
where mujoco is installed."""
import types

import numpy as np
import pytest

import mjx_amd
from mjx_amd import abi, mjcf
from mjx_amd.mjmodel import compile_mjmodel

# MuJoCo's enum values (mjmodel.h, 3.3) — the filler reads them from the module it is given
_E = {
    "mjtObj": {"mjOBJ_BODY": 1, "mjOBJ_JOINT": 3, "mjOBJ_GEOM": 5, "mjOBJ_SITE": 6, "mjOBJ_ACTUATOR": 19,
               "mjOBJ_TENDON": 18, "mjOBJ_SENSOR": 20, "mjOBJ_TUPLE": 23, "mjOBJ_KEY": 24},
    "mjtCone": {"mjCONE_PYRAMIDAL": 0, "mjCONE_ELLIPTIC": 1},
    "mjtSolver": {"mjSOL_PGS": 0, "mjSOL_CG": 1, "mjSOL_NEWTON": 2},
    "mjtIntegrator": {"mjINT_EULER": 0, "mjINT_RK4": 1, "mjINT_IMPLICIT": 2, "mjINT_IMPLICITFAST": 3},
    "mjtDisableBit": {"mjDSBL_FILTERPARENT": 1 << 10, "mjDSBL_EULERDAMP": 1 << 15},
    "mjtJoint": {"mjJNT_FREE": 0, "mjJNT_BALL": 1, "mjJNT_SLIDE": 2, "mjJNT_HINGE": 3},
    "mjtGeom": {"mjGEOM_PLANE": 0, "mjGEOM_SPHERE": 2, "mjGEOM_CAPSULE": 3, "mjGEOM_BOX": 6},
    "mjtTrn": {"mjTRN_JOINT": 0}, "mjtDyn": {"mjDYN_NONE": 0}, "mjtGain": {"mjGAIN_FIXED": 0},
    "mjtBias": {"mjBIAS_NONE": 0}, "mjtWrap": {"mjWRAP_JOINT": 1}, "mjtSensor": {"mjSENS_TOUCH": 0},
}
_OBJ_KIND = {1: "body", 3: "joint", 5: "geom", 6: "site", 19: "actuator", 18: "tendon", 20: "sensor", 24: "key"}


def _mat2quat(R):
    w = np.sqrt(max(0.0, 1.0 + R[0, 0] + R[1, 1] + R[2, 2])) / 2.0
    x = np.copysign(np.sqrt(max(0.0, 1.0 + R[0, 0] - R[1, 1] - R[2, 2])) / 2.0, R[2, 1] - R[1, 2])
    y = np.copysign(np.sqrt(max(0.0, 1.0 - R[0, 0] + R[1, 1] - R[2, 2])) / 2.0, R[0, 2] - R[2, 0])
    z = np.copysign(np.sqrt(max(0.0, 1.0 - R[0, 0] - R[1, 1] + R[2, 2])) / 2.0, R[1, 0] - R[0, 1])
    q = np.array([w, x, y, z])
    return q / np.linalg.norm(q)


def _fake_mujoco(m):
    mod = types.SimpleNamespace(**{k: types.SimpleNamespace(**v) for k, v in _E.items()})
    mod.mj_id2name = lambda mj, obj, i: m.names[_OBJ_KIND[obj]][i] or None
    return mod


def _mjmodel_view(m):
    """The MjModel attributes mujoco would expose for this model (MuJoCo's names and layouts)."""
    A = m.arrays
    v = types.SimpleNamespace()
    v.opt = types.SimpleNamespace(timestep=m.timestep, gravity=m.gravity, impratio=m.impratio, tolerance=m.tolerance,
                                  ls_tolerance=m.ls_tolerance, iterations=m.iterations, ls_iterations=m.ls_iterations,
                                  solver=m.solver, integrator=m.integrator, cone=0,
                                  disableflags=0 if m.eulerdamp else 1 << 15, enableflags=0)
    v.stat = types.SimpleNamespace(meaninertia=m.meaninertia)
    for k in ("nq", "nv", "nu", "nbody", "njnt", "ngeom", "nsite", "ntendon", "nsensor", "nsensordata", "nkey"):
        setattr(v, k, getattr(m, k))
    v.npair = v.neq = v.nmocap = v.nhfield = v.nmesh = v.na = 0
    for k, x in A.items():
        setattr(v, k, x)
    # principal inertia in body_iquat (mj_setConst's representation)
    pri, iq = np.zeros((m.nbody, 3)), np.zeros((m.nbody, 4))
    for b in range(m.nbody):
        xx, yy, zz, xy, xz, yz = A["body_inertia"][b]
        I = np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]])
        w, R = np.linalg.eigh(I)
        if np.linalg.det(R) < 0:
            R[:, 0] = -R[:, 0]
        pri[b], iq[b] = w, _mat2quat(R)
    v.body_inertia, v.body_iquat = pri, iq
    nu = m.nu
    v.actuator_trnid = np.stack([A["actuator_trnid"], -np.ones(nu, np.int32)], 1)
    v.actuator_gear = np.zeros((nu, 6))
    v.actuator_gear[:, 0] = A["actuator_gear"]
    v.actuator_trntype = v.actuator_dyntype = v.actuator_gaintype = v.actuator_biastype = np.zeros(nu, np.int32)
    v.actuator_gainprm = np.zeros((nu, 10))
    v.actuator_gainprm[:, 0] = 1.0
    adr, wt, wo, wp = [], [], [], []
    for t in range(m.ntendon):
        adr.append(len(wt))
        for w in range(A["tendon_num"][t]):
            wt.append(1)
            wo.append(A["tendon_jnt"][t, w])
            wp.append(A["tendon_coef"][t, w])
    v.tendon_adr, v.wrap_type, v.wrap_objid, v.wrap_prm = (np.array(x) for x in (adr, wt, wo, wp))
    v.tendon_stiffness = v.tendon_damping = np.zeros(m.ntendon)
    v.tendon_solref_lim, v.tendon_solimp_lim = A["tendon_solref"], A["tendon_solimp"]
    v.site_type = np.full(m.nsite, 6, np.int32)  # box sites (the humanoids' foot sensor zones)
    v.jnt_type = A["jnt_type"]
    return v


def _desc_fields(d):
    return {name: np.array(getattr(d, name)) if not isinstance(getattr(d, name), (int, float))
            else np.array(getattr(d, name)) for name, _ in abi.ModelDesc._fields_}


@pytest.mark.parametrize("name", ["humanoid_mjx", "humanoid"])
def test_descriptor_from_mjmodel_fields_matches_compiler(name):
    m = mjx_amd.load_model(name)
    if name == "humanoid":
        assert m.eulerdamp == 1  # Euler with eulerdamp: the disable flag round-trips
    got = compile_mjmodel(_mjmodel_view(m), _fake_mujoco(m))
    want_d, got_d = _desc_fields(abi.model_desc(m)), _desc_fields(abi.model_desc(got))
    for k, w in want_d.items():
        # body_inertia went through this view's eigen-decomposition + quaternion (~1e-10)
        tol = 1e-9 if k == "body_inertia" else 1e-12
        np.testing.assert_allclose(got_d[k], w, rtol=tol, atol=tol, err_msg=k)
    assert got.npair == m.npair and got.name2id("body", "pelvis") == m.name2id("body", "pelvis")
    assert got.name2id("sensor", "touch_foot_left") == m.name2id("sensor", "touch_foot_left")


def test_mjmodel_filler_rejects_unsupported_features():
    m = mjx_amd.load_model("humanoid_mjx")
    v = _mjmodel_view(m)
    v.opt.cone = 1
    with pytest.raises(mjcf.MJCFError, match="pyramidal"):
        compile_mjmodel(v, _fake_mujoco(m))
    v = _mjmodel_view(m)
    v.jnt_type = v.jnt_type.copy()
    v.jnt_type[3] = 2  # slide
    with pytest.raises(mjcf.MJCFError, match="hinge"):
        compile_mjmodel(v, _fake_mujoco(m))
    v = _mjmodel_view(m)
    v.neq = 1
    with pytest.raises(mjcf.MJCFError, match="neq"):
        compile_mjmodel(v, _fake_mujoco(m))


def test_descriptor_from_real_mjmodel():
    """Where mujoco is installed: the reference's own MjModel gives the compiler's descriptor."""
    mujoco = pytest.importorskip("mujoco")
    import os
    path = os.environ.get("MJL_REFERENCE_XML", "")
    if not os.path.exists(path):
        pytest.skip("set MJL_REFERENCE_XML to models/humanoid_mjx.xml of the reference")
    got = compile_mjmodel(mujoco.MjModel.from_xml_path(path), mujoco)
    want = mjcf.compile_xml(path)
    for k, w in _desc_fields(abi.model_desc(want)).items():
        np.testing.assert_allclose(_desc_fields(abi.model_desc(got))[k], w, rtol=1e-6, atol=1e-9, err_msg=k)

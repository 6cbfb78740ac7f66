"""CompiledModel (and so the C descriptor, abi.model_desc) from a MuJoCo `MjModel`: the maintainer-side
path for the reference, which already holds one (`mujoco.MjModel.from_xml_path`,
src/training_utils.py:80; mjx.put_model(mj_model), :105). Needs the `mujoco` Python bindings, which
this image lacks; `tests/test_mjmodel.py` runs it on an MjModel-shaped view of this
package's own compiler output, and the real-mujoco check there is skipped when `mujoco` is absent.

Every descriptor field maps to the MjModel attribute of the same name, except:
  * body_inertia: MjModel keeps principal moments `body_inertia` in the frame `body_iquat`; the
    descriptor holds the full tensor in the body frame, R(iquat) diag(I) R(iquat)^T;
  * body_subtree_end / body_level: derived from body_parentid (bodies are in depth-first order);
  * pair_*: MJX's collision candidates are not MjModel arrays (explicit <pair>s are rejected); they
    come from the geoms' contype / conaffinity / condim / friction / solref / solimp / solmix /
    margin / gap, the weld tree and `exclude_signature`, by mjcf.candidate_pairs;
  * actuator_trnid / actuator_gear: column 0 of MuJoCo's [nu, 2] / [nu, 6];
  * tendon_jnt / tendon_coef: the joint wraps (wrap_objid / wrap_prm) from tendon_adr;
  * tendon_solref / tendon_solimp: MuJoCo's tendon_solref_lim / tendon_solimp_lim;
  * options: opt.timestep / gravity / impratio / tolerance / ls_tolerance / iterations /
    ls_iterations / solver / integrator, eulerdamp = not (opt.disableflags & mjDSBL_EULERDAMP),
    meaninertia = stat.meaninertia; the invweight0 arrays are MuJoCo's own (mj_setConst).
Anything outside the kernels' feature set (ball / slide joints, non-motor actuators, non-touch
sensors, elliptic cones, equality constraints, other geom types, ...) raises MJCFError, as the MJCF
compiler does.
"""
from __future__ import annotations

import numpy as np

from . import mjcf
from .mjcf import CompiledModel, MJCFError


def _quat2mat(q):
    return mjcf.quat2mat(np.asarray(q, np.float64))


def _enum(mujoco, enum_name: str, member: str) -> int:
    return int(getattr(getattr(mujoco, enum_name), member))


def _name(mujoco, mj, obj: str, i: int) -> str:
    n = mujoco.mj_id2name(mj, _enum(mujoco, "mjtObj", obj), i)
    return n or ""


def compile_mjmodel(mj, mujoco=None) -> CompiledModel:
    """CompiledModel from a mujoco.MjModel (`mujoco`: the bindings module, imported when None)."""
    if mujoco is None:
        import mujoco  # noqa: F401  (the maintainer's environment; absent here)
    E = lambda e, m: _enum(mujoco, e, m)  # noqa: E731
    opt = mj.opt
    if int(opt.cone) != E("mjtCone", "mjCONE_PYRAMIDAL"):
        raise MJCFError("only pyramidal cones supported")
    solver = int(opt.solver)
    if solver not in (E("mjtSolver", "mjSOL_CG"), E("mjtSolver", "mjSOL_NEWTON")):
        raise MJCFError("only the CG and Newton solvers are supported")
    integ = int(opt.integrator)
    if integ not in (E("mjtIntegrator", "mjINT_EULER"), E("mjtIntegrator", "mjINT_IMPLICITFAST")):
        raise MJCFError("only Euler and implicitfast integrators supported")
    eulerdamp_bit = E("mjtDisableBit", "mjDSBL_EULERDAMP")
    filterparent_bit = E("mjtDisableBit", "mjDSBL_FILTERPARENT")
    if int(opt.disableflags) & ~(eulerdamp_bit | filterparent_bit) or int(opt.enableflags):
        raise MJCFError("option flags other than eulerdamp / filterparent not supported")
    for k in ("neq", "npair", "nmocap", "nhfield", "nmesh", "na"):
        if int(getattr(mj, k, 0)):
            raise MJCFError(f"{k} > 0 not supported")

    m = CompiledModel(name="mjmodel")
    m.timestep, m.gravity = float(opt.timestep), np.array(opt.gravity, np.float64)
    m.impratio, m.tolerance, m.ls_tolerance = float(opt.impratio), float(opt.tolerance), float(opt.ls_tolerance)
    m.iterations, m.ls_iterations = int(opt.iterations), int(opt.ls_iterations)
    m.solver = mjcf.SOLVER_CG if solver == E("mjtSolver", "mjSOL_CG") else mjcf.SOLVER_NEWTON
    m.integrator = mjcf.INT_EULER if integ == E("mjtIntegrator", "mjINT_EULER") else mjcf.INT_IMPLICITFAST
    m.eulerdamp = 0 if int(opt.disableflags) & eulerdamp_bit else 1
    m.meaninertia = float(mj.stat.meaninertia)

    nbody, njnt, ngeom, nsite, nu = int(mj.nbody), int(mj.njnt), int(mj.ngeom), int(mj.nsite), int(mj.nu)
    nq, nv, ntendon, nsensor = int(mj.nq), int(mj.nv), int(mj.ntendon), int(mj.nsensor)
    a = lambda k, dt=np.float64: np.array(getattr(mj, k), dt)  # noqa: E731
    A = {}
    # ---- bodies
    parent = a("body_parentid", np.int32)
    A["body_parentid"] = parent
    for k in ("body_rootid", "body_weldid", "body_jntadr", "body_jntnum", "body_dofadr", "body_dofnum"):
        A[k] = a(k, np.int32)
    level = np.zeros(nbody, np.int32)
    end = np.arange(1, nbody + 1, dtype=np.int32)
    for b in range(1, nbody):
        level[b] = level[parent[b]] + 1
    for b in range(nbody - 1, 0, -1):  # depth-first order: a subtree is [b, end[b])
        end[parent[b]] = max(end[parent[b]], end[b])
    A["body_subtree_end"], A["body_level"] = end, level
    A["body_pos"], A["body_quat"], A["body_ipos"] = a("body_pos"), a("body_quat"), a("body_ipos")
    inert = np.zeros((nbody, 6))
    iq, pri = a("body_iquat").reshape(nbody, 4), a("body_inertia").reshape(nbody, 3)
    for b in range(nbody):
        R = _quat2mat(iq[b])
        I = R @ np.diag(pri[b]) @ R.T
        inert[b] = [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]
    A["body_inertia"], A["body_mass"] = inert, a("body_mass")
    A["body_invweight0"] = a("body_invweight0").reshape(nbody, 2)
    # ---- joints / dofs
    jt = a("jnt_type", np.int32)
    free, hinge = E("mjtJoint", "mjJNT_FREE"), E("mjtJoint", "mjJNT_HINGE")
    if np.any((jt != free) & (jt != hinge)):
        raise MJCFError("only free and hinge joints supported")
    A["jnt_type"] = np.where(jt == free, mjcf.JNT_FREE, mjcf.JNT_HINGE).astype(np.int32)
    for k in ("jnt_qposadr", "jnt_dofadr", "jnt_bodyid", "jnt_limited"):
        A[k] = a(k, np.int32)
    for k in ("jnt_pos", "jnt_axis", "jnt_range", "jnt_stiffness", "jnt_margin", "jnt_solref", "jnt_solimp"):
        A[k] = a(k)
    for k in ("dof_bodyid", "dof_jntid", "dof_parentid"):
        A[k] = a(k, np.int32)
    for k in ("dof_damping", "dof_armature", "dof_invweight0", "qpos0", "qpos_spring"):
        A[k] = a(k)
    # ---- geoms and the collision candidates
    gtype = a("geom_type", np.int32)
    gmap = {E("mjtGeom", "mjGEOM_PLANE"): mjcf.GEOM_PLANE, E("mjtGeom", "mjGEOM_SPHERE"): mjcf.GEOM_SPHERE,
            E("mjtGeom", "mjGEOM_CAPSULE"): mjcf.GEOM_CAPSULE}
    if any(int(t) not in gmap for t in gtype):
        raise MJCFError("only plane / sphere / capsule geoms supported")
    A["geom_type"] = np.array([gmap[int(t)] for t in gtype], np.int32)
    for k in ("geom_bodyid", "geom_contype", "geom_conaffinity", "geom_condim"):
        A[k] = a(k, np.int32)
    for k in ("geom_pos", "geom_quat", "geom_size", "geom_friction"):
        A[k] = a(k)
    solref, solimp, solmix = a("geom_solref"), a("geom_solimp"), a("geom_solmix")
    margin, gap, prio = a("geom_margin"), a("geom_gap"), a("geom_priority", np.int32)
    geoms = [{"type": int(A["geom_type"][g]), "body": int(A["geom_bodyid"][g]), "contype": int(A["geom_contype"][g]),
              "conaffinity": int(A["geom_conaffinity"][g]), "condim": int(A["geom_condim"][g]),
              "friction": A["geom_friction"][g], "solref": list(solref[g]), "solimp": list(solimp[g]),
              "solmix": float(solmix[g]), "margin": float(margin[g]), "gap": float(gap[g]), "priority": int(prio[g])}
             for g in range(ngeom)]
    sig = np.array(getattr(mj, "exclude_signature", []), np.int64).reshape(-1)
    excludes = {(min(int(s) >> 16, int(s) & 0xFFFF), max(int(s) >> 16, int(s) & 0xFFFF)) for s in sig}
    pairs = mjcf.candidate_pairs(geoms, parent, A["body_weldid"], excludes,
                                 filterparent=not (int(opt.disableflags) & filterparent_bit))
    A["pair_geom1"] = np.array([p["g1"] for p in pairs], np.int32)
    A["pair_geom2"] = np.array([p["g2"] for p in pairs], np.int32)
    A["pair_kind"] = np.array([p["kind"] for p in pairs], np.int32)
    A["pair_condim"] = np.array([p["condim"] for p in pairs], np.int32)
    A["pair_friction"] = np.array([p["friction"] for p in pairs]).reshape(-1, 5)
    A["pair_solref"] = np.array([p["solref"] for p in pairs]).reshape(-1, 2)
    A["pair_solimp"] = np.array([p["solimp"] for p in pairs]).reshape(-1, 5)
    A["pair_margin"] = np.array([p["margin"] for p in pairs])
    A["pair_gap"] = np.array([p["gap"] for p in pairs])
    # ---- sites
    stype = a("site_type", np.int32)
    smap = {E("mjtGeom", "mjGEOM_BOX"): mjcf.GEOM_BOX, E("mjtGeom", "mjGEOM_SPHERE"): mjcf.GEOM_SPHERE,
            E("mjtGeom", "mjGEOM_CAPSULE"): mjcf.GEOM_CAPSULE}
    A["site_type"] = np.array([smap.get(int(t), -1) for t in stype], np.int32)
    A["site_bodyid"] = a("site_bodyid", np.int32)
    A["site_pos"], A["site_quat"], A["site_size"] = a("site_pos"), a("site_quat"), a("site_size")
    # ---- actuators: motors on hinge joints (gain 1, no bias, no dynamics)
    if nu:
        if np.any(a("actuator_trntype", np.int32) != E("mjtTrn", "mjTRN_JOINT")) \
                or np.any(a("actuator_dyntype", np.int32) != E("mjtDyn", "mjDYN_NONE")) \
                or np.any(a("actuator_gaintype", np.int32) != E("mjtGain", "mjGAIN_FIXED")) \
                or np.any(a("actuator_biastype", np.int32) != E("mjtBias", "mjBIAS_NONE")) \
                or np.any(a("actuator_gainprm").reshape(nu, -1)[:, 0] != 1.0):
            raise MJCFError("only motor actuators (joint transmission) supported")
    A["actuator_trnid"] = a("actuator_trnid", np.int32).reshape(nu, 2)[:, 0].copy()
    A["actuator_gear"] = a("actuator_gear").reshape(nu, 6)[:, 0].copy()
    A["actuator_ctrlrange"] = a("actuator_ctrlrange").reshape(nu, 2)
    A["actuator_ctrllimited"] = a("actuator_ctrllimited", np.int32)
    # ---- fixed tendons over joints
    tadr, tnum = a("tendon_adr", np.int32), a("tendon_num", np.int32)
    maxw = max([int(n) for n in tnum] + [1])
    tj, tc = np.full((ntendon, maxw), -1, np.int32), np.zeros((ntendon, maxw))
    if ntendon:
        wtype, wobj, wprm = a("wrap_type", np.int32), a("wrap_objid", np.int32), a("wrap_prm")
        if np.any(a("tendon_stiffness") != 0) or np.any(a("tendon_damping") != 0):
            raise MJCFError("tendon stiffness/damping not supported")
        for t in range(ntendon):
            for w in range(int(tnum[t])):
                i = int(tadr[t]) + w
                if int(wtype[i]) != E("mjtWrap", "mjWRAP_JOINT"):
                    raise MJCFError("only joint wraps supported in fixed tendons")
                tj[t, w], tc[t, w] = int(wobj[i]), float(wprm[i])
    A["tendon_num"], A["tendon_jnt"], A["tendon_coef"] = tnum, tj, tc
    A["tendon_limited"] = a("tendon_limited", np.int32)
    A["tendon_range"] = a("tendon_range").reshape(ntendon, 2)
    A["tendon_margin"] = a("tendon_margin")
    A["tendon_solref"] = a("tendon_solref_lim").reshape(ntendon, 2)
    A["tendon_solimp"] = a("tendon_solimp_lim").reshape(ntendon, 5)
    A["tendon_invweight0"] = a("tendon_invweight0")
    # ---- touch sensors on box sites
    st = a("sensor_type", np.int32)
    if np.any(st != E("mjtSensor", "mjSENS_TOUCH")):
        raise MJCFError("only touch sensors supported")
    A["sensor_type"] = np.full(nsensor, mjcf.SENS_TOUCH, np.int32)
    A["sensor_objid"], A["sensor_adr"] = a("sensor_objid", np.int32), a("sensor_adr", np.int32)
    if any(A["site_type"][s] != mjcf.GEOM_BOX for s in A["sensor_objid"]):
        raise MJCFError("touch sensor requires a box site")
    A["key_qpos"] = a("key_qpos").reshape(-1, nq)

    m.arrays = A
    m.names = {kind: [_name(mujoco, mj, obj, i) for i in range(n)] for kind, obj, n in (
        ("body", "mjOBJ_BODY", nbody), ("joint", "mjOBJ_JOINT", njnt), ("geom", "mjOBJ_GEOM", ngeom),
        ("site", "mjOBJ_SITE", nsite), ("actuator", "mjOBJ_ACTUATOR", nu), ("tendon", "mjOBJ_TENDON", ntendon),
        ("sensor", "mjOBJ_SENSOR", nsensor), ("key", "mjOBJ_KEY", int(mj.nkey)))}
    m.nq, m.nv, m.nu = nq, nv, nu
    m.nbody, m.njnt, m.ngeom, m.nsite = nbody, njnt, ngeom, nsite
    m.ntendon, m.npair, m.nsensor = ntendon, len(pairs), nsensor
    m.nsensordata, m.nkey = int(mj.nsensordata), int(mj.nkey)
    return m

"""MJCF -> compiled model constants (host side, float64).

Restates the subset of MuJoCo 3.3.6's model compiler (`mujoco.MjModel.from_xml_path`, called at
reference `src/training_utils.py:80` and `mjx_humanoid_speed_test.py:25,28`) that the two
reference humanoid models use (`models/humanoid_mjx.xml`, `models/humanoid.xml`):

* `<default>` class trees, `childclass`, per-element `class`
* bodies with `pos` (no body quat in the models; `quat` still honoured), `freejoint`, hinge joints
* capsule (`fromto` or `size`), sphere and plane geoms; `zaxis`/`quat` orientation
* inertia from geoms (density 1000, exact capsule/sphere formulas), combined per body
* contype/conaffinity, parent filtering, `<contact><exclude>`, contact-parameter mixing
* limited hinges (degrees -> radians), armature/damping/stiffness, fixed tendons with limits
* motors (joint transmission, gear, ctrlrange), touch sensors on box sites, keyframes
* `mj_setConst` quantities: qpos0, body/dof/tendon invweight0 and stat.meaninertia
  (computed here with an independent float64 forward pass at qpos0)

Anything outside that subset raises `MJCFError` at load time (the reference gets the same
behaviour from `mjx.put_model`, which rejects unsupported features).
"""
from __future__ import annotations

import hashlib
import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

# MuJoCo enums (mjtGeom, mjtJoint, mjtSolver, mjtIntegrator, mjtSensor) -- numeric values as in MuJoCo
GEOM_PLANE, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE, GEOM_ELLIPSOID, GEOM_CYLINDER, GEOM_BOX = 0, 1, 2, 3, 4, 5, 6
JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = 0, 1, 2, 3
SOLVER_PGS, SOLVER_CG, SOLVER_NEWTON = 0, 1, 2
INT_EULER, INT_RK4, INT_IMPLICIT, INT_IMPLICITFAST = 0, 1, 2, 3
SENS_TOUCH = 0  # our own numbering (only touch is supported)

# collision kinds (our numbering; geom1 type <= geom2 type as MuJoCo dispatches them)
COL_PLANE_SPHERE, COL_PLANE_CAPSULE, COL_SPHERE_SPHERE, COL_SPHERE_CAPSULE, COL_CAPSULE_CAPSULE = 0, 1, 2, 3, 4
COL_NCON = {COL_PLANE_SPHERE: 1, COL_PLANE_CAPSULE: 2, COL_SPHERE_SPHERE: 1,
            COL_SPHERE_CAPSULE: 1, COL_CAPSULE_CAPSULE: 1}

mjMINVAL = 1e-15
mjMINIMP = 0.0001
mjMAXIMP = 0.9999

_GEOM_TYPES = {"plane": GEOM_PLANE, "sphere": GEOM_SPHERE, "capsule": GEOM_CAPSULE,
               "ellipsoid": GEOM_ELLIPSOID, "cylinder": GEOM_CYLINDER, "box": GEOM_BOX}
_SITE_TYPES = {"sphere": GEOM_SPHERE, "capsule": GEOM_CAPSULE, "box": GEOM_BOX,
               "cylinder": GEOM_CYLINDER, "ellipsoid": GEOM_ELLIPSOID}

# MuJoCo built-in defaults for the attributes we read
_MAIN_DEFAULTS = {
    "geom": {"type": "sphere", "size": "0 0 0", "contype": "1", "conaffinity": "1", "condim": "3",
             "friction": "1 0.005 0.0001", "solref": "0.02 1", "solimp": "0.9 0.95 0.001 0.5 2",
             "solmix": "1", "margin": "0", "gap": "0", "density": "1000", "priority": "0",
             "pos": "0 0 0"},
    "joint": {"type": "hinge", "pos": "0 0 0", "axis": "0 0 1", "stiffness": "0", "damping": "0",
              "armature": "0", "springref": "0", "ref": "0", "solreflimit": "0.02 1",
              "solimplimit": "0.9 0.95 0.001 0.5 2", "margin": "0", "limited": "auto"},
    "site": {"type": "sphere", "size": "0.005 0.005 0.005", "pos": "0 0 0"},
    "motor": {"gear": "1 0 0 0 0 0", "ctrlrange": "0 0", "ctrllimited": "auto"},
    "tendon": {"solreflimit": "0.02 1", "solimplimit": "0.9 0.95 0.001 0.5 2", "margin": "0",
               "limited": "auto", "stiffness": "0", "damping": "0"},
}

_SOLIMP_DEFAULT = [0.9, 0.95, 0.001, 0.5, 2.0]


class MJCFError(ValueError):
    """Raised for MJCF features outside the supported subset (load-time rejection)."""


def _floats(s: str) -> List[float]:
    return [float(x) for x in s.split()]


def _pad_solimp(v: List[float]) -> List[float]:
    return list(v) + _SOLIMP_DEFAULT[len(v):]


# ----------------------------------------------------------------------------------------------
# small float64 rigid-body math (MuJoCo conventions: quat = [w,x,y,z], spatial vec = [ang; lin])
# ----------------------------------------------------------------------------------------------
def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                     w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def axis_angle_quat(axis, ang):
    s = math.sin(ang / 2)
    return np.array([math.cos(ang / 2), axis[0] * s, axis[1] * s, axis[2] * s])


def z2quat(vec):
    """Minimal rotation taking +z to `vec` (MuJoCo mjuu_z2quat)."""
    v = np.asarray(vec, float)
    n = np.linalg.norm(v)
    if n < mjMINVAL:
        return np.array([1.0, 0, 0, 0])
    v = v / n
    axis = np.cross([0.0, 0.0, 1.0], v)
    s = np.linalg.norm(axis)
    if s < 1e-10:
        axis = np.array([1.0, 0, 0])
    else:
        axis = axis / s
    ang = math.atan2(s, v[2])
    return axis_angle_quat(axis, ang)


# ----------------------------------------------------------------------------------------------
@dataclass
class CompiledModel:
    """Compiled model constants (float64). Field names follow mjModel where one exists."""
    name: str = ""
    source_sha256: str = ""
    # sizes
    nq: int = 0
    nv: int = 0
    nu: int = 0
    nbody: int = 0
    njnt: int = 0
    ngeom: int = 0
    nsite: int = 0
    ntendon: int = 0
    npair: int = 0
    nsensor: int = 0
    nsensordata: int = 0
    nkey: int = 0
    # options
    timestep: float = 0.002
    gravity: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -9.81]))
    impratio: float = 1.0
    tolerance: float = 1e-8
    ls_tolerance: float = 0.01
    iterations: int = 100
    ls_iterations: int = 50
    solver: int = SOLVER_NEWTON
    integrator: int = INT_EULER
    eulerdamp: int = 1
    cone: int = 0
    meaninertia: float = 1.0
    arrays: Dict[str, np.ndarray] = field(default_factory=dict)
    names: Dict[str, List[str]] = field(default_factory=dict)

    def __getattr__(self, k):  # convenient access m.body_mass etc.
        arrays = self.__dict__.get("arrays")
        if arrays is not None and k in arrays:
            return arrays[k]
        raise AttributeError(k)

    def name2id(self, kind: str, name: str) -> int:
        try:
            return self.names[kind].index(name)
        except ValueError:
            return -1

    @property
    def qpos0(self) -> np.ndarray:
        return self.arrays["qpos0"]

    def to_json_dict(self) -> dict:
        d = {k: getattr(self, k) for k in (
            "name", "source_sha256", "nq", "nv", "nu", "nbody", "njnt", "ngeom", "nsite", "ntendon",
            "npair", "nsensor", "nsensordata", "nkey", "timestep", "impratio", "tolerance",
            "ls_tolerance", "iterations", "ls_iterations", "solver", "integrator", "eulerdamp", "cone",
            "meaninertia")}
        d["gravity"] = [float(x) for x in self.gravity]
        d["arrays"] = {k: {"dtype": str(v.dtype), "shape": list(v.shape), "data": v.ravel().tolist()}
                       for k, v in self.arrays.items()}
        d["names"] = self.names
        return d

    @classmethod
    def from_json_dict(cls, d: dict) -> "CompiledModel":
        m = cls()
        for k, v in d.items():
            if k == "arrays":
                m.arrays = {a: np.array(e["data"], dtype=e["dtype"]).reshape(e["shape"]) for a, e in v.items()}
            elif k == "gravity":
                m.gravity = np.array(v, float)
            else:
                setattr(m, k, v)
        return m


# ----------------------------------------------------------------------------------------------
class _Defaults:
    def __init__(self):
        self.classes: Dict[str, Dict[str, Dict[str, str]]] = {}

    def build(self, root_default: Optional[ET.Element]):
        base = {k: dict(v) for k, v in _MAIN_DEFAULTS.items()}
        self.classes["main"] = base
        if root_default is not None:
            self._visit(root_default, "main", parent=None)

    def _visit(self, el: ET.Element, name: str, parent: Optional[str]):
        cur = {k: dict(v) for k, v in (self.classes[parent] if parent else self.classes["main"]).items()}
        for child in el:
            if child.tag == "default":
                continue
            tag = "motor" if child.tag in ("motor", "general") else child.tag
            cur.setdefault(tag, {}).update(child.attrib)
        self.classes[name] = cur
        for child in el:
            if child.tag == "default":
                cname = child.get("class")
                if cname is None:
                    raise MJCFError("nested <default> without class")
                self._visit(child, cname, name)

    def resolve(self, tag: str, el: ET.Element, childclass: Optional[str]) -> Dict[str, str]:
        cname = el.get("class") or childclass or "main"
        if cname not in self.classes:
            raise MJCFError(f"unknown default class '{cname}'")
        attrs = dict(self.classes[cname].get(tag, {}))
        attrs.update({k: v for k, v in el.attrib.items() if k != "class"})
        return attrs


def _geom_inertia(gtype: int, size, density: float):
    """Mass and principal inertia (geom frame, about geom centre) -- MuJoCo mjCGeom::SetInertia."""
    if gtype == GEOM_SPHERE:
        r = size[0]
        mass = density * 4.0 / 3.0 * math.pi * r ** 3
        i = 0.4 * mass * r * r
        return mass, np.array([i, i, i])
    if gtype == GEOM_CAPSULE:
        r, h = size[0], 2.0 * size[1]
        m_cyl = density * math.pi * r * r * h
        m_sph = density * 4.0 / 3.0 * math.pi * r ** 3
        mass = m_cyl + m_sph
        ixy = m_cyl * (3 * r * r + h * h) / 12.0 + m_sph * (0.4 * r * r + h * h / 4.0 + 3.0 * h * r / 8.0)
        iz = m_cyl * r * r / 2.0 + m_sph * 0.4 * r * r
        return mass, np.array([ixy, ixy, iz])
    raise MJCFError(f"inertia for geom type {gtype} not supported")


def candidate_pairs(geoms, body_parentid, body_weldid, excludes, filterparent: bool = True) -> list:
    """Candidate collision pairs by MuJoCo's filter (mj_collision's broadphase rules, as MJX's
    collision_driver takes them from the model): geoms on one weld body never collide; a body's geoms
    skip its weld parent's (filterparent, unless either is the world); `<exclude>` body pairs and
    incompatible contype / conaffinity bits drop out; plane-plane is skipped. Contact parameters mix
    as mj_contactParam does at equal priority: condim and friction by max, solref / solimp by the
    solmix-weighted mean (solref by min when either is direct), margin and gap by max. `geoms`: dicts
    with type, body, contype, conaffinity, condim, friction[3], solref[2], solimp[5], solmix, margin,
    gap, priority (the MJCF compiler's, or mjmodel.py's from an MjModel)."""
    ngeom = len(geoms)
    pairs = []
    for g1 in range(ngeom):
        for g2 in range(g1 + 1, ngeom):
            G1, G2 = geoms[g1], geoms[g2]
            b1, b2 = G1["body"], G2["body"]
            w1, w2 = body_weldid[b1], body_weldid[b2]
            if w1 == w2:
                continue
            p1 = body_weldid[body_parentid[w1]] if w1 > 0 else 0
            p2 = body_weldid[body_parentid[w2]] if w2 > 0 else 0
            if filterparent and w1 != 0 and w2 != 0 and (w1 == p2 or w2 == p1):
                continue  # filterparent
            if (min(b1, b2), max(b1, b2)) in excludes:
                continue
            if not ((G1["contype"] & G2["conaffinity"]) or (G2["contype"] & G1["conaffinity"])):
                continue
            if G1["type"] == GEOM_PLANE and G2["type"] == GEOM_PLANE:
                continue
            ga, gb = (g1, g2) if G1["type"] <= G2["type"] else (g2, g1)
            ta, tb = geoms[ga]["type"], geoms[gb]["type"]
            kind = {(GEOM_PLANE, GEOM_SPHERE): COL_PLANE_SPHERE, (GEOM_PLANE, GEOM_CAPSULE): COL_PLANE_CAPSULE,
                    (GEOM_SPHERE, GEOM_SPHERE): COL_SPHERE_SPHERE, (GEOM_SPHERE, GEOM_CAPSULE): COL_SPHERE_CAPSULE,
                    (GEOM_CAPSULE, GEOM_CAPSULE): COL_CAPSULE_CAPSULE}.get((ta, tb))
            if kind is None:
                raise MJCFError(f"collision pair types {ta},{tb} not supported")
            A, B = geoms[ga], geoms[gb]
            # contact parameter mixing (MuJoCo mj_contactParam, equal priority)
            if A["priority"] != B["priority"]:
                raise MJCFError("geom priority not supported")
            condim = max(A["condim"], B["condim"])
            if condim not in (1, 3):
                raise MJCFError(f"condim {condim} not supported")
            fr = np.maximum(A["friction"], B["friction"])
            mix = A["solmix"] / (A["solmix"] + B["solmix"]) if (A["solmix"] + B["solmix"]) > mjMINVAL else 0.5
            if A["solref"][0] > 0 and B["solref"][0] > 0:
                solref = [mix * A["solref"][i] + (1 - mix) * B["solref"][i] for i in range(2)]
            else:
                solref = [min(A["solref"][i], B["solref"][i]) for i in range(2)]
            solimp = [mix * A["solimp"][i] + (1 - mix) * B["solimp"][i] for i in range(5)]
            pairs.append({"g1": ga, "g2": gb, "kind": kind, "condim": condim,
                          "friction": np.array([fr[0], fr[0], fr[1], fr[2], fr[2]]),
                          "solref": solref, "solimp": solimp,
                          "margin": max(A["margin"], B["margin"]), "gap": max(A["gap"], B["gap"])})
    return pairs


def compile_xml(path: str) -> CompiledModel:
    with open(path, "rb") as f:
        raw = f.read()
    return compile_xml_string(raw.decode("utf-8"), name_hint=path, sha=hashlib.sha256(raw).hexdigest())


def compile_xml_string(text: str, name_hint: str = "", sha: str = "") -> CompiledModel:
    root = ET.fromstring(text)
    if root.tag != "mujoco":
        raise MJCFError("root element must be <mujoco>")
    m = CompiledModel(name=root.get("model", name_hint), source_sha256=sha or hashlib.sha256(text.encode()).hexdigest())

    comp = root.find("compiler")
    angle_deg = True
    if comp is not None:
        if comp.get("angle", "degree") == "radian":
            angle_deg = False
        if comp.get("inertiafromgeom", "auto") == "false":
            raise MJCFError("inertiafromgeom=false not supported")

    # ---- options --------------------------------------------------------------------------
    opt = root.find("option")
    solver_map = {"PGS": SOLVER_PGS, "CG": SOLVER_CG, "Newton": SOLVER_NEWTON}
    integ_map = {"Euler": INT_EULER, "RK4": INT_RK4, "implicit": INT_IMPLICIT, "implicitfast": INT_IMPLICITFAST}
    if opt is not None:
        m.timestep = float(opt.get("timestep", m.timestep))
        m.gravity = np.array(_floats(opt.get("gravity", "0 0 -9.81")))
        m.impratio = float(opt.get("impratio", 1.0))
        m.tolerance = float(opt.get("tolerance", 1e-8))
        m.ls_tolerance = float(opt.get("ls_tolerance", 0.01))
        m.iterations = int(opt.get("iterations", 100))
        m.ls_iterations = int(opt.get("ls_iterations", 50))
        m.solver = solver_map[opt.get("solver", "Newton")]
        m.integrator = integ_map[opt.get("integrator", "Euler")]
        if opt.get("cone", "pyramidal") != "pyramidal":
            raise MJCFError("only pyramidal cones supported")
        flag = opt.find("flag")
        if flag is not None:
            m.eulerdamp = 0 if flag.get("eulerdamp", "enable") == "disable" else 1
            for k, v in flag.attrib.items():
                if k not in ("eulerdamp",) and v not in ("enable",):
                    raise MJCFError(f"option flag {k}={v} not supported")
    if m.solver == SOLVER_PGS:
        raise MJCFError("PGS solver not supported (MJX has no PGS)")
    if m.integrator not in (INT_EULER, INT_IMPLICITFAST):
        raise MJCFError("only Euler and implicitfast integrators supported")

    defaults = _Defaults()
    defaults.build(root.find("default"))

    # ---- body tree ---------------------------------------------------------------------------
    bodies = []   # dicts
    joints = []
    geoms = []
    sites = []
    body_names, jnt_names, geom_names, site_names = [], [], [], []

    def add_body(el, parent, childclass, name):
        bid = len(bodies)
        b = {"parent": parent, "pos": np.zeros(3), "quat": np.array([1.0, 0, 0, 0]),
             "joints": [], "geoms": [], "sites": [], "level": 0 if parent < 0 else bodies[parent]["level"] + 1}
        if el is not None and parent >= 0:
            b["pos"] = np.array(_floats(el.get("pos", "0 0 0")))
            if "quat" in el.attrib:
                q = np.array(_floats(el.get("quat")))
                b["quat"] = q / np.linalg.norm(q)
            for a in ("euler", "axisangle", "xyaxes", "zaxis"):
                if a in el.attrib:
                    raise MJCFError(f"body orientation '{a}' not supported")
            if el.find("inertial") is not None:
                raise MJCFError("explicit <inertial> not supported")
        bodies.append(b)
        body_names.append(name)
        if el is None:
            return bid
        cc = el.get("childclass", childclass)
        for child in el:
            tag = child.tag
            if tag == "freejoint":
                jid = len(joints)
                joints.append({"type": JNT_FREE, "body": bid, "pos": np.zeros(3), "axis": np.array([0, 0, 1.0]),
                               "limited": 0, "range": np.zeros(2), "stiffness": 0.0, "damping": 0.0,
                               "armature": 0.0, "springref": 0.0, "ref": 0.0,
                               "solref": [0.02, 1.0], "solimp": list(_SOLIMP_DEFAULT), "margin": 0.0})
                jnt_names.append(child.get("name", ""))
                b["joints"].append(jid)
            elif tag == "joint":
                a = defaults.resolve("joint", child, cc)
                jt = a.get("type", "hinge")
                if jt == "free":
                    jtype = JNT_FREE
                elif jt == "hinge":
                    jtype = JNT_HINGE
                else:
                    raise MJCFError(f"joint type {jt} not supported")
                axis = np.array(_floats(a["axis"]))
                axis = axis / np.linalg.norm(axis)
                rng = np.array(_floats(a["range"])) if "range" in a else np.zeros(2)
                lim = a.get("limited", "auto")
                limited = int(lim == "true" or (lim == "auto" and "range" in a))
                if jtype == JNT_HINGE and angle_deg:
                    rng = rng * math.pi / 180.0
                jid = len(joints)
                joints.append({"type": jtype, "body": bid, "pos": np.array(_floats(a["pos"])), "axis": axis,
                               "limited": limited, "range": rng, "stiffness": float(a["stiffness"]),
                               "damping": float(a["damping"]), "armature": float(a["armature"]),
                               "springref": float(a["springref"]), "ref": float(a["ref"]),
                               "solref": _floats(a["solreflimit"]), "solimp": _pad_solimp(_floats(a["solimplimit"])),
                               "margin": float(a["margin"])})
                jnt_names.append(child.get("name", ""))
                b["joints"].append(jid)
            elif tag == "geom":
                a = defaults.resolve("geom", child, cc)
                gtype = _GEOM_TYPES.get(a["type"])
                if gtype is None or gtype not in (GEOM_PLANE, GEOM_SPHERE, GEOM_CAPSULE):
                    raise MJCFError(f"geom type {a['type']} not supported")
                size = (_floats(a["size"]) + [0, 0, 0])[:3]
                pos = np.array(_floats(a["pos"]))
                quat = np.array([1.0, 0, 0, 0])
                if "fromto" in a:
                    ft = np.array(_floats(a["fromto"]))
                    p0, p1 = ft[:3], ft[3:]
                    pos = 0.5 * (p0 + p1)
                    quat = z2quat(p1 - p0)
                    size[1] = 0.5 * float(np.linalg.norm(p1 - p0))
                elif "zaxis" in a:
                    quat = z2quat(_floats(a["zaxis"]))
                elif "quat" in a:
                    quat = np.array(_floats(a["quat"]))
                    quat = quat / np.linalg.norm(quat)
                for o in ("euler", "axisangle", "xyaxes"):
                    if o in a:
                        raise MJCFError(f"geom orientation '{o}' not supported")
                # an explicit mass sets the density (mjCGeom::SetInertia: density = mass / volume)
                # (worldbody geoms and planes carry no mass: MuJoCo ignores the attribute there)
                dens = float(a["density"])
                if "mass" in a and bid != 0 and gtype != GEOM_PLANE:
                    vol, _ = _geom_inertia(gtype, size, 1.0)
                    if not vol > 0.0:
                        raise MJCFError(f"geom with mass {a['mass']} has zero volume (size {size})")
                    dens = float(a["mass"]) / vol
                frv = _floats(a["friction"])  # missing trailing values keep MuJoCo's defaults
                fr = (frv + [1.0, 0.005, 0.0001][len(frv):])[:3]
                gid = len(geoms)
                geoms.append({"type": gtype, "body": bid, "pos": pos, "quat": quat, "size": np.array(size),
                              "contype": int(a["contype"]), "conaffinity": int(a["conaffinity"]),
                              "condim": int(a["condim"]), "friction": np.array(fr),
                              "solref": _floats(a["solref"]), "solimp": _pad_solimp(_floats(a["solimp"])),
                              "solmix": float(a["solmix"]), "margin": float(a["margin"]), "gap": float(a["gap"]),
                              "density": dens, "priority": int(a["priority"])})
                geom_names.append(child.get("name", ""))
                b["geoms"].append(gid)
            elif tag == "site":
                a = defaults.resolve("site", child, cc)
                stype = _SITE_TYPES.get(a.get("type", "sphere"))
                size = (_floats(a["size"]) + [0, 0, 0])[:3]
                quat = np.array(_floats(a["quat"])) if "quat" in a else np.array([1.0, 0, 0, 0])
                sid = len(sites)
                sites.append({"type": stype, "body": bid, "pos": np.array(_floats(a["pos"])),
                              "quat": quat / np.linalg.norm(quat), "size": np.array(size)})
                site_names.append(child.get("name", ""))
                b["sites"].append(sid)
            elif tag == "body":
                add_body(child, bid, cc, child.get("name", ""))
            elif tag in ("camera", "light", "inertial"):
                if tag == "inertial":
                    raise MJCFError("explicit <inertial> not supported")
            else:
                raise MJCFError(f"body child <{tag}> not supported")
        return bid

    wb = root.find("worldbody")
    # world body: handle its direct children with add_body-like logic
    add_body(wb, -1, None, "world")

    nbody, njnt, ngeom, nsite = len(bodies), len(joints), len(geoms), len(sites)

    # ---- per-body / per-dof bookkeeping ------------------------------------------------------
    nq = nv = 0
    jnt_qposadr, jnt_dofadr = [], []
    dof_bodyid, dof_jntid, dof_parentid = [], [], []
    body_dofadr = np.zeros(nbody, np.int32)
    body_dofnum = np.zeros(nbody, np.int32)
    body_jntadr = np.full(nbody, -1, np.int32)
    body_jntnum = np.zeros(nbody, np.int32)
    last_dof_of_body = [-1] * nbody
    for b in range(nbody):
        par = bodies[b]["parent"]
        parent_last = -1
        p = par
        while p >= 0:
            if last_dof_of_body[p] >= 0:
                parent_last = last_dof_of_body[p]
                break
            p = bodies[p]["parent"]
        body_dofadr[b] = nv
        if bodies[b]["joints"]:
            body_jntadr[b] = bodies[b]["joints"][0]
        body_jntnum[b] = len(bodies[b]["joints"])
        prev = parent_last
        for j in bodies[b]["joints"]:
            jt = joints[j]["type"]
            nqj, nvj = (7, 6) if jt == JNT_FREE else (1, 1)
            jnt_qposadr.append(nq)
            jnt_dofadr.append(nv)
            for k in range(nvj):
                dof_bodyid.append(b)
                dof_jntid.append(j)
                dof_parentid.append(prev)
                prev = nv + k
            nq += nqj
            nv += nvj
        body_dofnum[b] = nv - body_dofadr[b]
        last_dof_of_body[b] = prev if bodies[b]["joints"] else parent_last

    # weld ids and root ids
    body_weldid = np.zeros(nbody, np.int32)
    body_rootid = np.zeros(nbody, np.int32)
    for b in range(nbody):
        par = bodies[b]["parent"]
        if b == 0:
            continue
        body_weldid[b] = b if bodies[b]["joints"] else body_weldid[par]
        body_rootid[b] = b if par == 0 else body_rootid[par]
    # subtree ranges (bodies are in DFS preorder -> subtree of b is [b, end))
    body_subtree_end = np.zeros(nbody, np.int32)
    for b in range(nbody):
        e = b + 1
        while e < nbody:
            p = bodies[e]["parent"]
            while p > b:
                p = bodies[p]["parent"]
            if p != b:
                break
            e += 1
        body_subtree_end[b] = e

    # ---- inertia from geoms ------------------------------------------------------------------
    body_mass = np.zeros(nbody)
    body_ipos = np.zeros((nbody, 3))
    body_inertia = np.zeros((nbody, 6))  # full tensor about ipos in body frame: xx yy zz xy xz yz
    for b in range(1, nbody):
        gl = bodies[b]["geoms"]
        if not gl:
            continue
        ms, cs, Is = [], [], []
        for g in gl:
            G = geoms[g]
            mass, pri = _geom_inertia(G["type"], G["size"], G["density"])
            R = quat2mat(G["quat"])
            ms.append(mass)
            cs.append(G["pos"])
            Is.append(R @ np.diag(pri) @ R.T)
        M = sum(ms)
        com = sum(mi * ci for mi, ci in zip(ms, cs)) / M
        I = np.zeros((3, 3))
        for mi, ci, Ii in zip(ms, cs, Is):
            d = ci - com
            I += Ii + mi * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        body_mass[b] = M
        body_ipos[b] = com
        body_inertia[b] = [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]

    # ---- qpos0 / springs ---------------------------------------------------------------------
    qpos0 = np.zeros(nq)
    qpos_spring = np.zeros(nq)
    for j, J in enumerate(joints):
        a = jnt_qposadr[j]
        if J["type"] == JNT_FREE:
            b = J["body"]
            qpos0[a:a + 3] = bodies[b]["pos"]
            qpos0[a + 3:a + 7] = bodies[b]["quat"]
            qpos_spring[a:a + 7] = qpos0[a:a + 7]
        else:
            qpos0[a] = J["ref"]
            qpos_spring[a] = J["springref"]

    # ---- contact pairs -----------------------------------------------------------------------
    excludes = set()
    cont = root.find("contact")
    if cont is not None:
        for ex in cont:
            if ex.tag == "exclude":
                b1 = body_names.index(ex.get("body1"))
                b2 = body_names.index(ex.get("body2"))
                excludes.add((min(b1, b2), max(b1, b2)))
            else:
                raise MJCFError(f"<contact><{ex.tag}> not supported")
    pairs = candidate_pairs(geoms, [b["parent"] for b in bodies], body_weldid, excludes)

    # ---- actuators ---------------------------------------------------------------------------
    act = root.find("actuator")
    actuators = []
    act_names = []
    if act is not None:
        for a_el in act:
            if a_el.tag != "motor":
                raise MJCFError(f"actuator <{a_el.tag}> not supported")
            a = defaults.resolve("motor", a_el, None)
            jn = a.get("joint")
            if jn is None:
                raise MJCFError("only joint transmission supported")
            jid = jnt_names.index(jn)
            if joints[jid]["type"] != JNT_HINGE:
                raise MJCFError("motor on non-hinge joint not supported")
            gear = _floats(a["gear"])[0]
            cr = _floats(a["ctrlrange"])
            cl = a.get("ctrllimited", "auto")
            limited = int(cl == "true" or (cl == "auto" and "ctrlrange" in a_el.attrib))
            actuators.append({"jnt": jid, "gear": gear, "ctrlrange": cr, "ctrllimited": limited})
            act_names.append(a_el.get("name", ""))

    # ---- tendons -----------------------------------------------------------------------------
    ten = root.find("tendon")
    tendons = []
    ten_names = []
    if ten is not None:
        for t_el in ten:
            if t_el.tag != "fixed":
                raise MJCFError(f"tendon <{t_el.tag}> not supported")
            a = defaults.resolve("tendon", t_el, None)
            rng = _floats(a["range"]) if "range" in a else [0.0, 0.0]
            lim = a.get("limited", "auto")
            limited = int(lim == "true" or (lim == "auto" and "range" in a))
            if float(a["stiffness"]) != 0 or float(a["damping"]) != 0:
                raise MJCFError("tendon stiffness/damping not supported")
            jl, cl = [], []
            for w in t_el:
                if w.tag != "joint":
                    raise MJCFError("only joint wraps supported in fixed tendons")
                jl.append(jnt_names.index(w.get("joint")))
                cl.append(float(w.get("coef", "1")))
            tendons.append({"jnt": jl, "coef": cl, "range": rng, "limited": limited,
                            "solref": _floats(a["solreflimit"]), "solimp": _pad_solimp(_floats(a["solimplimit"])),
                            "margin": float(a["margin"])})
            ten_names.append(t_el.get("name", ""))

    # ---- sensors -----------------------------------------------------------------------------
    sen = root.find("sensor")
    sensors = []
    sen_names = []
    if sen is not None:
        for s_el in sen:
            if s_el.tag != "touch":
                raise MJCFError(f"sensor <{s_el.tag}> not supported")
            sid = site_names.index(s_el.get("site"))
            if sites[sid]["type"] != GEOM_BOX:
                raise MJCFError("touch sensor requires a box site")
            sensors.append({"type": SENS_TOUCH, "objid": sid, "adr": len(sensors), "dim": 1})
            sen_names.append(s_el.get("name", ""))

    # ---- keyframes ---------------------------------------------------------------------------
    keys, key_names = [], []
    kf = root.find("keyframe")
    if kf is not None:
        for k in kf:
            q = np.array(_floats(k.get("qpos"))) if "qpos" in k.attrib else qpos0.copy()
            if q.size != nq:
                raise MJCFError("keyframe qpos size mismatch")
            keys.append(q)
            key_names.append(k.get("name", ""))

    # ---- fill arrays -------------------------------------------------------------------------
    A = {}
    A["body_parentid"] = np.array([b["parent"] for b in bodies], np.int32)
    A["body_rootid"] = body_rootid
    A["body_weldid"] = body_weldid
    A["body_jntadr"] = body_jntadr
    A["body_jntnum"] = body_jntnum
    A["body_dofadr"] = body_dofadr
    A["body_dofnum"] = body_dofnum
    A["body_subtree_end"] = body_subtree_end
    A["body_level"] = np.array([b["level"] for b in bodies], np.int32)
    A["body_pos"] = np.array([b["pos"] for b in bodies])
    A["body_quat"] = np.array([b["quat"] for b in bodies])
    A["body_ipos"] = body_ipos
    A["body_inertia"] = body_inertia
    A["body_mass"] = body_mass
    A["jnt_type"] = np.array([j["type"] for j in joints], np.int32)
    A["jnt_qposadr"] = np.array(jnt_qposadr, np.int32)
    A["jnt_dofadr"] = np.array(jnt_dofadr, np.int32)
    A["jnt_bodyid"] = np.array([j["body"] for j in joints], np.int32)
    A["jnt_limited"] = np.array([j["limited"] for j in joints], np.int32)
    A["jnt_pos"] = np.array([j["pos"] for j in joints])
    A["jnt_axis"] = np.array([j["axis"] for j in joints])
    A["jnt_range"] = np.array([j["range"] for j in joints])
    A["jnt_stiffness"] = np.array([j["stiffness"] for j in joints])
    A["jnt_margin"] = np.array([j["margin"] for j in joints])
    A["jnt_solref"] = np.array([j["solref"] for j in joints])
    A["jnt_solimp"] = np.array([j["solimp"] for j in joints])
    A["dof_bodyid"] = np.array(dof_bodyid, np.int32)
    A["dof_jntid"] = np.array(dof_jntid, np.int32)
    A["dof_parentid"] = np.array(dof_parentid, np.int32)
    dof_damping = np.zeros(nv)
    dof_armature = np.zeros(nv)
    for d in range(nv):
        J = joints[dof_jntid[d]]
        dof_damping[d] = J["damping"]
        dof_armature[d] = J["armature"]
    A["dof_damping"] = dof_damping
    A["dof_armature"] = dof_armature
    A["qpos0"] = qpos0
    A["qpos_spring"] = qpos_spring
    A["geom_type"] = np.array([g["type"] for g in geoms], np.int32)
    A["geom_bodyid"] = np.array([g["body"] for g in geoms], np.int32)
    A["geom_contype"] = np.array([g["contype"] for g in geoms], np.int32)
    A["geom_conaffinity"] = np.array([g["conaffinity"] for g in geoms], np.int32)
    A["geom_condim"] = np.array([g["condim"] for g in geoms], np.int32)
    A["geom_pos"] = np.array([g["pos"] for g in geoms])
    A["geom_quat"] = np.array([g["quat"] for g in geoms])
    A["geom_size"] = np.array([g["size"] for g in geoms])
    A["geom_friction"] = np.array([g["friction"] for g in geoms])
    # per-geom contact parameters (MjModel's geom_solref ...; the pairs above hold their mixes)
    A["geom_solref"] = np.array([g["solref"] for g in geoms]).reshape(-1, 2)
    A["geom_solimp"] = np.array([g["solimp"] for g in geoms]).reshape(-1, 5)
    A["geom_solmix"] = np.array([g["solmix"] for g in geoms])
    A["geom_margin"] = np.array([g["margin"] for g in geoms])
    A["geom_gap"] = np.array([g["gap"] for g in geoms])
    A["geom_priority"] = np.array([g["priority"] for g in geoms], np.int32)
    A["pair_geom1"] = np.array([p["g1"] for p in pairs], np.int32)
    A["pair_geom2"] = np.array([p["g2"] for p in pairs], np.int32)
    A["pair_kind"] = np.array([p["kind"] for p in pairs], np.int32)
    A["pair_condim"] = np.array([p["condim"] for p in pairs], np.int32)
    A["pair_friction"] = np.array([p["friction"] for p in pairs]).reshape(-1, 5)
    A["pair_solref"] = np.array([p["solref"] for p in pairs]).reshape(-1, 2)
    A["pair_solimp"] = np.array([p["solimp"] for p in pairs]).reshape(-1, 5)
    A["pair_margin"] = np.array([p["margin"] for p in pairs])
    A["pair_gap"] = np.array([p["gap"] for p in pairs])
    A["site_type"] = np.array([s["type"] for s in sites], np.int32)
    A["site_bodyid"] = np.array([s["body"] for s in sites], np.int32)
    A["site_pos"] = np.array([s["pos"] for s in sites]).reshape(-1, 3)
    A["site_quat"] = np.array([s["quat"] for s in sites]).reshape(-1, 4)
    A["site_size"] = np.array([s["size"] for s in sites]).reshape(-1, 3)
    A["actuator_trnid"] = np.array([a["jnt"] for a in actuators], np.int32)
    A["actuator_gear"] = np.array([a["gear"] for a in actuators])
    A["actuator_ctrlrange"] = np.array([a["ctrlrange"] for a in actuators]).reshape(-1, 2)
    A["actuator_ctrllimited"] = np.array([a["ctrllimited"] for a in actuators], np.int32)
    A["tendon_num"] = np.array([len(t["jnt"]) for t in tendons], np.int32)
    maxw = max([len(t["jnt"]) for t in tendons] + [1])
    tj = np.full((len(tendons), maxw), -1, np.int32)
    tc = np.zeros((len(tendons), maxw))
    for i, t in enumerate(tendons):
        tj[i, :len(t["jnt"])] = t["jnt"]
        tc[i, :len(t["coef"])] = t["coef"]
    A["tendon_jnt"] = tj
    A["tendon_coef"] = tc
    A["tendon_limited"] = np.array([t["limited"] for t in tendons], np.int32)
    A["tendon_range"] = np.array([t["range"] for t in tendons]).reshape(-1, 2)
    A["tendon_margin"] = np.array([t["margin"] for t in tendons])
    A["tendon_solref"] = np.array([t["solref"] for t in tendons]).reshape(-1, 2)
    A["tendon_solimp"] = np.array([t["solimp"] for t in tendons]).reshape(-1, 5)
    A["sensor_type"] = np.array([s["type"] for s in sensors], np.int32)
    A["sensor_objid"] = np.array([s["objid"] for s in sensors], np.int32)
    A["sensor_adr"] = np.array([s["adr"] for s in sensors], np.int32)
    A["key_qpos"] = np.array(keys).reshape(-1, nq)
    A["exclude_signature"] = np.array(sorted((b1 << 16) + b2 for b1, b2 in excludes), np.int64)  # MjModel's

    m.arrays = A
    m.names = {"body": body_names, "joint": jnt_names, "geom": geom_names, "site": site_names,
               "actuator": act_names, "tendon": ten_names, "sensor": sen_names, "key": key_names}
    m.nq, m.nv, m.nu = nq, nv, len(actuators)
    m.nbody, m.njnt, m.ngeom, m.nsite = nbody, njnt, ngeom, nsite
    m.ntendon, m.npair, m.nsensor = len(tendons), len(pairs), len(sensors)
    m.nsensordata = len(sensors)
    m.nkey = len(keys)
    _set_const(m)
    return m


# ----------------------------------------------------------------------------------------------
# mj_setConst subset: forward kinematics + CRB mass matrix at qpos0 (float64, numpy)
# ----------------------------------------------------------------------------------------------
def _fk_and_mass(m: CompiledModel, qpos: np.ndarray):
    A = m.arrays
    nb, nv = m.nbody, m.nv
    xpos = np.zeros((nb, 3))
    xmat = np.zeros((nb, 3, 3))
    xmat[0] = np.eye(3)
    xquat = np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    xanchor = np.zeros((m.njnt, 3))
    xaxis = np.zeros((m.njnt, 3))
    for b in range(1, nb):
        p = A["body_parentid"][b]
        pos = xpos[p] + xmat[p] @ A["body_pos"][b]
        quat = quat_mul(xquat[p], A["body_quat"][b])
        for j in range(A["body_jntadr"][b], A["body_jntadr"][b] + A["body_jntnum"][b]):
            qa = A["jnt_qposadr"][j]
            if A["jnt_type"][j] == JNT_FREE:
                pos = qpos[qa:qa + 3].copy()
                quat = qpos[qa + 3:qa + 7] / np.linalg.norm(qpos[qa + 3:qa + 7])
                xanchor[j] = pos
                xaxis[j] = quat2mat(quat)[:, 2]
            else:
                R = quat2mat(quat)
                anchor = pos + R @ A["jnt_pos"][j]
                xanchor[j] = anchor
                xaxis[j] = R @ A["jnt_axis"][j]
                quat = quat_mul(quat, axis_angle_quat(A["jnt_axis"][j], qpos[qa] - A["qpos0"][qa]))
                R = quat2mat(quat)
                pos = anchor - R @ A["jnt_pos"][j]
        quat = quat / np.linalg.norm(quat)
        xpos[b], xquat[b], xmat[b] = pos, quat, quat2mat(quat)
    xipos = np.array([xpos[b] + xmat[b] @ A["body_ipos"][b] for b in range(nb)])
    mass = A["body_mass"]
    # subtree com
    subtree_com = np.zeros((nb, 3))
    for b in range(nb):
        e = A["body_subtree_end"][b]
        ms = mass[b:e].sum()
        subtree_com[b] = (mass[b:e, None] * xipos[b:e]).sum(0) / ms if ms > mjMINVAL else xipos[b]
    # 6x6 spatial inertia about subtree_com[root] in world-aligned frame
    def sp_inertia(b):
        I6 = np.zeros((6, 6))
        if mass[b] == 0:
            return I6
        c = xipos[b] - subtree_com[A["body_rootid"][b]]
        t = A["body_inertia"][b]
        Ib = np.array([[t[0], t[3], t[4]], [t[3], t[1], t[5]], [t[4], t[5], t[2]]])
        Iw = xmat[b] @ Ib @ xmat[b].T + mass[b] * (np.dot(c, c) * np.eye(3) - np.outer(c, c))
        cx = np.array([[0, -c[2], c[1]], [c[2], 0, -c[0]], [-c[1], c[0], 0]])
        I6[:3, :3] = Iw
        I6[:3, 3:] = mass[b] * cx
        I6[3:, :3] = -mass[b] * cx
        I6[3:, 3:] = mass[b] * np.eye(3)
        return I6
    cinert = [sp_inertia(b) for b in range(nb)]
    cdof = np.zeros((nv, 6))
    for d in range(nv):
        j = A["dof_jntid"][d]
        b = A["dof_bodyid"][d]
        root_com = subtree_com[A["body_rootid"][b]]
        if A["jnt_type"][j] == JNT_FREE:
            k = d - A["jnt_dofadr"][j]
            if k < 3:
                cdof[d, 3 + k] = 1.0
            else:
                ax = xmat[b][:, k - 3]
                cdof[d, :3] = ax
                cdof[d, 3:] = np.cross(ax, root_com - xanchor[j])
        else:
            ax = xaxis[j]
            cdof[d, :3] = ax
            cdof[d, 3:] = np.cross(ax, root_com - xanchor[j])
    crb = [None] * nb
    for b in range(nb):
        crb[b] = sum(cinert[c] for c in range(b, A["body_subtree_end"][b]))
    M = np.zeros((nv, nv))
    for i in range(nv):
        f = crb[A["dof_bodyid"][i]] @ cdof[i]
        j = i
        while j >= 0:
            M[i, j] = M[j, i] = cdof[j] @ f
            j = A["dof_parentid"][j]
    M += np.diag(A["dof_armature"])
    return dict(xpos=xpos, xmat=xmat, xquat=xquat, xipos=xipos, subtree_com=subtree_com, cdof=cdof, M=M)


def body_jacobian(m: CompiledModel, kin: dict, b: int, point: np.ndarray):
    """jacp, jacr (3 x nv) of a point attached to body b (MuJoCo mj_jac)."""
    A = m.arrays
    jacp = np.zeros((3, m.nv))
    jacr = np.zeros((3, m.nv))
    if b == 0:
        return jacp, jacr
    # last dof affecting body b
    d = -1
    bb = b
    while bb > 0:
        if A["body_dofnum"][bb] > 0:
            d = A["body_dofadr"][bb] + A["body_dofnum"][bb] - 1
            break
        bb = A["body_parentid"][bb]
    off = point - kin["subtree_com"][A["body_rootid"][b]]
    while d >= 0:
        c = kin["cdof"][d]
        jacr[:, d] = c[:3]
        jacp[:, d] = c[3:] + np.cross(c[:3], off)
        d = A["dof_parentid"][d]
    return jacp, jacr


def _set_const(m: CompiledModel):
    A = m.arrays
    kin = _fk_and_mass(m, A["qpos0"])
    M = kin["M"]
    Minv = np.linalg.inv(M)
    nb = m.nbody
    inv0 = np.zeros((nb, 2))
    for b in range(1, nb):
        if A["body_weldid"][b] == 0:
            continue
        jacp, jacr = body_jacobian(m, kin, b, kin["xipos"][b])
        J = np.vstack([jacp, jacr])
        Am = J @ Minv @ J.T
        inv0[b, 0] = max(mjMINVAL, (Am[0, 0] + Am[1, 1] + Am[2, 2]) / 3.0)
        inv0[b, 1] = max(mjMINVAL, (Am[3, 3] + Am[4, 4] + Am[5, 5]) / 3.0)
    A["body_invweight0"] = inv0
    dinv = np.zeros(m.nv)
    for j in range(m.njnt):
        da = A["jnt_dofadr"][j]
        if A["jnt_type"][j] == JNT_FREE:
            dinv[da:da + 3] = np.mean(np.diag(Minv)[da:da + 3])
            dinv[da + 3:da + 6] = np.mean(np.diag(Minv)[da + 3:da + 6])
        else:
            dinv[da] = Minv[da, da]
    A["dof_invweight0"] = dinv
    tinv = np.zeros(m.ntendon)
    for t in range(m.ntendon):
        Jt = np.zeros(m.nv)
        for w in range(A["tendon_num"][t]):
            Jt[A["jnt_dofadr"][A["tendon_jnt"][t, w]]] += A["tendon_coef"][t, w]
        tinv[t] = max(mjMINVAL, Jt @ Minv @ Jt)
    A["tendon_invweight0"] = tinv
    m.meaninertia = float(np.trace(M) / m.nv) if m.nv else 1.0


def load_model(path: str) -> CompiledModel:
    """Load an MJCF `.xml` (compiled here) or a pre-compiled `.json` model."""
    if path.endswith(".json"):
        import json
        with open(path) as f:
            return CompiledModel.from_json_dict(json.load(f))
    return compile_xml(path)

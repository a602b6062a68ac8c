"""MJCF -> compiled POD model (``mpcr_model_t``, include/mpcr_model.h).

The reference loads its scene with ``mujoco.MjModel.from_xml_path`` and ships
it to the device with ``mjx.put_model`` (SBP/mjx_planner.py:100-108).  MuJoCo
is not available here, so this module is our own compiler for the subset of
MJCF the reference's scenes use:

* ``<include>`` (file-level and inside ``<worldbody>``), nested ``<default>``
  classes with inheritance and ``childclass``;
* bodies, hinge/slide/free joints, armature/damping/range/``autolimits``,
  ``gravcomp``, explicit ``<inertial>`` and geom-inferred inertia (plane,
  sphere, capsule, box and STL meshes, MuJoCo "legacy" mesh inertia);
* geoms/sites, contact-pair filtering (contype/conaffinity, same-weld,
  parent-weld unless world, ``<contact><exclude>``), mixed contact params;
* joint equalities, ``<option>`` (timestep/iterations/ls_iterations/flags);
* ``mj_setConst``-style constants at qpos0: body/dof invweight0, meaninertia.

Everything is fp64 numpy; the result serialises to the blob the C ABI loads
(``Model.to_blob``).  Semantics are restated from MuJoCo's documented
behaviour; see DESIGN.md "Model front-end" for what is and is not pinned.
"""

from __future__ import annotations

import copy
import ctypes
import math
import os
import re
import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

from . import cmodel

# ---------------------------------------------------------------------------
# small quaternion helpers (w, x, y, z)
# ---------------------------------------------------------------------------


def quat_mul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([
        aw * bw - ax * bx - ay * by - az * bz,
        aw * bx + ax * bw + ay * bz - az * by,
        aw * by - ax * bz + ay * bw + az * bx,
        aw * bz + ax * by - ay * bx + az * bw,
    ])


def quat_normalize(q):
    q = np.asarray(q, dtype=np.float64)
    n = np.linalg.norm(q)
    if n < 1e-15:
        return np.array([1.0, 0.0, 0.0, 0.0])
    return q / n


def quat2mat(q):
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def mat2quat(R):
    """Rotation matrix -> unit quaternion (w >= 0)."""
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = quat_normalize(q)
    if q[0] < 0:
        q = -q
    return q


def axisangle2quat(axis, angle):
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.linalg.norm(axis)
    s = math.sin(angle / 2)
    return np.array([math.cos(angle / 2), axis[0] * s, axis[1] * s, axis[2] * s])


# ---------------------------------------------------------------------------
# constants (MuJoCo defaults)
# ---------------------------------------------------------------------------

GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4,
              "cylinder": 5, "box": 6, "mesh": 7}
JNT_TYPES = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}
JNT_NQ = {0: 7, 1: 4, 2: 1, 3: 1}
JNT_NV = {0: 6, 1: 3, 2: 1, 3: 1}

DEFAULT_SOLREF = (0.02, 1.0)
DEFAULT_SOLIMP = (0.9, 0.95, 0.001, 0.5, 2.0)

COLLISION_FUNC = {
    # (type1, type2) with type1 <= type2  ->  (func id, contact slots)
    (0, 3): (cmodel.COL_PLANE_CAPSULE, 2),
    (0, 6): (cmodel.COL_PLANE_BOX, 4),
    (3, 3): (cmodel.COL_CAPSULE_CAPSULE, 1),
    (3, 6): (cmodel.COL_CAPSULE_BOX, 2),
    (6, 6): (cmodel.COL_BOX_BOX, 4),
}

CONVEX_TYPES = (2, 3, 5, 6, 7)  # sphere, capsule, cylinder, box, mesh (convex hull)


def collision_func(t1, t2):
    """(func, contact slots) of a pair with t1 <= t2: the dedicated primitive
    functions, else the general convex one (one contact, MuJoCo's own
    general-convex path also yields one).  Plane - mesh owns 4 slots: MJX's
    plane_convex manifold (oracle col_plane_mesh)."""
    if (t1, t2) in COLLISION_FUNC:
        return COLLISION_FUNC[(t1, t2)]
    if t1 == 0 and t2 in CONVEX_TYPES:
        return (cmodel.COL_PLANE_CONVEX, 4 if t2 == 7 else 1)
    if t1 in CONVEX_TYPES and t2 in CONVEX_TYPES:
        return (cmodel.COL_CONVEX, 1)
    return None


ROBOT_GEOM_NAMES = tuple(f"robot_{i}" for i in range(10))  # SBP/mjx_planner.py:113


class MJCFError(ValueError):
    pass


def _floats(s, n=None):
    v = [float(x) for x in s.split()]
    if n is not None and len(v) != n:
        raise MJCFError(f"expected {n} numbers, got {s!r}")
    return v


# ---------------------------------------------------------------------------
# mesh loading + "legacy" mesh inertia
# ---------------------------------------------------------------------------


def load_stl(path):
    """Return (ntri, 3, 3) float64 triangle vertices of an STL file."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) >= 84:
        (ntri,) = struct.unpack_from("<I", data, 80)
        if 84 + 50 * ntri == len(data):
            dt = np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")])
            arr = np.frombuffer(data, dtype=dt, count=ntri, offset=84)
            return arr["v"].astype(np.float64)
    # ASCII fallback
    verts = re.findall(rb"vertex\s+(\S+)\s+(\S+)\s+(\S+)", data)
    if not verts or len(verts) % 3:
        raise MJCFError(f"cannot parse STL {path}")
    return np.array(verts, dtype=np.float64).reshape(-1, 3, 3)


def load_obj(path):
    verts, faces = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                verts.append([float(x) for x in line.split()[1:4]])
            elif line.startswith("f "):
                idx = [int(tok.split("/")[0]) for tok in line.split()[1:]]
                idx = [i - 1 if i > 0 else len(verts) + i for i in idx]
                for k in range(1, len(idx) - 1):
                    faces.append((idx[0], idx[k], idx[k + 1]))
    v = np.array(verts, dtype=np.float64)
    return v[np.array(faces, dtype=np.int64)]


def mesh_inertia(tris, density):
    """Volume-based mass, centre of mass and inertia (about the COM, mesh frame).

    Restates MuJoCo's default ("legacy") mesh inertia: every triangle forms a
    tetrahedron with the area-weighted surface centroid as apex and its volume
    is taken as |det|/6 (so non-convex meshes over-count, as in MuJoCo).
    """
    v0, v1, v2 = tris[:, 0], tris[:, 1], tris[:, 2]
    cr = np.cross(v1 - v0, v2 - v0)
    area = 0.5 * np.linalg.norm(cr, axis=1)
    facecen = (area[:, None] * (v0 + v1 + v2) / 3.0).sum(0) / area.sum()
    a = v0 - facecen
    b = v1 - facecen
    c = v2 - facecen
    vol = np.abs(np.einsum("ij,ij->i", a, np.cross(b, c))) / 6.0
    volume = vol.sum()
    if volume <= 1e-12:
        raise MJCFError("mesh volume too small")
    com = (vol[:, None] * (facecen + v0 + v1 + v2) / 4.0).sum(0) / volume
    d = facecen - com
    p1, p2, p3 = v0 - com, v1 - com, v2 - com
    s = d[None, :] + p1 + p2 + p3
    acc = (np.einsum("ki,kj->kij", s, s) + np.outer(d, d)[None]
           + np.einsum("ki,kj->kij", p1, p1) + np.einsum("ki,kj->kij", p2, p2)
           + np.einsum("ki,kj->kij", p3, p3))
    P = (vol[:, None, None] / 20.0 * acc).sum(0) * density
    inertia = np.trace(P) * np.eye(3) - P
    return density * volume, com, inertia


def geom_inertia(gtype, size, density):
    """Mass and inertia (about the geom centre, geom frame) of a primitive."""
    if gtype == 2:  # sphere
        r = size[0]
        m = density * 4.0 / 3.0 * math.pi * r ** 3
        i = 0.4 * m * r * r
        return m, np.diag([i, i, i])
    if gtype == 3:  # capsule: cylinder + two hemispheres
        r, hl = size[0], size[1]
        h = 2 * hl
        m = density * (math.pi * r * r * h + 4.0 / 3.0 * math.pi * r ** 3)
        ms = m * 4 * r / (4 * r + 3 * h)
        mc = m - ms
        ixx = mc * (3 * r * r + h * h) / 12.0
        izz = mc * r * r / 2.0
        si = 2 * ms * r * r / 5.0
        ixx += si + ms * h * (3 * r + 2 * h) / 8.0
        izz += si
        return m, np.diag([ixx, ixx, izz])
    if gtype == 5:  # cylinder
        r, hl = size[0], size[1]
        h = 2 * hl
        m = density * math.pi * r * r * h
        ixx = m * (3 * r * r + h * h) / 12.0
        return m, np.diag([ixx, ixx, m * r * r / 2.0])
    if gtype == 6:  # box
        x, y, z = size
        m = density * 8 * x * y * z
        return m, np.diag([m * (y * y + z * z) / 3, m * (x * x + z * z) / 3, m * (x * x + y * y) / 3])
    if gtype == 4:  # ellipsoid
        a, b, c = size
        m = density * 4.0 / 3.0 * math.pi * a * b * c
        return m, np.diag([m * (b * b + c * c) / 5, m * (a * a + c * c) / 5, m * (a * a + b * b) / 5])
    if gtype == 0:  # plane: massless
        return 0.0, np.zeros((3, 3))
    raise MJCFError(f"no inertia for geom type {gtype}")


# ---------------------------------------------------------------------------
# XML front end: includes + defaults
# ---------------------------------------------------------------------------


def _expand_includes(elem, basedir):
    """Replace <include file=...> in-place by the children of the included root."""
    out = []
    for child in list(elem):
        if child.tag == "include":
            path = os.path.join(basedir, child.get("file"))
            sub = ET.parse(path).getroot()
            _expand_includes(sub, os.path.dirname(path))
            out.extend(list(sub))
        else:
            _expand_includes(child, basedir)
            out.append(child)
    for c in list(elem):
        elem.remove(c)
    for c in out:
        elem.append(c)


class _Defaults:
    """Nested default classes: class name -> {tag: {attr: value}}."""

    def __init__(self):
        self.classes = {"main": {}}
        self.parent = {"main": None}

    def parse(self, elem, parent_cls=None):
        name = elem.get("class", "main")
        base = copy.deepcopy(self.classes[parent_cls]) if parent_cls else {}
        for child in elem:
            if child.tag == "default":
                continue
            tag = child.tag
            d = base.setdefault(tag, {})
            d.update(child.attrib)
        self.classes[name] = base
        self.parent[name] = parent_cls
        for child in elem:
            if child.tag == "default":
                self.parse(child, name)

    def attrs(self, cls, tag, elem):
        a = dict(self.classes.get(cls, self.classes["main"]).get(tag, {}))
        a.update(elem.attrib)
        return a


@dataclass
class _Body:
    name: str
    parent: int
    pos: np.ndarray
    quat: np.ndarray
    gravcomp: float = 0.0
    inertial: dict | None = None
    joints: list = field(default_factory=list)
    geoms: list = field(default_factory=list)
    sites: list = field(default_factory=list)


# ---------------------------------------------------------------------------
# the compiled model
# ---------------------------------------------------------------------------


class _NamedView:
    def __init__(self, id, pos=None, quat=None):
        self.id = id
        self.pos = pos
        self.quat = quat


class Model:
    """Compiled model: numpy arrays named like mjModel + the POD struct."""

    def __init__(self):
        self.names = {"body": [], "joint": [], "geom": [], "site": []}

    # -- mjModel-like name lookups used by the MPC driver ------------------
    def _id(self, kind, name):
        try:
            return self.names[kind].index(name)
        except ValueError:
            raise KeyError(f"no {kind} named {name!r}") from None

    def body(self, name):
        i = self._id("body", name)
        return _NamedView(i, self.body_pos[i], self.body_quat[i])

    def site(self, name):
        i = self._id("site", name)
        return _NamedView(i, self.site_pos[i], self.site_quat[i])

    def geom(self, name):
        i = self._id("geom", name)
        return _NamedView(i, self.geom_pos[i], self.geom_quat[i])

    # -- serialisation ------------------------------------------------------
    def to_struct(self) -> cmodel.mpcr_model_t:
        return cmodel.pack(self)

    def to_blob(self) -> bytes:
        return bytes(self.to_struct())

    def save(self, path):
        with open(path, "wb") as f:
            f.write(self.to_blob())


# ---------------------------------------------------------------------------
# compiler
# ---------------------------------------------------------------------------


def _orientation(a, angle_scale, eulerseq="xyz"):
    if "quat" in a:
        return quat_normalize(_floats(a["quat"], 4))
    if "axisangle" in a:
        v = _floats(a["axisangle"], 4)
        return axisangle2quat(v[:3], v[3] * angle_scale)
    if "euler" in a:
        e = np.array(_floats(a["euler"], 3)) * angle_scale
        q = np.array([1.0, 0, 0, 0])
        for ax, ang in zip(eulerseq, e):
            axis = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1]}[ax.lower()]
            r = axisangle2quat(axis, ang)
            q = quat_mul(q, r) if ax.islower() else quat_mul(r, q)
        return quat_normalize(q)
    if "xyaxes" in a:
        v = _floats(a["xyaxes"], 6)
        x = np.array(v[:3])
        x /= np.linalg.norm(x)
        y = np.array(v[3:])
        y -= x * np.dot(x, y)
        y /= np.linalg.norm(y)
        z = np.cross(x, y)
        return mat2quat(np.column_stack([x, y, z]))
    if "zaxis" in a:
        z = np.array(_floats(a["zaxis"], 3))
        z /= np.linalg.norm(z)
        ref = np.array([0.0, 0.0, 1.0])
        ax = np.cross(ref, z)
        s = np.linalg.norm(ax)
        if s < 1e-12:
            return np.array([1.0, 0, 0, 0]) if z[2] > 0 else np.array([0.0, 1, 0, 0])
        return axisangle2quat(ax / s, math.atan2(s, np.dot(ref, z)))
    return np.array([1.0, 0.0, 0.0, 0.0])


def compile_mjcf(path: str, timestep: float | None = None) -> Model:
    """Parse and compile an MJCF file into a :class:`Model`."""
    path = os.path.abspath(path)
    root = ET.parse(path).getroot()
    _expand_includes(root, os.path.dirname(path))

    # global compiler settings (last one wins, as in MuJoCo)
    angle_scale = math.pi / 180.0
    autolimits = True
    meshdir = ""
    eulerseq = "xyz"
    for c in root.iter("compiler"):
        if c.get("angle") == "radian":
            angle_scale = 1.0
        elif c.get("angle") == "degree":
            angle_scale = math.pi / 180.0
        if "autolimits" in c.attrib:
            autolimits = c.get("autolimits") == "true"
        if "meshdir" in c.attrib:
            meshdir = c.get("meshdir")
        if "eulerseq" in c.attrib:
            eulerseq = c.get("eulerseq")
    basedir = os.path.dirname(path)

    # options
    opt = dict(timestep=0.002, iterations=100, ls_iterations=50, tolerance=1e-8,
               ls_tolerance=0.01, impratio=1.0, gravity=(0.0, 0.0, -9.81),
               integrator="Euler", cone="pyramidal", solver="Newton", viscosity=0.0, density=0.0)
    disable = 0
    flag_bits = {"eulerdamp": cmodel.DSBL_EULERDAMP, "refsafe": cmodel.DSBL_REFSAFE,
                 "warmstart": cmodel.DSBL_WARMSTART, "gravity": cmodel.DSBL_GRAVITY,
                 "contact": cmodel.DSBL_CONTACT, "limit": cmodel.DSBL_LIMIT,
                 "equality": cmodel.DSBL_EQUALITY, "passive": cmodel.DSBL_PASSIVE,
                 "filterparent": cmodel.DSBL_FILTERPARENT}
    for o in root.iter("option"):
        for k in ("timestep", "tolerance", "ls_tolerance", "impratio", "viscosity", "density"):
            if k in o.attrib:
                opt[k] = float(o.get(k))
        for k in ("iterations", "ls_iterations"):
            if k in o.attrib:
                opt[k] = int(o.get(k))
        if "gravity" in o.attrib:
            opt["gravity"] = tuple(_floats(o.get("gravity"), 3))
        for k in ("integrator", "cone", "solver"):
            if k in o.attrib:
                opt[k] = o.get(k)
        for fl in o.iter("flag"):
            for k, v in fl.attrib.items():
                if k in flag_bits:
                    if v == "disable":
                        disable |= flag_bits[k]
                    else:
                        disable &= ~flag_bits[k]
    if timestep is not None:
        opt["timestep"] = float(timestep)  # SBP/mjx_planner.py:103
    integrators = {"Euler": cmodel.INT_EULER, "implicitfast": cmodel.INT_IMPLICITFAST}
    if opt["integrator"] not in integrators:
        raise MJCFError(f"integrator {opt['integrator']!r} not supported (Euler, implicitfast)")
    cones = {"pyramidal": cmodel.CONE_PYRAMIDAL, "elliptic": cmodel.CONE_ELLIPTIC}
    if opt["cone"] not in cones:
        raise MJCFError(f"cone {opt['cone']!r} not supported (pyramidal, elliptic)")
    if opt["solver"] != "Newton":
        raise MJCFError("only the Newton solver is supported")

    defaults = _Defaults()
    for d in root.findall("default"):
        defaults.parse(d)

    # meshes
    meshes = {}
    for asset in root.findall("asset"):
        for m in asset.findall("mesh"):
            a = defaults.attrs(m.get("class", "main"), "mesh", m)  # mesh scale may come from a class
            fname = a.get("file")
            name = a.get("name") or os.path.splitext(os.path.basename(fname))[0]
            scale = _floats(a.get("scale", "1 1 1"), 3)
            meshes[name] = (os.path.join(basedir, meshdir, fname), np.array(scale))

    # ---- body tree (preorder) ---------------------------------------------
    bodies = [_Body("world", -1, np.zeros(3), np.array([1.0, 0, 0, 0]))]

    def walk(belem, parent, childclass):
        for child in belem:
            tag = child.tag
            cls = child.get("class", childclass)
            if tag == "body":
                bcls = child.get("childclass", childclass)
                a = child.attrib
                b = _Body(a.get("name", f"body{len(bodies)}"), parent,
                          np.array(_floats(a.get("pos", "0 0 0"), 3)),
                          _orientation(a, angle_scale, eulerseq),
                          float(a.get("gravcomp", 0.0)))
                bodies.append(b)
                walk(child, len(bodies) - 1, bcls)
            elif tag in ("joint", "freejoint"):
                a = defaults.attrs(cls, "joint", child)
                if tag == "freejoint":
                    a = dict(child.attrib)
                    a["type"] = "free"
                bodies[parent].joints.append(a)
            elif tag == "geom":
                bodies[parent].geoms.append(defaults.attrs(cls, "geom", child))
            elif tag == "site":
                bodies[parent].sites.append(defaults.attrs(cls, "site", child))
            elif tag == "inertial":
                bodies[parent].inertial = dict(child.attrib)

    for wb in root.findall("worldbody"):
        walk(wb, 0, "main")

    m = Model()
    nbody = len(bodies)
    m.nbody = nbody
    m.opt = opt
    m.disableflags = disable

    # ---- joints & dofs --------------------------------------------------------
    jnt = []
    for bi, b in enumerate(bodies):
        for a in b.joints:
            jt = JNT_TYPES[a.get("type", "hinge")]
            rng = a.get("range")
            limited_attr = a.get("limited", "auto")
            r = _floats(rng, 2) if rng else [0.0, 0.0]
            if jt == 3:
                r = [x * angle_scale for x in r]
            if limited_attr == "true":
                limited = True
            elif limited_attr == "false":
                limited = False
            else:
                limited = bool(autolimits and rng is not None and r[0] < r[1])
            jnt.append(dict(
                name=a.get("name", f"joint{len(jnt)}"), type=jt, body=bi,
                pos=np.array(_floats(a.get("pos", "0 0 0"), 3)),
                axis=np.array(_floats(a.get("axis", "0 0 1"), 3)),
                range=r, limited=limited,
                armature=float(a.get("armature", 0.0)),
                damping=float(a.get("damping", 0.0)),
                ref=float(a.get("ref", 0.0)) * (angle_scale if jt == 3 else 1.0),
                solref=_floats(a.get("solreflimit", " ".join(map(str, DEFAULT_SOLREF))), 2),
                solimp=(_floats(a.get("solimplimit", " ".join(map(str, DEFAULT_SOLIMP))))
                        + list(DEFAULT_SOLIMP))[:5],
                margin=float(a.get("margin", 0.0)),
                stiffness=float(a.get("stiffness", 0.0)),
                springref=float(a.get("springref", 0.0)) * (angle_scale if jt == 3 else 1.0),
                actfrcrange=_floats(a["actuatorfrcrange"], 2) if "actuatorfrcrange" in a else [0.0, 0.0],
                actfrclimited=(a.get("actuatorfrclimited") == "true" or (
                    a.get("actuatorfrclimited", "auto") == "auto" and autolimits and "actuatorfrcrange" in a)),
            ))
            if np.linalg.norm(jnt[-1]["axis"]) > 0:
                jnt[-1]["axis"] = jnt[-1]["axis"] / np.linalg.norm(jnt[-1]["axis"])
    m.njnt = len(jnt)
    body_jntadr = [-1] * nbody
    body_jntnum = [0] * nbody
    for j, J in enumerate(jnt):
        if body_jntadr[J["body"]] < 0:
            body_jntadr[J["body"]] = j
        body_jntnum[J["body"]] += 1

    qposadr, dofadr = [], []
    nq = nv = 0
    for J in jnt:
        qposadr.append(nq)
        dofadr.append(nv)
        nq += JNT_NQ[J["type"]]
        nv += JNT_NV[J["type"]]
    m.nq, m.nv = nq, nv

    body_dofadr = [-1] * nbody
    body_dofnum = [0] * nbody
    dof_bodyid, dof_jntid = [], []
    for j, J in enumerate(jnt):
        for k in range(JNT_NV[J["type"]]):
            d = dofadr[j] + k
            dof_bodyid.append(J["body"])
            dof_jntid.append(j)
            if body_dofadr[J["body"]] < 0:
                body_dofadr[J["body"]] = d
            body_dofnum[J["body"]] += 1

    parent = [b.parent for b in bodies]
    # weldid: nearest ancestor-or-self with joints (0 = world)
    weld = [0] * nbody
    for i in range(1, nbody):
        weld[i] = i if body_jntnum[i] > 0 else weld[parent[i]]
    rootid = [0] * nbody
    for i in range(1, nbody):
        rootid[i] = i if parent[i] == 0 else rootid[parent[i]]

    # last dof of each body chain, for dof_parentid
    lastdof = [-1] * nbody
    dof_parentid = [-1] * nv
    for i in range(1, nbody):
        prev = lastdof[parent[i]]
        for k in range(body_dofnum[i]):
            d = body_dofadr[i] + k
            dof_parentid[d] = prev
            prev = d
        lastdof[i] = prev
    body_dofmask = [0] * nbody
    for i in range(1, nbody):
        mask = body_dofmask[parent[i]]
        for k in range(body_dofnum[i]):
            mask |= 1 << (body_dofadr[i] + k)
        body_dofmask[i] = mask
    if nv > 32:
        raise MJCFError("nv > 32 not supported by the dof bitmask")
    # trees: dofs sharing a root body
    dof_treeid = []
    roots = []
    for d in range(nv):
        r = rootid[dof_bodyid[d]]
        if r not in roots:
            roots.append(r)
        dof_treeid.append(roots.index(r))

    # ---- geoms / sites ---------------------------------------------------------
    geoms = []
    for bi, b in enumerate(bodies):
        for a in b.geoms:
            gtype = GEOM_TYPES[a.get("type", "sphere")]
            size = _floats(a.get("size", "0 0 0"))
            size = (size + [0.0, 0.0, 0.0])[:3]
            pos = np.array(_floats(a.get("pos", "0 0 0"), 3))
            quat = _orientation(a, angle_scale, eulerseq)
            if "fromto" in a:
                ft = np.array(_floats(a["fromto"], 6))
                p0, p1 = ft[:3], ft[3:]
                pos = 0.5 * (p0 + p1)
                vec = p1 - p0
                L = np.linalg.norm(vec)
                z = vec / L
                ref = np.array([0.0, 0, 1])
                ax = np.cross(ref, z)
                s = np.linalg.norm(ax)
                quat = (np.array([1.0, 0, 0, 0]) if s < 1e-12 and z[2] > 0 else
                        np.array([0.0, 1, 0, 0]) if s < 1e-12 else
                        axisangle2quat(ax / s, math.atan2(s, z[2])))
                size[1] = L / 2
            sr = _floats(a.get("solref", " ".join(map(str, DEFAULT_SOLREF))), 2)
            si = (_floats(a.get("solimp", " ".join(map(str, DEFAULT_SOLIMP)))) + list(DEFAULT_SOLIMP))[:5]
            fr = (_floats(a.get("friction", "1 0.005 0.0001")) + [0.005, 0.0001])[:3]
            geoms.append(dict(
                name=a.get("name", ""), type=gtype, body=bi, size=np.array(size),
                pos=pos, quat=quat,
                contype=int(a.get("contype", 1)), conaffinity=int(a.get("conaffinity", 1)),
                condim=int(a.get("condim", 3)), group=int(a.get("group", 0)),
                friction=fr, solref=sr, solimp=si,
                solmix=float(a.get("solmix", 1.0)), margin=float(a.get("margin", 0.0)),
                gap=float(a.get("gap", 0.0)), priority=int(a.get("priority", 0)),
                density=float(a.get("density", 1000.0)),
                mass=float(a["mass"]) if "mass" in a else None,
                mesh=a.get("mesh"),
            ))
    sites = []
    for bi, b in enumerate(bodies):
        for a in b.sites:
            sites.append(dict(name=a.get("name", ""), body=bi,
                              pos=np.array(_floats(a.get("pos", "0 0 0"), 3)),
                              quat=_orientation(a, angle_scale, eulerseq)))

    # ---- body inertia ----------------------------------------------------------
    mass = np.zeros(nbody)
    ipos = np.zeros((nbody, 3))
    iquat = np.tile([1.0, 0, 0, 0], (nbody, 1))
    inertia = np.zeros((nbody, 3))
    for bi in range(1, nbody):
        b = bodies[bi]
        if b.inertial is not None:
            a = b.inertial
            mass[bi] = float(a["mass"])
            ipos[bi] = _floats(a.get("pos", "0 0 0"), 3)
            if "diaginertia" in a:
                iquat[bi] = _orientation(a, angle_scale, eulerseq)
                inertia[bi] = _floats(a["diaginertia"], 3)
            elif "fullinertia" in a:
                f = _floats(a["fullinertia"], 6)
                I = np.array([[f[0], f[3], f[4]], [f[3], f[1], f[5]], [f[4], f[5], f[2]]])
                Rq = quat2mat(_orientation(a, angle_scale, eulerseq))
                w, V = np.linalg.eigh(Rq @ I @ Rq.T)
                if np.linalg.det(V) < 0:
                    V[:, 2] = -V[:, 2]
                iquat[bi] = mat2quat(V)
                inertia[bi] = w
            continue
        # inertia from geoms; static (world-welded) bodies never move, skip them
        if weld[bi] == 0:
            continue
        tot_m, tot_c, parts = 0.0, np.zeros(3), []
        for g in geoms:
            if g["body"] != bi or not (0 <= g["group"] <= 5) or g["type"] == 0:
                continue
            if g["type"] == 7:
                mpath, scale = meshes[g["mesh"]]
                if not os.path.exists(mpath):
                    raise MJCFError(f"mesh {mpath} needed for inertia of body {b.name!r} is missing")
                tris = load_stl(mpath) if mpath.lower().endswith(".stl") else load_obj(mpath)
                tris = tris * scale[None, None, :]
                gm, gc, gI = mesh_inertia(tris, g["density"])
                if g["mass"] is not None:
                    gI *= g["mass"] / gm
                    gm = g["mass"]
                R = quat2mat(g["quat"])
                c = g["pos"] + R @ gc
                I_b = R @ gI @ R.T
            else:
                gm, gI = geom_inertia(g["type"], g["size"], g["density"])
                if g["mass"] is not None:
                    gI = gI * (g["mass"] / gm) if gm > 0 else gI
                    gm = g["mass"]
                R = quat2mat(g["quat"])
                c = g["pos"]
                I_b = R @ gI @ R.T
            parts.append((gm, c, I_b))
            tot_m += gm
            tot_c += gm * c
        if tot_m <= 0:
            raise MJCFError(f"body {b.name!r} has dofs but no mass")
        com = tot_c / tot_m
        I = np.zeros((3, 3))
        for gm, c, I_b in parts:
            d = c - com
            I += I_b + gm * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        w, V = np.linalg.eigh(I)
        if np.linalg.det(V) < 0:
            V[:, 2] = -V[:, 2]
        mass[bi] = tot_m
        ipos[bi] = com
        iquat[bi] = mat2quat(V)
        inertia[bi] = w

    # ---- collision pairs -----------------------------------------------------
    excludes = set()
    for c in root.findall("contact"):
        for e in c.findall("exclude"):
            b1 = [b.name for b in bodies].index(e.get("body1"))
            b2 = [b.name for b in bodies].index(e.get("body2"))
            excludes.add((min(b1, b2), max(b1, b2)))
    filterparent = not (disable & cmodel.DSBL_FILTERPARENT)
    pairs = []
    for i in range(len(geoms)):
        for j in range(i + 1, len(geoms)):
            g1, g2 = geoms[i], geoms[j]
            if not ((g1["contype"] & g2["conaffinity"]) or (g2["contype"] & g1["conaffinity"])):
                continue
            b1, b2 = g1["body"], g2["body"]
            w1, w2 = weld[b1], weld[b2]
            if w1 == w2:
                continue
            wp1 = weld[parent[w1]] if w1 > 0 else 0
            wp2 = weld[parent[w2]] if w2 > 0 else 0
            if filterparent and w1 != 0 and w2 != 0 and (w1 == wp2 or w2 == wp1):
                continue
            if (min(b1, b2), max(b1, b2)) in excludes:
                continue
            a, bb = (i, j) if g1["type"] <= g2["type"] else (j, i)
            key = (geoms[a]["type"], geoms[bb]["type"])
            fn = collision_func(*key)
            if fn is None:
                raise MJCFError(f"no narrow phase for geom types {key} "
                                f"({geoms[a]['name']!r}, {geoms[bb]['name']!r})")
            func, ncon = fn
            ga, gb = geoms[a], geoms[bb]
            if func == cmodel.COL_CONVEX and {ga["type"], gb["type"]} <= {6, 7}:
                ncon = 4  # a polyhedron pair (mesh-mesh, box-mesh): the face-clipping manifold's slots
            if func == cmodel.COL_PLANE_CONVEX and gb["type"] == 5:
                ncon = 4  # plane-cylinder: MuJoCo's mjc_PlaneCylinder (up to 4 points)
            if ga["priority"] != gb["priority"]:  # the higher priority geom's parameters
                gp = ga if ga["priority"] > gb["priority"] else gb
                condim, friction = gp["condim"], gp["friction"][0]
                solref, solimp = list(gp["solref"]), list(gp["solimp"])
            else:
                # mixing (same priority): max friction/condim, solmix-weighted solref/solimp
                mix = ga["solmix"] / (ga["solmix"] + gb["solmix"]) if (ga["solmix"] + gb["solmix"]) > 0 else 0.5
                if ga["solref"][0] > 0 and gb["solref"][0] > 0:
                    solref = [mix * ga["solref"][k] + (1 - mix) * gb["solref"][k] for k in range(2)]
                else:
                    solref = [min(ga["solref"][k], gb["solref"][k]) for k in range(2)]
                solimp = [mix * ga["solimp"][k] + (1 - mix) * gb["solimp"][k] for k in range(5)]
                condim, friction = max(ga["condim"], gb["condim"]), max(ga["friction"][0], gb["friction"][0])
            pairs.append(dict(g1=a, g2=bb, func=func, ncon=ncon, condim=condim, friction=friction,
                              solref=solref, solimp=solimp,
                              margin=max(ga["margin"], gb["margin"]),
                              gap=max(ga["gap"], gb["gap"])))
    for p in pairs:
        if p["condim"] not in (1, 3):
            raise MJCFError(f"condim {p['condim']} not supported (1 and 3 only)")
    pairs.sort(key=lambda p: (p["func"], p["g1"], p["g2"]))
    robot = [g["name"] in ROBOT_GEOM_NAMES for g in geoms]
    conadr = slot = 0
    for p in pairs:
        p["conadr"] = conadr
        conadr += p["ncon"]
        if robot[p["g1"]] or robot[p["g2"]]:
            p["slotadr"] = slot
            slot += p["ncon"]
        else:
            p["slotadr"] = -1
    m.ncon = conadr
    m.nslot = slot

    # ---- equality ---------------------------------------------------------------
    eqs = []
    jnames = [J["name"] for J in jnt]
    for e in root.findall("equality"):
        for q in e:
            if q.tag == "joint":
                a = defaults.attrs(q.get("class", "main"), "equality", q)
                j1 = jnames.index(a["joint1"])
                j2 = jnames.index(a["joint2"]) if "joint2" in a else -1
                poly = (_floats(a.get("polycoef", "0 1 0 0 0")) + [0] * 5)[:5]
                eqs.append(dict(type=cmodel.EQ_JOINT, obj1=j1, obj2=j2, data=poly + [0.0],
                                solref=_floats(a.get("solref", "0.02 1"), 2),
                                solimp=(_floats(a.get("solimp", "0.9 0.95 0.001 0.5 2")) + list(DEFAULT_SOLIMP))[:5]))
            elif q.tag == "connect":
                a = defaults.attrs(q.get("class", "main"), "equality", q)
                bnames = [b.name for b in bodies]
                b1 = bnames.index(a["body1"])
                b2 = bnames.index(a["body2"]) if "body2" in a else 0
                anchor = _floats(a.get("anchor", "0 0 0"), 3)
                eqs.append(dict(type=cmodel.EQ_CONNECT, obj1=b1, obj2=b2, data=anchor + [0.0, 0.0, 0.0],
                                solref=_floats(a.get("solref", "0.02 1"), 2),
                                solimp=(_floats(a.get("solimp", "0.9 0.95 0.001 0.5 2")) + list(DEFAULT_SOLIMP))[:5]))
            else:
                raise MJCFError(f"equality <{q.tag}> not supported (joint, connect)")

    # ---- reference configuration ---------------------------------------------
    qpos0 = np.zeros(nq)
    for j, J in enumerate(jnt):
        a = qposadr[j]
        if J["type"] == 0:
            b = bodies[J["body"]]
            if b.parent != 0:
                raise MJCFError("free joints must be on children of the world body")
            qpos0[a:a + 3] = b.pos
            qpos0[a + 3:a + 7] = b.quat
        elif J["type"] == 1:
            qpos0[a:a + 4] = [1, 0, 0, 0]
        else:
            qpos0[a] = J["ref"]

    # ---- fill arrays -------------------------------------------------------------
    m.names["body"] = [b.name for b in bodies]
    m.names["joint"] = jnames
    m.names["geom"] = [g["name"] for g in geoms]
    m.names["site"] = [s["name"] for s in sites]
    m.body_parentid = np.array(parent)
    m.body_rootid = np.array(rootid)
    m.body_weldid = np.array(weld)
    m.body_jntnum = np.array(body_jntnum)
    m.body_jntadr = np.array(body_jntadr)
    m.body_dofnum = np.array(body_dofnum)
    m.body_dofadr = np.array(body_dofadr)
    m.body_dofmask = np.array(body_dofmask, dtype=np.uint64)
    m.body_pos = np.array([b.pos for b in bodies])
    m.body_quat = np.array([b.quat for b in bodies])
    m.body_ipos = ipos
    m.body_iquat = iquat
    m.body_mass = mass
    m.body_inertia = inertia
    m.body_gravcomp = np.array([b.gravcomp for b in bodies])
    m.jnt_type = np.array([J["type"] for J in jnt], dtype=np.int64)
    m.jnt_qposadr = np.array(qposadr, dtype=np.int64)
    m.jnt_dofadr = np.array(dofadr, dtype=np.int64)
    m.jnt_bodyid = np.array([J["body"] for J in jnt], dtype=np.int64)
    m.jnt_limited = np.array([int(J["limited"]) for J in jnt], dtype=np.int64)
    m.jnt_pos = np.array([J["pos"] for J in jnt]).reshape(-1, 3)
    m.jnt_axis = np.array([J["axis"] for J in jnt]).reshape(-1, 3)
    m.jnt_range = np.array([J["range"] for J in jnt]).reshape(-1, 2)
    m.jnt_solref = np.array([J["solref"] for J in jnt]).reshape(-1, 2)
    m.jnt_solimp = np.array([J["solimp"] for J in jnt]).reshape(-1, 5)
    m.jnt_margin = np.array([J["margin"] for J in jnt])
    m.jnt_stiffness = np.array([J["stiffness"] for J in jnt])
    m.jnt_springref = np.array([J["springref"] for J in jnt])
    m.jnt_actfrclimited = np.array([int(J["actfrclimited"]) for J in jnt], dtype=np.int64)
    m.jnt_actfrcrange = np.array([J["actfrcrange"] for J in jnt]).reshape(-1, 2)
    m.dof_bodyid = np.array(dof_bodyid, dtype=np.int64)
    m.dof_jntid = np.array(dof_jntid, dtype=np.int64)
    m.dof_parentid = np.array(dof_parentid, dtype=np.int64)
    m.dof_treeid = np.array(dof_treeid, dtype=np.int64)
    m.ntree = len(roots)
    m.dof_armature = np.array([jnt[dof_jntid[d]]["armature"] for d in range(nv)])
    m.dof_damping = np.array([jnt[dof_jntid[d]]["damping"] for d in range(nv)])
    m.qpos0 = qpos0
    m.qpos_init = qpos0.copy()
    m.qvel_init = np.zeros(nv)
    m.ngeom = len(geoms)
    m.geom_type = np.array([g["type"] for g in geoms], dtype=np.int64)
    m.geom_bodyid = np.array([g["body"] for g in geoms], dtype=np.int64)
    m.geom_contype = np.array([g["contype"] for g in geoms], dtype=np.int64)
    m.geom_conaffinity = np.array([g["conaffinity"] for g in geoms], dtype=np.int64)
    m.geom_condim = np.array([g["condim"] for g in geoms], dtype=np.int64)
    m.geom_robot = np.array(robot, dtype=np.int64)
    m.geom_pos = np.array([g["pos"] for g in geoms]).reshape(-1, 3)
    m.geom_quat = np.array([g["quat"] for g in geoms]).reshape(-1, 4)
    m.geom_size = np.array([g["size"] for g in geoms]).reshape(-1, 3)

    def rbound(g):
        s = g["size"]
        return {0: 0.0, 2: s[0], 3: s[0] + s[1], 4: max(s), 5: math.hypot(s[0], s[1]),
                6: float(np.linalg.norm(s))}.get(g["type"], 0.0)
    m.geom_rbound = np.array([rbound(g) for g in geoms])
    _convex_hulls(m, geoms, pairs, meshes)
    m.nsite = len(sites)
    m.site_bodyid = np.array([s["body"] for s in sites], dtype=np.int64)
    m.site_pos = np.array([s["pos"] for s in sites]).reshape(-1, 3)
    m.site_quat = np.array([s["quat"] for s in sites]).reshape(-1, 4)
    m.npair = len(pairs)
    m.pairs = pairs
    for k in ("g1", "g2", "func", "ncon", "conadr", "slotadr", "condim"):
        setattr(m, "pair_" + {"g1": "geom1", "g2": "geom2"}.get(k, k),
                np.array([p[k] for p in pairs], dtype=np.int64))
    m.pair_friction = np.array([p["friction"] for p in pairs])
    m.pair_solref = np.array([p["solref"] for p in pairs]).reshape(-1, 2)
    m.pair_solimp = np.array([p["solimp"] for p in pairs]).reshape(-1, 5)
    m.pair_margin = np.array([p["margin"] for p in pairs])
    m.pair_gap = np.array([p["gap"] for p in pairs])
    m.neq = len(eqs)
    m.eq_type = np.array([e["type"] for e in eqs], dtype=np.int64)
    m.eq_obj1 = np.array([e["obj1"] for e in eqs], dtype=np.int64)
    m.eq_obj2 = np.array([e["obj2"] for e in eqs], dtype=np.int64)
    m.eq_data = np.array([e["data"] for e in eqs]).reshape(-1, 6)
    m.eq_solref = np.array([e["solref"] for e in eqs]).reshape(-1, 2)
    m.eq_solimp = np.array([e["solimp"] for e in eqs]).reshape(-1, 5)

    # planner ids (SBP/mjx_planner.py:120-121) and controlled dofs (:254,267-270)
    m.hande_body = m.names["body"].index("hande") if "hande" in m.names["body"] else -1
    m.tcp_site = m.names["site"].index("tcp") if "tcp" in m.names["site"] else -1
    # the planner controls the leading hinge/slide dofs (qpos == qvel indexing),
    # at most 6; cem_planner refuses a model whose count differs from num_dof
    nctrl = 0
    while nctrl < min(6, nv):
        jt = m.jnt_type[m.dof_jntid[nctrl]]
        if jt not in (2, 3) or m.jnt_qposadr[m.dof_jntid[nctrl]] != nctrl:
            break
        nctrl += 1
    m.nctrl = nctrl
    m.ctrl_qposadr = np.arange(m.nctrl)
    m.ctrl_dofadr = np.arange(m.nctrl)

    _actuators(m, root, defaults, jnt, jnames, autolimits)
    m.integrator = integrators[opt["integrator"]]
    m.timestep = opt["timestep"]
    m.iterations = opt["iterations"]
    m.ls_iterations = opt["ls_iterations"]
    m.tolerance = opt["tolerance"]
    m.ls_tolerance = opt["ls_tolerance"]
    m.impratio = opt["impratio"]
    m.cone = cones[opt["cone"]]
    m.viscosity = opt["viscosity"]
    m.density = opt["density"]
    m.gravity = np.array(opt["gravity"])
    m.source = path

    _spatial_tendons(m, root, defaults)
    set_const(m)
    _connect_anchors(m)
    return m


# ---------------------------------------------------------------------------
# collision meshes, tendons / actuators, connect anchors
# ---------------------------------------------------------------------------


FACE_MAXV = 16  # vertices kept per hull face polygon (the manifold clips against them)


def _polygon_faces(hv, tris, eqs, nbrs):
    """Hull faces as planar polygons: Qhull's triangles merged across shared
    edges when their planes agree (unit normals within 1e-6, offsets within
    1e-7 of the hull's size), each face's vertices in counter-clockwise order
    about its outward normal.  Returns [(normal, offset, all vertices
    (ordered), kept vertices)]: a face with more than FACE_MAXV vertices keeps
    FACE_MAXV of them evenly spaced around it (an inscribed polygon; what the
    contact manifold clips against), the incidence lists use all of them."""
    nt = len(tris)
    parent = list(range(nt))

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a

    scale = max(float(np.max(np.linalg.norm(hv, axis=1))), 1e-9)
    for a in range(nt):
        for b in nbrs[a]:
            if b < 0 or b < a:
                continue
            if (np.abs(eqs[a, :3] - eqs[b, :3]).max() < 1e-6 and abs(eqs[a, 3] - eqs[b, 3]) < 1e-7 * scale):
                ra, rb = find(a), find(b)
                if ra != rb:
                    parent[max(ra, rb)] = min(ra, rb)
    groups = {}
    for t in range(nt):
        groups.setdefault(find(t), []).append(t)
    faces = []
    for root in sorted(groups):
        ts = groups[root]
        n = eqs[ts, :3].mean(axis=0)
        n /= np.linalg.norm(n)
        vs = sorted({int(x) for t in ts for x in tris[t]})
        P = hv[vs]
        off = float((P @ n).mean())
        # order counter-clockwise about n (angles in the face plane)
        u = np.cross(n, [1.0, 0.0, 0.0] if abs(n[0]) < 0.9 else [0.0, 1.0, 0.0])
        u /= np.linalg.norm(u)
        w = np.cross(n, u)
        c = P.mean(axis=0)
        ang = np.arctan2((P - c) @ w, (P - c) @ u)
        order = [vs[k] for k in np.argsort(ang, kind="stable")]
        kept = order if len(order) <= FACE_MAXV else [order[(k * len(order)) // FACE_MAXV] for k in range(FACE_MAXV)]
        faces.append((n, off, order, kept))
    return faces


def convex_hull(verts):
    """Hull vertices (recentred on their mean), the centre, the vertex graph
    (neighbour lists) of a point cloud -- what hill-climbing support queries
    walk (MuJoCo keeps the same graph, mesh_graph) -- and the hull's faces
    (_polygon_faces, in the recentred frame)."""
    from scipy.spatial import ConvexHull
    v = np.unique(np.asarray(verts, dtype=np.float64).reshape(-1, 3), axis=0)
    h = ConvexHull(v)
    idx = np.asarray(h.vertices)
    remap = {int(g): k for k, g in enumerate(idx)}
    hv = v[idx]
    c = hv.mean(axis=0)
    nbr = [set() for _ in idx]
    tris = np.array([[remap[int(x)] for x in tri] for tri in h.simplices], dtype=np.int64)
    for t in tris:
        for a in range(3):
            for b in range(3):
                if a != b:
                    nbr[t[a]].add(t[b])
    eqs = np.array(h.equations, dtype=np.float64)
    eqs[:, 3] = -(eqs[:, 3] + eqs[:, :3] @ c)  # n . x = offset in the recentred frame
    faces = _polygon_faces(hv - c, tris, eqs, np.asarray(h.neighbors))
    return hv - c, c, [sorted(n) for n in nbr], faces


def box_faces(size):
    """The 8 corners (bit k of the index: + side of axis k) and 6 faces
    (+x, -x, +y, -y, +z, -z) of a box in its frame, as _polygon_faces."""
    corners = np.array([[size[0] if i & 1 else -size[0], size[1] if i & 2 else -size[1],
                         size[2] if i & 4 else -size[2]] for i in range(8)], dtype=np.float64)
    faces = []
    for ax in range(3):
        for sg in (1, -1):
            n = np.zeros(3)
            n[ax] = sg
            vs = [i for i in range(8) if ((i >> ax) & 1) == (sg > 0)]
            P = corners[vs]
            u = np.zeros(3)
            u[(ax + 1) % 3] = 1.0
            w = np.cross(n, u)
            ang = np.arctan2(P @ w, P @ u)
            order = [vs[k] for k in np.argsort(ang, kind="stable")]
            faces.append((n, float(size[ax]), order, order))
    return corners, faces


def _convex_hulls(m, geoms, pairs, meshes):
    """Hulls of the mesh geoms any pair uses; the geom frame is moved to the
    hull centre (an interior point, as MuJoCo recentres meshes), which is
    where the convex narrow phase starts its portal."""
    ng = len(geoms)
    m.geom_hulladr = -np.ones(ng, dtype=np.int64)
    m.geom_hullnum = np.zeros(ng, dtype=np.int64)
    # polygon faces (the polyhedron contact manifold, mesh-mesh / box-mesh
    # pairs): per mesh hull and per box that meets a mesh; a box's 8 corners
    # go after the hull vertices (geom_cornadr), outside every climb graph
    m.geom_faceadr = -np.ones(ng, dtype=np.int64)
    m.geom_facenum = np.zeros(ng, dtype=np.int64)
    m.geom_cornadr = -np.ones(ng, dtype=np.int64)
    used = {p["g1"] for p in pairs} | {p["g2"] for p in pairs}
    poly = set()
    for p in pairs:
        t1, t2 = geoms[p["g1"]]["type"], geoms[p["g2"]]["type"]
        if {t1, t2} <= {6, 7} and 7 in (t1, t2):
            poly |= {p["g1"], p["g2"]}
    cache, verts, adjadr, adjnum, adj = {}, [], [], [], []
    faces = []  # (normal, offset, all global vertices, kept global vertices)
    for gi in sorted(used):
        g = geoms[gi]
        if g["type"] != 7:
            continue
        if g["mesh"] not in cache:
            mpath, scale = meshes[g["mesh"]]
            tris = load_stl(mpath) if mpath.lower().endswith(".stl") else load_obj(mpath)
            hv, c, nbr, fcs = convex_hull(tris.reshape(-1, 3) * scale[None, :])
            base = len(verts)
            for k, n in enumerate(nbr):
                adjadr.append(len(adj))
                adjnum.append(len(n))
                adj.extend(base + x for x in n)
            verts.extend(hv.tolist())
            fbase = len(faces)
            faces.extend((n, off, [base + x for x in al], [base + x for x in kp]) for n, off, al, kp in fcs)
            cache[g["mesh"]] = (base, len(hv), c, float(np.max(np.linalg.norm(hv, axis=1))), fbase, len(fcs))
        base, num, c, rb, fbase, nf = cache[g["mesh"]]
        m.geom_hulladr[gi] = base
        m.geom_hullnum[gi] = num
        m.geom_pos[gi] = m.geom_pos[gi] + quat2mat(m.geom_quat[gi]) @ c
        m.geom_rbound[gi] = rb
        if gi in poly:
            m.geom_faceadr[gi], m.geom_facenum[gi] = fbase, nf
    nmesh_verts = len(verts)
    for gi in sorted(poly):
        if geoms[gi]["type"] != 6:
            continue
        corners, fcs = box_faces(np.asarray(m.geom_size[gi], dtype=np.float64))
        base = len(verts)
        verts.extend(corners.tolist())
        adjadr.extend([len(adj)] * 8)
        adjnum.extend([0] * 8)
        m.geom_cornadr[gi] = base
        m.geom_faceadr[gi], m.geom_facenum[gi] = len(faces), len(fcs)
        faces.extend((n, off, [base + x for x in al], [base + x for x in kp]) for n, off, al, kp in fcs)
    m.nhullv = len(verts)
    m.nhulla = len(adj)
    m.hull_vert = np.array(verts, dtype=np.float64).reshape(-1, 3)
    m.hull_adjadr = np.array(adjadr, dtype=np.int64)
    m.hull_adjnum = np.array(adjnum, dtype=np.int64)
    m.hull_adj = np.array(adj, dtype=np.int64)
    # faces: plane (n, offset: n . x = offset on the face) and kept polygon;
    # per vertex the faces it belongs to (every vertex of a face, kept or not)
    m.nface = len(faces)
    m.face_plane = np.array([list(f[0]) + [f[1]] for f in faces], dtype=np.float64).reshape(-1, 4)
    m.face_vadr = np.cumsum([0] + [len(f[3]) for f in faces[:-1]]).astype(np.int64) if faces else np.zeros(0, np.int64)
    m.face_vnum = np.array([len(f[3]) for f in faces], dtype=np.int64)
    m.face_vert = np.array([v for f in faces for v in f[3]], dtype=np.int64)
    m.nfacev = int(m.face_vert.size)
    inc = [[] for _ in range(len(verts))]
    for fi, f in enumerate(faces):
        for v in f[2]:
            inc[v].append(fi)
    m.vert_faceadr = np.cumsum([0] + [len(x) for x in inc[:-1]]).astype(np.int64) if inc else np.zeros(0, np.int64)
    m.vert_facenum = np.array([len(x) for x in inc], dtype=np.int64)
    m.vert_face = np.array([f for x in inc for f in x], dtype=np.int64)
    m.nvface = int(m.vert_face.size)
    del nmesh_verts


def _actuators(m, root, defaults, jnt, jnames, autolimits):
    """<tendon><fixed> and <actuator> (general / motor / position) with joint
    or fixed-tendon transmissions, flattened to (dof, qpos adr, moment)."""
    tendons = {}
    for t in root.findall("tendon"):
        for f in t.findall("fixed"):
            tendons[f.get("name")] = [(jnames.index(j.get("joint")), float(j.get("coef", 1.0)))
                                      for j in f.findall("joint")]
    acts = []
    for a_el in root.findall("actuator"):
        for el in a_el:
            tag = el.tag
            if tag not in ("general", "motor", "position"):
                raise MJCFError(f"actuator <{tag}> not supported (general, motor, position)")
            a = defaults.attrs(el.get("class", "main"), tag, el)
            gear = _floats(a.get("gear", "1"))[0]
            if "joint" in a:
                j = jnames.index(a["joint"])
                trn = [(j, gear)]
            elif "tendon" in a:
                trn = [(j, c * gear) for j, c in tendons[a["tendon"]]]
            else:
                raise MJCFError("actuators need a joint or tendon transmission")
            if len(trn) > 2:
                raise MJCFError("tendon transmissions of more than 2 joints are not supported")
            if tag == "motor":
                gaintype, biastype, gp, bp = "fixed", "none", [1.0, 0, 0], [0.0, 0, 0]
            elif tag == "position":
                kp = float(a.get("kp", 1.0))
                kv = float(a.get("kv", 0.0))
                gaintype, biastype, gp, bp = "fixed", "affine", [kp, 0, 0], [0.0, -kp, -kv]
            else:
                gaintype, biastype = a.get("gaintype", "fixed"), a.get("biastype", "none")
                gp = (_floats(a.get("gainprm", "1")) + [0.0, 0.0])[:3]
                bp = (_floats(a.get("biasprm", "0")) + [0.0, 0.0, 0.0])[:3]
            if gaintype not in ("fixed", "affine") or biastype not in ("none", "affine"):
                raise MJCFError(f"gaintype {gaintype!r} / biastype {biastype!r} not supported")

            def lim(name):
                rng = _floats(a[name + "range"], 2) if name + "range" in a else [0.0, 0.0]
                flag = a.get(name + "limited", "auto")
                on = flag == "true" or (flag == "auto" and autolimits and name + "range" in a)
                return rng, int(on)
            cr, cl = lim("ctrl")
            fr, fl = lim("force")
            acts.append(dict(trn=trn, gaintype=0 if gaintype == "fixed" else 1,
                             biastype=0 if biastype == "none" else 1, gainprm=gp, biasprm=bp,
                             ctrlrange=cr, ctrllimited=cl, forcerange=fr, forcelimited=fl))
    m.nu = len(acts)
    nu = max(m.nu, 0)
    m.act_ntrn = np.array([len(a["trn"]) for a in acts], dtype=np.int64)
    m.act_dof = np.array([[m.jnt_dofadr[j] for j, _ in a["trn"]] + [-1] * (2 - len(a["trn"])) for a in acts],
                         dtype=np.int64).reshape(nu, 2)
    m.act_qadr = np.array([[m.jnt_qposadr[j] for j, _ in a["trn"]] + [-1] * (2 - len(a["trn"])) for a in acts],
                          dtype=np.int64).reshape(nu, 2)
    m.act_moment = np.array([[c for _, c in a["trn"]] + [0.0] * (2 - len(a["trn"])) for a in acts]).reshape(nu, 2)
    for k in ("gaintype", "biastype", "ctrllimited", "forcelimited"):
        setattr(m, "act_" + k, np.array([a[k] for a in acts], dtype=np.int64))
    for k, w in (("gainprm", 3), ("biasprm", 3), ("ctrlrange", 2), ("forcerange", 2)):
        setattr(m, "act_" + k, np.array([a[k] for a in acts], dtype=np.float64).reshape(nu, w))
    m.act_ctrl = np.zeros(nu)  # MjData.ctrl starts at 0 and the reference never sets it


def _spatial_tendons(m, root, defaults):
    """<tendon><spatial> through exactly two sites (no wrapping geoms, no
    pulleys), kept for their length limits (scene_robotiq_hande.xml:34-39).
    Limit solref/solimp/margin default as MuJoCo's tendon defaults."""
    sites = m.names["site"]
    ten = []
    for t in root.findall("tendon"):
        for sp in t.findall("spatial"):
            a = defaults.attrs(sp.get("class", "main"), "tendon", sp)
            kids = list(sp)
            if len(kids) != 2 or any(k.tag != "site" for k in kids):
                raise MJCFError("spatial tendons must run through exactly two sites")
            s1, s2 = (sites.index(k.get("site")) for k in kids)
            rng = _floats(a.get("range", "0 0"), 2)
            flag = a.get("limited", "auto")
            lim = flag == "true" or (flag == "auto" and "range" in a)
            ten.append(dict(site=(s1, s2), limited=int(lim), range=rng,
                            solref=(_floats(a.get("solreflimit", "0.02 1")) + [1.0])[:2],
                            solimp=(_floats(a.get("solimplimit", "0.9 0.95 0.001 0.5 2"))
                                    + [0.5, 2.0])[:5],
                            margin=float(a.get("margin", 0.0))))
    m.nten = len(ten)
    n = m.nten
    m.ten_site = np.array([t["site"] for t in ten], dtype=np.int64).reshape(n, 2)
    m.ten_limited = np.array([t["limited"] for t in ten], dtype=np.int64)
    m.ten_range = np.array([t["range"] for t in ten], dtype=np.float64).reshape(n, 2)
    m.ten_solref = np.array([t["solref"] for t in ten], dtype=np.float64).reshape(n, 2)
    m.ten_solimp = np.array([t["solimp"] for t in ten], dtype=np.float64).reshape(n, 5)
    m.ten_margin = np.array([t["margin"] for t in ten], dtype=np.float64)
    m.ten_invweight0 = np.zeros(n)


def tendon_jac(m, k, t):
    """Length and moment row (nv) of spatial tendon t at the kinematics k."""
    s1, s2 = m.ten_site[t]
    p = [k["xpos"][m.site_bodyid[s]] + k["xmat"][m.site_bodyid[s]] @ m.site_pos[s] for s in (s1, s2)]
    dif = p[1] - p[0]
    L = float(np.linalg.norm(dif))
    j1, _ = body_jac(m, k, m.site_bodyid[s1], p[0])
    j2, _ = body_jac(m, k, m.site_bodyid[s2], p[1])
    return L, (dif / max(L, 1e-15)) @ (j2 - j1)


def _connect_anchors(m):
    """eq_data[3:6] of connect equalities: the body1 anchor expressed in
    body2's frame at qpos0 (MuJoCo's compiler does the same)."""
    if not m.neq or not (m.eq_type == cmodel.EQ_CONNECT).any():
        return
    k = kinematics0(m, m.qpos0)
    for e in range(m.neq):
        if m.eq_type[e] != cmodel.EQ_CONNECT:
            continue
        b1, b2 = m.eq_obj1[e], m.eq_obj2[e]
        p = k["xpos"][b1] + k["xmat"][b1] @ m.eq_data[e, :3]
        m.eq_data[e, 3:6] = k["xmat"][b2].T @ (p - k["xpos"][b2])


# ---------------------------------------------------------------------------
# mj_setConst restatement: invweight0 and meaninertia at qpos0
# ---------------------------------------------------------------------------


def _cross(a, b):
    return np.cross(a, b)


def kinematics0(m, qpos):
    """Body frames, COM quantities, cdof and the joint-space inertia at qpos."""
    nb = m.nbody
    xpos = np.zeros((nb, 3))
    xquat = np.tile([1.0, 0, 0, 0], (nb, 1))
    xanchor = np.zeros((m.njnt, 3))
    xaxis = np.zeros((m.njnt, 3))
    for b in range(1, nb):
        p = m.body_parentid[b]
        pos = xpos[p] + quat2mat(xquat[p]) @ m.body_pos[b]
        quat = quat_mul(xquat[p], m.body_quat[b])
        for j in range(m.body_jntadr[b], m.body_jntadr[b] + m.body_jntnum[b]) if m.body_jntnum[b] else []:
            t = m.jnt_type[j]
            a = m.jnt_qposadr[j]
            if t == 0:
                pos = qpos[a:a + 3].copy()
                quat = quat_normalize(qpos[a + 3:a + 7])
                xanchor[j] = pos
                xaxis[j] = [0, 0, 1]
                continue
            R = quat2mat(quat)
            xaxis[j] = R @ m.jnt_axis[j]
            xanchor[j] = R @ m.jnt_pos[j] + pos
            if t == 2:
                pos = pos + xaxis[j] * (qpos[a] - m.qpos0[a])
            elif t == 3:
                quat = quat_mul(quat, axisangle2quat(m.jnt_axis[j], qpos[a] - m.qpos0[a]))
                pos = xanchor[j] - quat2mat(quat) @ m.jnt_pos[j]
        xpos[b] = pos
        xquat[b] = quat_normalize(quat)
    xmat = np.array([quat2mat(q) for q in xquat])
    xipos = np.array([xpos[b] + xmat[b] @ m.body_ipos[b] for b in range(nb)])
    # subtree com
    mass = m.body_mass
    sm = mass.copy()
    smc = mass[:, None] * xipos
    for b in range(nb - 1, 0, -1):
        p = m.body_parentid[b]
        sm[p] += sm[b]
        smc[p] += smc[b]
    subtree_com = np.where(sm[:, None] > 1e-15, smc / np.maximum(sm[:, None], 1e-300), xipos)
    # cinert (10-vector) about subtree_com[root]
    cinert = np.zeros((nb, 6, 6))  # full spatial inertia matrix for simplicity
    for b in range(1, nb):
        R = xmat[b] @ quat2mat(m.body_iquat[b])
        Ic = R @ np.diag(m.body_inertia[b]) @ R.T
        d = xipos[b] - subtree_com[m.body_rootid[b]]
        mb = mass[b]
        I = Ic + mb * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        dx = np.array([[0, -d[2], d[1]], [d[2], 0, -d[0]], [-d[1], d[0], 0]])
        S = np.zeros((6, 6))
        S[:3, :3] = I
        S[:3, 3:] = mb * dx
        S[3:, :3] = -mb * dx
        S[3:, 3:] = mb * np.eye(3)
        cinert[b] = S
    cdof = np.zeros((m.nv, 6))
    for j in range(m.njnt):
        b = m.jnt_bodyid[j]
        d0 = m.jnt_dofadr[j]
        off = subtree_com[m.body_rootid[b]] - xanchor[j]
        t = m.jnt_type[j]
        if t == 0:
            for k in range(3):
                cdof[d0 + k, 3 + k] = 1.0
            for k in range(3):
                ax = xmat[b][:, k]
                cdof[d0 + 3 + k, :3] = ax
                cdof[d0 + 3 + k, 3:] = np.cross(ax, off)
        elif t == 1:
            for k in range(3):
                ax = xmat[b][:, k]
                cdof[d0 + k, :3] = ax
                cdof[d0 + k, 3:] = np.cross(ax, off)
        elif t == 2:
            cdof[d0, 3:] = xaxis[j]
        else:
            cdof[d0, :3] = xaxis[j]
            cdof[d0, 3:] = np.cross(xaxis[j], off)
    crb = cinert.copy()
    for b in range(nb - 1, 0, -1):
        p = m.body_parentid[b]
        if p > 0:
            crb[p] += crb[b]
    M = np.zeros((m.nv, m.nv))
    for i in range(m.nv):
        f = crb[m.dof_bodyid[i]] @ cdof[i]
        j = i
        while j >= 0:
            M[i, j] = M[j, i] = cdof[j] @ f
            j = m.dof_parentid[j]
        M[i, i] += m.dof_armature[i]
    return dict(xpos=xpos, xquat=xquat, xmat=xmat, xipos=xipos, subtree_com=subtree_com,
                cdof=cdof, M=M)


def body_jac(m, k, b, point):
    """Translational / rotational Jacobian (3 x nv each) of a point on body b."""
    jp = np.zeros((3, m.nv))
    jr = np.zeros((3, m.nv))
    com = k["subtree_com"][m.body_rootid[b]]
    for d in range(m.nv):
        if int(m.body_dofmask[b]) >> d & 1:
            c = k["cdof"][d]
            jr[:, d] = c[:3]
            jp[:, d] = c[3:] + np.cross(c[:3], point - com)
    return jp, jr


def set_const(m):
    k = kinematics0(m, m.qpos0)
    M = k["M"]
    Minv = np.linalg.inv(M) if m.nv else np.zeros((0, 0))
    m.meaninertia = float(np.trace(M) / m.nv) if m.nv else 1.0
    iw = np.zeros((m.nbody, 2))
    for b in range(1, m.nbody):
        if m.body_weldid[b] == 0:
            continue
        jp, jr = body_jac(m, k, b, k["xipos"][b])
        J = np.vstack([jp, jr])
        A = J @ Minv @ J.T
        iw[b, 0] = (A[0, 0] + A[1, 1] + A[2, 2]) / 3
        iw[b, 1] = (A[3, 3] + A[4, 4] + A[5, 5]) / 3
    m.body_invweight0 = iw
    dw = np.zeros(m.nv)
    for j in range(m.njnt):
        d0 = m.jnt_dofadr[j]
        t = m.jnt_type[j]
        if t == 0:
            dw[d0:d0 + 3] = np.mean(np.diag(Minv)[d0:d0 + 3])
            dw[d0 + 3:d0 + 6] = np.mean(np.diag(Minv)[d0 + 3:d0 + 6])
        elif t == 1:
            dw[d0:d0 + 3] = np.mean(np.diag(Minv)[d0:d0 + 3])
        else:
            dw[d0] = Minv[d0, d0]
    m.dof_invweight0 = dw
    # tendon_invweight0 = J_ten M^-1 J_ten^T (mj_setConst)
    for t in range(getattr(m, "nten", 0)):
        _, J = tendon_jac(m, k, t)
        m.ten_invweight0[t] = float(J @ Minv @ J)
    return m


def compile_blob(path: str, timestep: float = 0.0) -> bytes:
    """The serialised mpcr_model_t of an MJCF file (timestep <= 0: the file's
    own): what libmpcr_mjcf.so hands to mpcr_model_from_blob when
    mpcr_model_load is given an .xml path (the C-ABI's MJCF entry)."""
    m = compile_mjcf(path, timestep if timestep and timestep > 0 else None)
    return bytes(m.to_struct())


def load_model(path: str, timestep: float | None = None) -> Model:
    """Load an MJCF (.xml) or a precompiled model bundle (.npz)."""
    if path.endswith(".npz"):
        from . import models as _models
        return _models.load_bundle(path, timestep)
    return compile_mjcf(path, timestep)

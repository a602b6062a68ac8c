"""ctypes mirror of ``mpcr_model_t`` (include/mpcr_model.h) and the packer.

Kept field-for-field identical to the C header; ``tests/test_model.py`` checks
``ctypes.sizeof`` against the size the C library reports.
"""

from __future__ import annotations

import ctypes

import numpy as np

MAGIC = 0x4D504352
VERSION = 9  # v9: no support start table (the engine builds it from hull_vert)

MAX_BODY, MAX_JNT, MAX_DOF, MAX_NQ = 48, 40, 32, 48
MAX_GEOM, MAX_SITE, MAX_PAIR, MAX_EQ = 128, 24, 768, 8
MAX_SLOT, MAX_CTRL, MAX_ACT = 512, 8, 16
MAX_HULLV, MAX_HULLA = 8192, 49152
MAX_TEN = 4
MAX_FACE, MAX_FACEV, MAX_VFACE, FACE_MAXV = 12288, 49152, 65536, 16

COL_PLANE_CAPSULE, COL_PLANE_BOX, COL_CAPSULE_CAPSULE, COL_CAPSULE_BOX, COL_BOX_BOX = 0, 1, 2, 3, 4
COL_PLANE_SPHERE, COL_SPHERE_SPHERE, COL_SPHERE_CAPSULE, COL_SPHERE_BOX = 5, 6, 7, 8
COL_CONVEX, COL_PLANE_CONVEX = 9, 10
EQ_CONNECT, EQ_JOINT = 0, 2
INT_EULER, INT_IMPLICITFAST = 0, 3
CONE_PYRAMIDAL, CONE_ELLIPTIC = 0, 1
GAIN_FIXED, GAIN_AFFINE = 0, 1
BIAS_NONE, BIAS_AFFINE = 0, 1

DSBL_EULERDAMP, DSBL_REFSAFE, DSBL_WARMSTART, DSBL_GRAVITY = 1, 2, 4, 8
DSBL_CONTACT, DSBL_LIMIT, DSBL_EQUALITY, DSBL_PASSIVE, DSBL_FILTERPARENT = 16, 32, 64, 128, 256

_i, _u, _d = ctypes.c_int32, ctypes.c_uint32, ctypes.c_double


def _a(t, *dims):
    for n in reversed(dims):
        t = t * n
    return t


class mpcr_model_t(ctypes.Structure):
    _fields_ = [
        ("magic", _u), ("version", _u), ("nbytes", _u), ("pad0", _u),
        ("nbody", _i), ("njnt", _i), ("nq", _i), ("nv", _i), ("ngeom", _i), ("nsite", _i),
        ("npair", _i), ("neq", _i), ("ncon", _i), ("nslot", _i), ("nctrl", _i),
        ("hande_body", _i), ("tcp_site", _i), ("iterations", _i), ("ls_iterations", _i),
        ("disableflags", _i), ("integrator", _i), ("cone", _i), ("ntree", _i),
        ("nu", _i), ("nhullv", _i), ("nhulla", _i), ("pad_sz", _i),
        ("timestep", _d), ("tolerance", _d), ("ls_tolerance", _d), ("impratio", _d),
        ("meaninertia", _d), ("gravity", _a(_d, 3)), ("pad1", _d),
        ("body_parentid", _a(_i, MAX_BODY)), ("body_rootid", _a(_i, MAX_BODY)),
        ("body_weldid", _a(_i, MAX_BODY)), ("body_jntnum", _a(_i, MAX_BODY)),
        ("body_jntadr", _a(_i, MAX_BODY)), ("body_dofnum", _a(_i, MAX_BODY)),
        ("body_dofadr", _a(_i, MAX_BODY)), ("body_dofmask", _a(_u, MAX_BODY)),
        ("body_pos", _a(_d, MAX_BODY, 3)), ("body_quat", _a(_d, MAX_BODY, 4)),
        ("body_ipos", _a(_d, MAX_BODY, 3)), ("body_iquat", _a(_d, MAX_BODY, 4)),
        ("body_mass", _a(_d, MAX_BODY)), ("body_inertia", _a(_d, MAX_BODY, 3)),
        ("body_gravcomp", _a(_d, MAX_BODY)), ("body_invweight0", _a(_d, MAX_BODY, 2)),
        ("jnt_type", _a(_i, MAX_JNT)), ("jnt_qposadr", _a(_i, MAX_JNT)),
        ("jnt_dofadr", _a(_i, MAX_JNT)), ("jnt_bodyid", _a(_i, MAX_JNT)),
        ("jnt_limited", _a(_i, MAX_JNT)),
        ("jnt_pos", _a(_d, MAX_JNT, 3)), ("jnt_axis", _a(_d, MAX_JNT, 3)),
        ("jnt_range", _a(_d, MAX_JNT, 2)), ("jnt_solref", _a(_d, MAX_JNT, 2)),
        ("jnt_solimp", _a(_d, MAX_JNT, 5)), ("jnt_margin", _a(_d, MAX_JNT)),
        ("jnt_stiffness", _a(_d, MAX_JNT)), ("jnt_springref", _a(_d, MAX_JNT)),
        ("jnt_actfrclimited", _a(_i, MAX_JNT)), ("jnt_actfrcrange", _a(_d, MAX_JNT, 2)),
        ("dof_bodyid", _a(_i, MAX_DOF)), ("dof_jntid", _a(_i, MAX_DOF)),
        ("dof_parentid", _a(_i, MAX_DOF)), ("dof_treeid", _a(_i, MAX_DOF)),
        ("dof_armature", _a(_d, MAX_DOF)), ("dof_damping", _a(_d, MAX_DOF)),
        ("dof_invweight0", _a(_d, MAX_DOF)),
        ("qpos0", _a(_d, MAX_NQ)), ("qpos_init", _a(_d, MAX_NQ)), ("qvel_init", _a(_d, MAX_DOF)),
        ("geom_type", _a(_i, MAX_GEOM)), ("geom_bodyid", _a(_i, MAX_GEOM)),
        ("geom_contype", _a(_i, MAX_GEOM)), ("geom_conaffinity", _a(_i, MAX_GEOM)),
        ("geom_condim", _a(_i, MAX_GEOM)), ("geom_robot", _a(_i, MAX_GEOM)),
        ("geom_pos", _a(_d, MAX_GEOM, 3)), ("geom_quat", _a(_d, MAX_GEOM, 4)),
        ("geom_size", _a(_d, MAX_GEOM, 3)), ("geom_rbound", _a(_d, MAX_GEOM)),
        ("site_bodyid", _a(_i, MAX_SITE)), ("site_pos", _a(_d, MAX_SITE, 3)),
        ("site_quat", _a(_d, MAX_SITE, 4)),
        ("pair_geom1", _a(_i, MAX_PAIR)), ("pair_geom2", _a(_i, MAX_PAIR)),
        ("pair_func", _a(_i, MAX_PAIR)), ("pair_ncon", _a(_i, MAX_PAIR)),
        ("pair_conadr", _a(_i, MAX_PAIR)), ("pair_slotadr", _a(_i, MAX_PAIR)),
        ("pair_condim", _a(_i, MAX_PAIR)), ("pad2", _i),
        ("pair_friction", _a(_d, MAX_PAIR)), ("pair_solref", _a(_d, MAX_PAIR, 2)),
        ("pair_solimp", _a(_d, MAX_PAIR, 5)), ("pair_margin", _a(_d, MAX_PAIR)),
        ("pair_gap", _a(_d, MAX_PAIR)),
        ("eq_type", _a(_i, MAX_EQ)), ("eq_obj1", _a(_i, MAX_EQ)), ("eq_obj2", _a(_i, MAX_EQ)),
        ("pad3", _i), ("eq_data", _a(_d, MAX_EQ, 6)), ("eq_solref", _a(_d, MAX_EQ, 2)),
        ("eq_solimp", _a(_d, MAX_EQ, 5)),
        ("ctrl_qposadr", _a(_i, MAX_CTRL)), ("ctrl_dofadr", _a(_i, MAX_CTRL)),
        ("act_ntrn", _a(_i, MAX_ACT)), ("act_dof", _a(_i, MAX_ACT, 2)), ("act_qadr", _a(_i, MAX_ACT, 2)),
        ("act_gaintype", _a(_i, MAX_ACT)), ("act_biastype", _a(_i, MAX_ACT)),
        ("act_ctrllimited", _a(_i, MAX_ACT)), ("act_forcelimited", _a(_i, MAX_ACT)), ("pad4", _i),
        ("act_moment", _a(_d, MAX_ACT, 2)), ("act_gainprm", _a(_d, MAX_ACT, 3)),
        ("act_biasprm", _a(_d, MAX_ACT, 3)), ("act_ctrlrange", _a(_d, MAX_ACT, 2)),
        ("act_forcerange", _a(_d, MAX_ACT, 2)), ("act_ctrl", _a(_d, MAX_ACT)),
        ("geom_hulladr", _a(_i, MAX_GEOM)), ("geom_hullnum", _a(_i, MAX_GEOM)),
        ("hull_adjadr", _a(_i, MAX_HULLV)), ("hull_adjnum", _a(_i, MAX_HULLV)),
        ("hull_adj", _a(_i, MAX_HULLA)), ("hull_vert", _a(_d, MAX_HULLV, 3)),
        ("viscosity", _d), ("density", _d), ("nten", _i), ("pad5", _i),
        ("ten_site", _a(_i, MAX_TEN, 2)), ("ten_limited", _a(_i, MAX_TEN)),
        ("ten_range", _a(_d, MAX_TEN, 2)), ("ten_solref", _a(_d, MAX_TEN, 2)),
        ("ten_solimp", _a(_d, MAX_TEN, 5)), ("ten_margin", _a(_d, MAX_TEN)),
        ("ten_invweight0", _a(_d, MAX_TEN)),
        ("nface", _i), ("nfacev", _i), ("nvface", _i), ("pad6", _i),
        ("geom_faceadr", _a(_i, MAX_GEOM)), ("geom_facenum", _a(_i, MAX_GEOM)), ("geom_cornadr", _a(_i, MAX_GEOM)),
        ("face_vadr", _a(_i, MAX_FACE)), ("face_vnum", _a(_i, MAX_FACE)), ("face_vert", _a(_i, MAX_FACEV)),
        ("vert_faceadr", _a(_i, MAX_HULLV)), ("vert_facenum", _a(_i, MAX_HULLV)), ("vert_face", _a(_i, MAX_VFACE)),
        ("face_plane", _a(_d, MAX_FACE, 4)),
    ]


_LIMITS = dict(nbody=MAX_BODY, njnt=MAX_JNT, nv=MAX_DOF, nq=MAX_NQ, ngeom=MAX_GEOM,
               nsite=MAX_SITE, npair=MAX_PAIR, neq=MAX_EQ, nslot=MAX_SLOT, nctrl=MAX_CTRL, nu=MAX_ACT,
               nhullv=MAX_HULLV, nhulla=MAX_HULLA, nten=MAX_TEN, nface=MAX_FACE, nfacev=MAX_FACEV,
               nvface=MAX_VFACE)

# struct field -> Model attribute (when the names differ)
_ALIASES = {}


def _fill(dst, src):
    src = np.asarray(src)
    if src.size == 0:
        return
    view = np.ctypeslib.as_array(dst)
    flat = np.ravel(src)
    inner = view.shape[1] if view.ndim == 2 else 1
    if view.ndim == 2 and src.ndim == 2 and src.shape[1] != inner:
        rows = np.zeros((src.shape[0], inner))
        rows[:, :src.shape[1]] = src
        flat = rows.ravel()
    view.reshape(-1)[:flat.size] = flat.astype(view.dtype)


def pack(m) -> mpcr_model_t:
    for k, lim in _LIMITS.items():
        if getattr(m, k, 0) > lim:
            raise ValueError(f"model {k}={getattr(m, k)} exceeds capacity {lim}")
    s = mpcr_model_t()
    s.magic = MAGIC
    s.version = VERSION
    s.nbytes = ctypes.sizeof(mpcr_model_t)
    scalars = ("nbody", "njnt", "nq", "nv", "ngeom", "nsite", "npair", "neq", "ncon", "nslot",
               "nctrl", "hande_body", "tcp_site", "iterations", "ls_iterations", "disableflags",
               "ntree", "timestep", "tolerance", "ls_tolerance", "impratio", "meaninertia")
    for k in ("nu", "nhullv", "nhulla", "integrator", "cone", "nten", "nface", "nfacev", "nvface"):
        setattr(s, k, int(getattr(m, k, 0)))
    for k in ("geom_faceadr", "geom_cornadr"):  # -1: no faces / corners (models without polyhedron pairs)
        np.ctypeslib.as_array(getattr(s, k))[:] = -1
    for k in ("viscosity", "density"):
        setattr(s, k, float(getattr(m, k, 0.0)))
    for k in scalars:
        setattr(s, k, getattr(m, k))
    for k in range(3):
        s.gravity[k] = float(m.gravity[k])
    for name, _ in mpcr_model_t._fields_:
        if name in scalars or name.startswith("pad") or name in ("magic", "version", "nbytes", "gravity",
                                                                 "integrator", "cone", "nu", "nhullv",
                                                                 "nhulla", "nten", "viscosity", "density",
                                                                 "nface", "nfacev", "nvface"):
            continue
        attr = _ALIASES.get(name, name)
        if hasattr(m, attr):
            _fill(getattr(s, name), getattr(m, attr))
    return s

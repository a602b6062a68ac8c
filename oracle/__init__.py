"""CPU oracle — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package.  The product path
(``manipulator_mujoco_amd``) never imports, links or executes anything here.

* ``liboracle.so`` (built from ``mpcr_oracle.c`` by ``make``): fp64 scalar C
  restatement of the rollout + MuJoCo step + cost (see the header of
  ``mpcr_oracle.c`` for what is pinned and what is "parity unpinned");
* ``cem_np``: numpy transliterations of the reference's pure-algebra planner
  pieces (basis, projection, cost, elite, mean/cov update).
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build(force: bool = False) -> str:
    """liboracle.so (fp64, the checker) and liboracle_f32.so (the same source
    in float: bench.py's cpu_baseline and the parity bar's fp32 probe)."""
    path = os.path.join(_HERE, "liboracle.so")
    srcs = [os.path.join(_HERE, f) for f in ("mpcr_oracle.c", "oracle_f32.c")] + [
        os.path.join(os.path.dirname(_HERE), "include", "mpcr_model.h")]
    outs = [path, os.path.join(_HERE, "liboracle_f32.so")]
    newest = max(os.path.getmtime(f) for f in srcs)
    if force or any(not os.path.exists(o) or os.path.getmtime(o) < newest for o in outs):
        subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        if os.environ.get("MPCR_ORACLE_CRASH_BT"):
            _LIB.oracle_install_crash_bt()
        dp = ctypes.POINTER(ctypes.c_double)
        _LIB.oracle_rollout.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp, dp,
                                        dp, dp, dp, ctypes.POINTER(ctypes.c_int), ctypes.c_double,
                                        ctypes.c_uint, ctypes.c_int]
        _LIB.oracle_rollout.restype = ctypes.c_int
        _LIB.oracle_step.argtypes = [ctypes.c_void_p, dp, dp, dp, dp, dp, dp, dp, dp, dp,
                                     ctypes.POINTER(ctypes.c_int)]
        _LIB.oracle_step.restype = ctypes.c_int
        _LIB.oracle_model_size.restype = ctypes.c_int
        _LIB.oracle_cone_eval.argtypes = [ctypes.c_double] + [dp] * 4 + [ctypes.c_double] + [dp] * 4
        _LIB.oracle_cone_eval.restype = ctypes.c_int
        _LIB.oracle_set_floor.argtypes = [ctypes.c_int, ctypes.c_double]
    return _LIB


FLOOR_DEFAULTS = (1e-6, 0.0, 1e-6, 1e-5)  # Newton, support band, support tie, MPR tol (mpcr_oracle.c g_floor)
DEFAULT_EXACT = 1 | 2 | 4  # mpcr_oracle.c g_exact: MuJoCo's Newton / line-search stop, ccd_tolerance


def _both():
    return (lib(), lib_f32())


class exact:
    """Context manager: run the oracle (fp64 and fp32 builds) with the rules
    of the EXACT_* mask MuJoCo-exact (no kernel-matching floors, bands or
    tolerances; oracle_set_exact in mpcr_oracle.c) and, optionally, the
    other rules at the given values (``floors``: Newton floor, support band,
    support tie (< 0: mju_sign), MPR tolerance).  Global to the libraries:
    not for concurrent callers."""

    def __init__(self, mask=31, floors=None):
        self.mask = int(mask)  # EXACT_* bits of mpcr_oracle.c; 31 = every rule
        self.floors = floors

    def __enter__(self):
        self.prev = lib().oracle_get_exact()
        for L in _both():
            L.oracle_set_exact(self.mask)
            if self.floors is not None:
                for k, v in enumerate(self.floors):
                    L.oracle_set_floor(k, float(v))
        return self

    def __exit__(self, *exc):
        for L in _both():
            L.oracle_set_exact(self.prev)
            if self.floors is not None:
                for k, v in enumerate(FLOOR_DEFAULTS):
                    L.oracle_set_floor(k, float(v))
        return False


_LIB32 = None


def lib_f32():
    """The fp32 build (oracle_f32.c: every double of the oracle as float) --
    bench.py's cpu_baseline only; the parity checker is the fp64 build."""
    global _LIB32
    if _LIB32 is None:
        build()
        _LIB32 = ctypes.CDLL(os.path.join(_HERE, "liboracle_f32.so"))
        fp = ctypes.POINTER(ctypes.c_float)
        _LIB32.oracle_rollout.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, fp, fp, fp, fp, fp, fp,
                                          fp, fp, fp, ctypes.POINTER(ctypes.c_int), ctypes.c_float,
                                          ctypes.c_uint, ctypes.c_int]
        _LIB32.oracle_rollout.restype = ctypes.c_int
        _LIB32.oracle_set_floor.argtypes = [ctypes.c_int, ctypes.c_float]  # double is float in that build
    return _LIB32


def _f32_type(t):
    if t is ctypes.c_double:
        return ctypes.c_float
    if isinstance(t, type) and issubclass(t, ctypes.Array):
        return _f32_type(t._type_) * t._length_
    return t


def struct_f32(model):
    """The compiled model as the fp32 build's struct: the same header with
    float fields (oracle_f32.c), values rounded from the fp64 struct."""
    s = model.to_struct()
    F = type("mpcr_model_f32_t", (ctypes.Structure,),
             {"_fields_": [(n, _f32_type(t)) for n, t in type(s)._fields_]})
    f = F()
    for n, t in type(s)._fields_:
        v = getattr(s, n)
        if isinstance(v, ctypes.Array):
            np.ctypeslib.as_array(getattr(f, n))[...] = np.ctypeslib.as_array(v)
        else:
            setattr(f, n, v)
    f.nbytes = ctypes.sizeof(F)
    return f


def _p(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def rollout(model, thetadot, q0, w, ptgt, qtgt, want_theta=True, want_slots=False, want_eef=False, workers=None,
            noise=0.0, seed=0):
    """fp64 oracle rollout; thetadot is (n, nctrl*H) joint-major.  workers > 1
    splits the candidates over that many threads (test checker only).
    noise > 0: after every step qpos / qvel / warm start are scaled by
    (1 + noise * u), u uniform in [-1, 1) keyed by (seed, candidate, step) --
    the conditioning probe of tests/parity_util.py."""
    s = model.to_struct()
    td = np.ascontiguousarray(thetadot, dtype=np.float64)
    n = td.shape[0]
    nc = model.nctrl
    H = td.shape[1] // nc
    cost4 = np.zeros((n, 4))
    theta = np.zeros((n, nc * H)) if want_theta else None
    slots = np.zeros((n, H, max(model.nslot, 1))) if want_slots else None
    eef = np.zeros((n, H, 7)) if want_eef else None
    info = np.zeros((n, 3), dtype=np.int32)
    q0 = np.ascontiguousarray(q0, dtype=np.float64)
    w = np.ascontiguousarray(w, dtype=np.float64)
    pt = np.ascontiguousarray(ptgt, dtype=np.float64)
    qt = np.ascontiguousarray(qtgt, dtype=np.float64)
    L = lib()

    def run(a, b):  # rows [a, b); ctypes drops the GIL, the C side allocates per call
        def sub(x):
            return None if x is None else x[a:b]
        return L.oracle_rollout(ctypes.byref(s), b - a, H, _p(td[a:b]), _p(q0), _p(w), _p(pt), _p(qt),
                                _p(cost4[a:b]), _p(sub(theta)), _p(sub(slots)), _p(sub(eef)),
                                info[a:b].ctypes.data_as(ctypes.POINTER(ctypes.c_int)), float(noise), int(seed), int(a))

    nw = max(1, min(workers or 1, n // 16))
    if nw == 1:
        st = run(0, n)
    else:
        from concurrent.futures import ThreadPoolExecutor
        cuts = np.linspace(0, n, nw + 1).astype(int)
        with ThreadPoolExecutor(nw) as ex:
            sts = list(ex.map(lambda i: run(cuts[i], cuts[i + 1]), range(nw)))
        st = min(sts) if min(sts) < 0 else max(sts)
    if st < 0:
        raise RuntimeError(f"oracle_rollout failed ({st})")
    # maxrows / maxcon: the busiest step's constraint rows / active contacts
    # nneg: the integer #{c < 0} count inside cost_c (SBP/mjx_planner.py:296)
    out = dict(cost4=cost4, theta=theta, status=st, maxrows=info[:, 0], maxcon=info[:, 1], nneg=info[:, 2])
    if want_slots:
        out["slots"] = slots[:, :, :model.nslot]
    if want_eef:
        out["eef"] = eef
    return out


class Runner:
    """Cost-only rollouts on a fixed thread pool over one prepared model
    struct -- what bench.py's cpu_baseline times: the pool is started and the
    model converted before the clock, each call is only the C rollouts
    (ctypes drops the GIL, so the threads run the C code concurrently).

    exact_mask: the EXACT_* rules of mpcr_oracle.c for these rollouts (None =
    the library default, MuJoCo's stop tests).  bench.py's fp32 baseline uses
    EXACT_MPR only, i.e. the kernel's own rules (ccd_tolerance 1e-6 and the
    fp32 Newton / line-search floors): fp32 without the floors iterates on
    rounding noise, which would inflate the GPU/CPU ratio.  Set on
    the library while the Runner lives (process-global: one Runner at a time)."""

    def __init__(self, model, workers, q0, w, ptgt, qtgt, precision="fp64", exact_mask=None):
        from concurrent.futures import ThreadPoolExecutor
        self.model, self.workers = model, max(1, int(workers))
        self.dt = np.float32 if precision == "fp32" else np.float64
        self.s = struct_f32(model) if precision == "fp32" else model.to_struct()
        self.L = lib_f32() if precision == "fp32" else lib()
        ct = ctypes.c_float if precision == "fp32" else ctypes.c_double
        self.p = lambda a: None if a is None else a.ctypes.data_as(ctypes.POINTER(ct))  # noqa: E731
        self.args = [np.ascontiguousarray(x, dtype=self.dt) for x in (q0, w, ptgt, qtgt)]
        self.prev_exact = None
        if exact_mask is not None:
            self.prev_exact = self.L.oracle_get_exact()
            self.L.oracle_set_exact(int(exact_mask))
        self.ex = ThreadPoolExecutor(self.workers)
        list(self.ex.map(lambda i: i, range(self.workers)))  # start every thread now

    def rollout(self, td):
        td = np.ascontiguousarray(td, dtype=self.dt)
        n, H = td.shape[0], td.shape[1] // self.model.nctrl
        cost4 = np.zeros((n, 4), dtype=self.dt)
        # 8 chunks per thread: candidates differ in work (contacts, rows), so
        # one static chunk per thread would leave threads idle at the end
        cuts = np.linspace(0, n, min(8 * self.workers, n) + 1).astype(int)
        q0, w, pt, qt = self.args
        p = self.p

        def run(i):
            a, b = cuts[i], cuts[i + 1]
            return self.L.oracle_rollout(ctypes.byref(self.s), int(b - a), H, p(td[a:b]), p(q0), p(w), p(pt),
                                         p(qt), p(cost4[a:b]), None, None, None, None, 0.0, 0, 0)

        st = list(self.ex.map(run, range(len(cuts) - 1)))
        if min(st) < 0:
            raise RuntimeError(f"oracle_rollout failed ({min(st)})")
        return cost4

    def close(self):
        self.ex.shutdown()
        if self.prev_exact is not None:
            self.L.oracle_set_exact(self.prev_exact)
            self.prev_exact = None


def cone_eval(mu, fri, D, jar, jv, alpha):
    """The oracle's elliptic cone (one condim-3 contact): cost, force, Hessian
    at jar and the line function along jar + alpha jv."""
    c = ctypes.c_double(0)
    f, H, line = np.zeros(3), np.zeros(9), np.zeros(3)
    a = [np.ascontiguousarray(x, dtype=np.float64) for x in (fri, D, jar, jv)]
    lib().oracle_cone_eval(float(mu), *(_p(x) for x in a), float(alpha), ctypes.byref(c), _p(f), _p(H), _p(line))
    return c.value, f, H.reshape(3, 3), line


def step_debug(model, qpos, qvel, qacc_ws, precision="fp64"):
    """The step's active contacts / rows / qacc_smooth / qacc in the kernel's
    debug layout (engine.parse_step_debug).  precision="fp32": the fp32 build
    (probe F of tests/parity_util.py) on the state rounded to fp32."""
    from manipulator_mujoco_amd.engine import parse_step_debug
    if precision == "fp32":
        fp = ctypes.POINTER(ctypes.c_float)
        a = [np.ascontiguousarray(x, dtype=np.float32) for x in (qpos, qvel, qacc_ws)]
        out = np.zeros(1234, dtype=np.float32)  # rollout.h DBG_N
        lib_f32().oracle_step_debug(ctypes.byref(struct_f32(model)), *(x.ctypes.data_as(fp) for x in a),
                                    out.ctypes.data_as(fp))
        return parse_step_debug(out, model.nv)
    s = model.to_struct()
    out = np.zeros(1234)  # rollout.h DBG_N
    a = [np.ascontiguousarray(x, dtype=np.float64) for x in (qpos, qvel, qacc_ws)]
    lib().oracle_step_debug(ctypes.byref(s), *(_p(x) for x in a), _p(out))
    return parse_step_debug(out, model.nv)


def step(model, qpos, qvel, qacc_ws):
    """One mj_step restatement; returns a dict of the intermediate quantities."""
    s = model.to_struct()
    nv = model.nv
    qpos = np.array(qpos, dtype=np.float64)
    qvel = np.array(qvel, dtype=np.float64)
    qws = np.array(qacc_ws, dtype=np.float64)
    M = np.zeros((nv, nv))
    bias = np.zeros(nv)
    pas = np.zeros(nv)
    qacc = np.zeros(nv)
    eef = np.zeros(7)
    dist = np.zeros(max(model.ncon, 1))
    nefc = ctypes.c_int(0)
    st = lib().oracle_step(ctypes.byref(s), _p(qpos), _p(qvel), _p(qws), _p(M), _p(bias), _p(pas), _p(qacc),
                           _p(eef), _p(dist), ctypes.byref(nefc))
    return dict(qpos=qpos, qvel=qvel, qacc_warmstart=qws, M=M, qfrc_bias=bias, qfrc_passive=pas, qacc=qacc,
                eef=eef, dist=dist[:model.ncon], nefc=nefc.value, status=st)

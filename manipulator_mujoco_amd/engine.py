"""Python handle on a libmpcr engine (one compiled model on one GPU).

``Engine.rollout_cost`` is the fused hot path: Bernstein basis -> H physics
steps -> cost, one wavefront per candidate.
Accepts either torch device tensors (zero-copy, launched on the current
torch stream) or host numpy arrays (staged through the engine's buffers).
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import MPCR_F_DEVICE_PTRS, MPCR_F_RESET_BEST, MPCR_LAYOUT_THETADOT, MPCR_LAYOUT_XI, check


def _f32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class Model:
    """Host model handle (``mpcr_model``) built from a compiled model."""

    def __init__(self, compiled):
        lib = _lib.load()
        self.compiled = compiled
        blob = compiled.to_blob()
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        h = ctypes.c_void_p()
        check(lib.mpcr_model_from_blob(self._blob, len(blob), ctypes.byref(h)))
        self.handle = h

    def hull_starts(self, R: int = 0, exact: bool = False):
        """The support start table engines build for this model
        (mpcr_model_hull_starts; R = 0: the library's MPCR_LUT_R): per-geom
        first cell (-1: no hull), the global hull vertex of every cell and,
        with exact, the cells whose climb the engine skips."""
        lib = _lib.load()
        adr = np.empty(max(1, self.compiled.ngeom), dtype=np.int32)
        i32p, u8p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint8)
        n = lib.mpcr_model_hull_starts(self.handle, R, adr.ctypes.data_as(i32p), None, None, 0)
        check(int(min(n, 0)))
        cells = np.empty(max(1, n), dtype=np.int32)
        ex = np.empty(max(1, n), dtype=np.uint8)
        check(int(min(lib.mpcr_model_hull_starts(self.handle, R, None, cells.ctypes.data_as(i32p),
                                                 ex.ctypes.data_as(u8p) if exact else None, n), 0)))
        out = (adr[:self.compiled.ngeom], cells[:n])
        return out + (ex[:n].astype(bool),) if exact else out

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.load().mpcr_model_free(self.handle)
        except Exception:  # interpreter shutdown
            pass
        self.handle = None


class Engine:
    def __init__(self, compiled_model, num_steps: int, max_n: int, pdot: np.ndarray, device: int = 0):
        lib = _lib.load()
        self.model = Model(compiled_model)
        self.H = int(num_steps)
        self.max_n = int(max_n)
        self.nctrl = int(compiled_model.nctrl)
        self.nslot = int(compiled_model.nslot)
        pdot = np.ascontiguousarray(pdot, dtype=np.float32)
        if pdot.shape[0] != self.H:
            raise ValueError(f"pdot has {pdot.shape[0]} rows, expected num_steps={self.H}")
        self.nbasis = pdot.shape[1]
        self.device = int(device)
        h = ctypes.c_void_p()
        check(lib.mpcr_engine_create(self.model.handle, self.device, self.max_n, self.H, pdot.ctypes.data,
                                     self.nbasis, ctypes.byref(h)))
        self.handle = h

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.load().mpcr_engine_free(self.handle)
        except Exception:  # interpreter shutdown
            pass
        self.handle = None

    def dispatches(self, n: int) -> int:
        """Kernel dispatches one rollout_cost over n candidates issues
        (mpcr_engine_dispatches: horizon segments x candidate groups for large
        dual-arm batches, else 1) -- per-dispatch profiler counters times this
        are per call."""
        out = ctypes.c_int()
        check(_lib.load().mpcr_engine_dispatches(self.handle, int(n), ctypes.byref(out)))
        return int(out.value)

    @staticmethod
    def _vec(x, n, dtype):
        a = np.zeros(n, dtype=dtype)
        x = np.asarray(x, dtype=dtype).reshape(-1)
        a[: x.size] = x
        return a

    def rollout_cost(self, inp, layout: int, q0, w, ptgt, qtgt, cost4=None, theta=None, thetadot=None,
                     best_key=None, index_base: int = 0, status=None, reset_best: bool = True, stream=None):
        """Run the fused rollout.

        torch path: ``inp``/outputs are CUDA tensors (float32, contiguous);
        ``best_key`` an int64 tensor of one element.  numpy path: host arrays.
        Returns cost4 (and fills the optional outputs in place).
        """
        lib = _lib.load()
        q0 = self._vec(q0, 8, np.float64)
        w = self._vec(w, 3, np.float32)
        pt = self._vec(ptgt, 3, np.float32)
        qt = self._vec(qtgt, 4, np.float32)
        dp = ctypes.POINTER(ctypes.c_double)
        try:
            import torch
            is_torch = isinstance(inp, torch.Tensor)
        except ImportError:  # pragma: no cover
            is_torch = False
        n = int(inp.shape[0])
        if is_torch:
            import torch
            if not inp.is_cuda or inp.dtype != torch.float32 or not inp.is_contiguous():
                raise ValueError("input must be a contiguous float32 CUDA tensor")
            if cost4 is None:
                cost4 = torch.empty((n, 4), dtype=torch.float32, device=inp.device)
            ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
            st = stream if stream is not None else torch.cuda.current_stream(inp.device).cuda_stream
            flags = MPCR_F_DEVICE_PTRS | (MPCR_F_RESET_BEST if reset_best else 0)
            check(lib.mpcr_rollout_cost(self.handle, ptr(inp), layout, n, q0.ctypes.data_as(dp), _f32p(w),
                                        _f32p(pt), _f32p(qt), ptr(cost4), ptr(theta), ptr(thetadot),
                                        ptr(best_key), int(index_base), ptr(status), flags, ctypes.c_void_p(st)))
            return cost4
        inp = np.ascontiguousarray(inp, dtype=np.float32)
        if cost4 is None:
            cost4 = np.zeros((n, 4), dtype=np.float32)
        key = np.zeros(1, dtype=np.uint64) if best_key is not None else None
        hp = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None  # noqa: E731
        check(lib.mpcr_rollout_cost(self.handle, hp(inp), layout, n, q0.ctypes.data_as(dp), _f32p(w), _f32p(pt),
                                    _f32p(qt), hp(cost4), hp(theta), hp(thetadot), hp(key), int(index_base),
                                    hp(status), 0, None))
        if best_key is not None:
            best_key[...] = key
        return cost4

    @staticmethod
    def params(q0, w, ptgt, qtgt):
        """The 20-float parameter block ``mpcr_rollout_cost_dp`` reads on the
        device: init_pos[8] | w[3], 0 | ptgt[3], 0 | qtgt[4]."""
        p = np.zeros(20, dtype=np.float32)
        q0 = np.asarray(q0, dtype=np.float64).reshape(-1)
        p[: q0.size] = q0
        p[8:11] = np.asarray(w, dtype=np.float32).reshape(-1)[:3]
        p[12:15] = np.asarray(ptgt, dtype=np.float32).reshape(-1)[:3]
        p[16:20] = np.asarray(qtgt, dtype=np.float32).reshape(-1)[:4]
        return p

    def rollout_cost_dp(self, inp, layout: int, params, cost4, theta=None, thetadot=None, best_key=None,
                        index_base: int = 0, status=None, reset_best: bool = True, stream=None):
        """``rollout_cost`` with the per-call arguments in a device tensor
        (``params``, 20 float32, see ``Engine.params``): graph-capturable."""
        import torch
        for name, t in (("input", inp), ("params", params), ("cost4", cost4)):
            if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous float32 CUDA tensor")
        if params.numel() < 20:
            raise ValueError("params needs 20 floats")
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        st = stream if stream is not None else torch.cuda.current_stream(inp.device).cuda_stream
        flags = MPCR_F_DEVICE_PTRS | (MPCR_F_RESET_BEST if reset_best else 0)
        check(_lib.load().mpcr_rollout_cost_dp(self.handle, ptr(inp), layout, int(inp.shape[0]), ptr(params),
                                               ptr(cost4), ptr(theta), ptr(thetadot), ptr(best_key),
                                               int(index_base), ptr(status), flags, ctypes.c_void_p(st)))
        return cost4

    def trace(self, inp, layout: int, q0, w, ptgt, qtgt):
        """Debug/parity run (host arrays): cost4, theta, per-step eef pose, masked slot distances."""
        lib = _lib.load()
        inp = np.ascontiguousarray(inp, dtype=np.float32)
        n = inp.shape[0]
        q0 = self._vec(q0, 8, np.float64)
        w = self._vec(w, 3, np.float32)
        pt = self._vec(ptgt, 3, np.float32)
        qt = self._vec(qtgt, 4, np.float32)
        cost4 = np.zeros((n, 4), dtype=np.float32)
        theta = np.zeros((n, self.nctrl * self.H), dtype=np.float32)
        eef = np.zeros((n, self.H, 7), dtype=np.float32)
        slots = np.zeros((n, self.H, max(self.nslot, 1)), dtype=np.float32)
        check(lib.mpcr_rollout_trace(self.handle, inp.ctypes.data_as(ctypes.c_void_p), layout, n,
                                     q0.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), _f32p(w), _f32p(pt),
                                     _f32p(qt), cost4.ctypes.data_as(ctypes.c_void_p),
                                     theta.ctypes.data_as(ctypes.c_void_p), eef.ctypes.data_as(ctypes.c_void_p),
                                     slots.ctypes.data_as(ctypes.c_void_p)))
        return dict(cost4=cost4, theta=theta, eef=eef, slots=slots[:, :, : self.nslot])


class Plant:
    """One environment of a compiled model stepped on the GPU by the rollout
    kernel (``mpcr_plant_*``): the closed-loop plant of
    ``run_cem_planner`` (CPU ``MjData`` + ``mj_step`` in the reference,
    SBP/mpc_planner.py:109-114,179-180).  State is fp32 on the device."""

    def __init__(self, compiled_model, device: int = 0):
        lib = _lib.load()
        self.model = Model(compiled_model)
        self.nq, self.nv = int(compiled_model.nq), int(compiled_model.nv)
        self.nctrl = int(compiled_model.nctrl)
        h = ctypes.c_void_p()
        check(lib.mpcr_plant_create(self.model.handle, int(device), ctypes.byref(h)))
        self.handle = h
        self.qpos = np.zeros(self.nq)
        self.qvel = np.zeros(self.nv)
        self.qacc = np.zeros(self.nv)
        self.eef = np.zeros(7)
        self._pull()

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.load().mpcr_plant_free(self.handle)
        except Exception:  # interpreter shutdown
            pass
        self.handle = None

    def _pull(self):
        dp = ctypes.POINTER(ctypes.c_double)
        check(_lib.load().mpcr_plant_get_state(self.handle, self.qpos.ctypes.data_as(dp),
                                               self.qvel.ctypes.data_as(dp), self.qacc.ctypes.data_as(dp),
                                               self.eef.ctypes.data_as(dp)))

    def set_state(self, qpos=None, qvel=None, qacc_warmstart=None):
        dp = ctypes.POINTER(ctypes.c_double)
        arr = lambda x, n: None if x is None else np.ascontiguousarray(x, dtype=np.float64).reshape(n)  # noqa: E731
        qp, qv, qw = arr(qpos, self.nq), arr(qvel, self.nv), arr(qacc_warmstart, self.nv)
        check(_lib.load().mpcr_plant_set_state(self.handle, None if qp is None else qp.ctypes.data_as(dp),
                                               None if qv is None else qv.ctypes.data_as(dp),
                                               None if qw is None else qw.ctypes.data_as(dp)))
        self._pull()

    def forward(self):
        """mj_forward: qacc and the eef pose at the current state."""
        check(_lib.load().mpcr_plant_step(self.handle, None, 0, None))
        self._pull()

    def step(self, qvel_ctrl=None):
        """qvel[:nctrl] = qvel_ctrl; mj_step.  Afterwards ``eef`` holds the tcp
        position / hande quaternion of the state the step started from (as
        MjData.site_xpos / xquat after mj_step)."""
        dp = ctypes.POINTER(ctypes.c_double)
        v = None
        if qvel_ctrl is not None:
            v = np.ascontiguousarray(qvel_ctrl, dtype=np.float64).reshape(self.nctrl)
        check(_lib.load().mpcr_plant_step(self.handle, None if v is None else v.ctypes.data_as(dp), 1, None))
        self._pull()

    def step_debug(self, qvel_ctrl, mpr_pair=-1):
        """step() that also returns the step's active contacts, constraint-row
        parameters, qacc_smooth and qacc (``parse_step_debug``; parity
        debugging, mpcr_plant_step_debug)."""
        lib = _lib.load()
        buf = np.zeros(lib.mpcr_plant_dbg_size(), dtype=np.float32)
        v = np.ascontiguousarray(qvel_ctrl, dtype=np.float64).reshape(self.nctrl)
        check(lib.mpcr_plant_step_debug(self.handle, v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                        buf.ctypes.data_as(ctypes.c_void_p), int(mpr_pair)))
        self._pull()
        return parse_step_debug(buf, self.nv)

    @property
    def site_xpos_tcp(self):
        return self.eef[:3].copy()

    @property
    def xquat_hande(self):
        return self.eef[3:7].copy()


__all__ = ["Engine", "Model", "Plant", "MPCR_LAYOUT_XI", "MPCR_LAYOUT_THETADOT"]


DBG_CON, DBG_MAXCON, DBG_MAXROW, DBG_NV = 2, 48, 200, 32  # rollout.h DBG_* layout


def parse_step_debug(buf, nv):
    """DBG_* buffer (kernel or oracle_step_debug) -> dict of numpy arrays."""
    buf = np.asarray(buf, dtype=np.float64)
    ncon, nefc = int(buf[0]), int(buf[1])
    con = buf[DBG_CON:DBG_CON + 8 * DBG_MAXCON].reshape(DBG_MAXCON, 8)[:min(ncon, DBG_MAXCON)]
    r0 = DBG_CON + 8 * DBG_MAXCON
    rows = buf[r0:r0 + 3 * DBG_MAXROW].reshape(DBG_MAXROW, 3)[:min(nefc, DBG_MAXROW)]
    q0 = r0 + 3 * DBG_MAXROW
    return dict(ncon=ncon, nefc=nefc, con_pos=con[:, 0:3], con_dist=con[:, 3], con_pair=con[:, 4].astype(int),
                con_normal=con[:, 5:8], efc_D=rows[:, 0], efc_aref=rows[:, 1], efc_vel=rows[:, 2],
                qacc_smooth=buf[q0:q0 + nv], qacc=buf[q0 + DBG_NV:q0 + DBG_NV + nv],
                info=buf[q0 + 2 * DBG_NV:q0 + 2 * DBG_NV + 8],
                grad=buf[q0 + 2 * DBG_NV + 8:q0 + 2 * DBG_NV + 8 + nv],
                search=buf[q0 + 3 * DBG_NV + 8:q0 + 3 * DBG_NV + 8 + nv],
                mpr=buf[q0 + 4 * DBG_NV + 8:q0 + 4 * DBG_NV + 8 + 112])

"""Device-resident CEM distribution step (libmpcr ``mpcr_cem_*`` / ``mpcr_topk``).

Wraps the HIP kernels of ``csrc/cem.hip`` for torch CUDA tensors, launched on
the current torch stream (so a whole CEM iteration can be captured in a
graph).  Reference functions (SBP/mjx_planner.py):

  ``factor`` + ``sample_project``  compute_xi_samples (:312-316) fused with
                                   compute_projection_filter (:180-249)
  ``project``                      compute_projection_filter alone
  ``topk``                         compute_ellite_samples' argsort (:305-310)
  ``update``                       compute_mean_cov / comp_prod (:318-335)

Every call requires a gfx950 device and the built library; there is no
torch or CPU fallback.
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import MPCR_F_DEVICE_PTRS, check

NBASIS = 11


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _dev(t, dtype, name):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != dtype or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous {dtype} CUDA tensor")
    return t


class CemContext:
    """Projection tables (basis rows, KKT inverse) + the Cholesky factor for
    one (num_dof, horizon) planner on one device."""

    def __init__(self, P, Pdot, Pddot, num_dof: int, max_n: int, device: int = 0, qinv=None):
        lib = _lib.load()
        P, Pdot, Pddot = (np.ascontiguousarray(x, dtype=np.float64) for x in (P, Pdot, Pddot))
        if P.shape[1] != NBASIS:
            raise ValueError(f"the CEM kernels are built for an order-10 basis ({NBASIS} columns)")
        self.num_dof = int(num_dof)
        self.H = int(P.shape[0])
        self.nvar = self.num_dof * NBASIS
        self.max_n = int(max_n)
        self.device = int(device)
        q = None
        if qinv is not None:
            q = np.ascontiguousarray(qinv, dtype=np.float64)
            ne = self.nvar + 5 * self.num_dof
            if q.shape != (ne, ne):
                raise ValueError(f"qinv must be {ne}x{ne}")
        h = ctypes.c_void_p()
        check(lib.mpcr_cem_create(self.device, self.num_dof, self.H, NBASIS, P.ctypes.data, Pdot.ctypes.data,
                                  Pddot.ctypes.data, q.ctypes.data if q is not None else None, self.max_n,
                                  ctypes.byref(h)))
        self.handle = h

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.load().mpcr_cem_free(self.handle)
        except Exception:  # interpreter shutdown
            pass
        self.handle = None

    @staticmethod
    def _stream(t, stream):
        import torch
        return ctypes.c_void_p(stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream)

    def factor(self, cov, reg: float = 0.003, stream=None):
        """L = chol(cov + reg I) for the next ``sample_project``."""
        import torch
        _dev(cov, torch.float32, "cov")
        check(_lib.load().mpcr_cem_factor(self.handle, _ptr(cov), float(reg), MPCR_F_DEVICE_PTRS,
                                          self._stream(cov, stream)))

    def sample_project(self, n, mean, seed, counter, b_eq, maxiter, bounds, rho=1.0, xi_samples=None, out=None,
                       xi_in=None, beq_shared=True, index_base=0, stream=None):
        """xi_samples = mean + z L^T (Philox (seed, counter), candidate i drawn
        as global candidate ``index_base + i``); or ``xi_in`` when mean is
        None; then ``maxiter`` ADMM iterations.  Returns the projected
        (n, nvar) tensor."""
        import torch
        ref = mean if mean is not None else xi_in
        if ref is None:
            raise ValueError("need mean or xi_in")
        f32 = dict(dtype=torch.float32, device=ref.device)
        if out is None:
            out = torch.empty((n, self.nvar), **f32)
        for name, t in (("mean", mean), ("xi_in", xi_in), ("xi_samples", xi_samples), ("out", out),
                        ("b_eq", b_eq)):
            if t is not None:
                _dev(t, torch.float32, name)
        bnd = (ctypes.c_float * 3)(*[float(b) for b in bounds])
        stride = 0 if beq_shared else 5 * self.num_dof
        check(_lib.load().mpcr_cem_sample_project(
            self.handle, int(n), _ptr(mean), ctypes.c_uint64(int(seed) & (2**64 - 1)),
            ctypes.c_uint64(int(counter) & (2**64 - 1)), int(index_base), _ptr(xi_in), _ptr(xi_samples), _ptr(b_eq), stride,
            int(maxiter), bnd, float(rho), _ptr(out), MPCR_F_DEVICE_PTRS, self._stream(ref, stream)))
        return out

    def project(self, xi, b_eq, maxiter, bounds, rho=1.0, out=None, beq_shared=True, stream=None):
        return self.sample_project(xi.shape[0], None, 0, 0, b_eq, maxiter, bounds, rho, out=out, xi_in=xi,
                                   beq_shared=beq_shared, stream=stream)

    def update(self, xi, cost, stride, elite_idx, lamda, alpha_mean, alpha_cov, mean, cov, reg=1e-4, stream=None):
        """In-place weighted elite mean/cov update (compute_mean_cov)."""
        import torch
        _dev(xi, torch.float32, "xi"); _dev(cost, torch.float32, "cost")
        _dev(elite_idx, torch.int32, "elite_idx"); _dev(mean, torch.float32, "mean"); _dev(cov, torch.float32, "cov")
        check(_lib.load().mpcr_cem_update(self.handle, _ptr(xi), int(xi.shape[0]), _ptr(cost), int(stride),
                                          _ptr(elite_idx), int(elite_idx.shape[0]), float(lamda), float(alpha_mean),
                                          float(alpha_cov), float(reg), _ptr(mean), _ptr(cov), MPCR_F_DEVICE_PTRS,
                                          self._stream(xi, stream)))


def topk(engine, cost, k, stride=1, out=None, stream=None):
    """Indices of the k smallest of cost[i*stride] in stable-argsort order
    (NaN last) through ``mpcr_topk`` on ``engine``'s device."""
    import torch
    _dev(cost, torch.float32, "cost")
    n = cost.numel() // stride
    if out is None:
        out = torch.empty(k, dtype=torch.int32, device=cost.device)
    st = stream if stream is not None else torch.cuda.current_stream(cost.device).cuda_stream
    check(_lib.load().mpcr_topk(engine.handle, _ptr(cost), int(stride), int(n), int(k), _ptr(out),
                                MPCR_F_DEVICE_PTRS, ctypes.c_void_p(st)))
    return out


__all__ = ["CemContext", "topk", "NBASIS"]

"""Multi-GPU exchanges: one process per GPU, candidates sharded by rank.

Rollouts need one exchange, the global best candidate
(``idx_min = argmin(cost_batch[-1])``, SBP/mjx_planner.py:395).  Each rank's
rollout kernel atomically min-reduces a packed 64-bit key
``ordered(cost) << 32 | global_index`` (NaN first, ties to the lowest index:
jnp.argmin semantics); ranks then all-reduce that single int64 with MIN —
one 8-byte RCCL collective over xGMI (``nccl`` backend) or gloo on CPU.

A sharded CEM iteration adds the elite exchange
(``gather_elites``): every global elite is among its rank's local top-E, so
ranks all-gather their local top-E rows (cost + xi) and every rank selects
the same global top-E from the gathered block.  Gathered positions are
rank-major and each rank's rows are in (cost, index) order, so ties broken
by position are ties broken by global index: the selection equals the
single-GPU ``argsort(kind="stable")[:E]`` in order and the replicated
mean/cov update is bit-identical to the single-GPU one.
"""

from __future__ import annotations

import os

import numpy as np

SIGN = -(1 << 63)


def ordered_key(cost: float, index: int) -> int:
    """Host restatement of the kernel's key (for tests and CPU ranks)."""
    u = int(np.float32(cost).view(np.uint32))
    if np.isnan(np.float32(cost)):
        k = 0
    elif u & 0x80000000:
        k = (~u) & 0xFFFFFFFF
    else:
        k = u | 0x80000000
    return (k << 32) | (index & 0xFFFFFFFF)


def decode_key(key: int):
    key &= 0xFFFFFFFFFFFFFFFF
    hi, idx = key >> 32, key & 0xFFFFFFFF
    if hi == 0:
        return idx, float("nan")
    u = (hi & 0x7FFFFFFF) if hi & 0x80000000 else (~hi) & 0xFFFFFFFF
    return idx, float(np.uint32(u).view(np.float32))


def _host_staged(group):
    """gloo moves CPU tensors (used by the CPU tests and for ranks sharing one
    GPU); RCCL moves device tensors."""
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo"


def allreduce_min_key(key_tensor, group=None):
    """In-place global MIN of a 1-element int64 tensor holding an unsigned
    packed key (sign bit flipped around the signed reduction)."""
    import torch.distributed as dist

    t = key_tensor.cpu() if _host_staged(group) and key_tensor.is_cuda else key_tensor
    t ^= SIGN
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    t ^= SIGN
    if t is not key_tensor:
        key_tensor.copy_(t)
    return key_tensor


def all_gather(x, group=None):
    """(world, *x.shape) all-gather of a contiguous tensor, on x's device."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    src = x.contiguous()
    if _host_staged(group) and src.is_cuda:
        src = src.cpu()
    shape = tuple(src.shape)
    out = torch.empty((world * shape[0],) + shape[1:], dtype=src.dtype, device=src.device)  # dim-0 concat
    dist.all_gather_into_tensor(out, src, group=group)
    return out.view((world,) + shape).to(x.device)


def broadcast(x, src, group=None):
    """In-place broadcast from group rank src."""
    import torch.distributed as dist

    g_src = dist.get_global_rank(group, src) if group is not None and group is not dist.group.WORLD else src
    t = x.cpu() if _host_staged(group) and x.is_cuda else x
    dist.broadcast(t, src=g_src, group=group)
    if t is not x:
        x.copy_(t)
    return x


def shard(n_total: int, rank: int, world: int):
    """Contiguous candidate shard [lo, hi) of rank."""
    per = (n_total + world - 1) // world
    lo = min(rank * per, n_total)
    return lo, min(lo + per, n_total)


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def gather_elites(cost, xi, k, topk_fn, group=None):
    """Global top-``k`` elites of a sharded batch.

    cost: local (n,) float32; xi: local (n, nv) rows the update reads;
    topk_fn(cost_1d, k) -> int indices of the k smallest in stable-argsort
    order, NaN last (``mpcr_topk`` on a GPU rank).  Every rank must hold the
    same n.  Returns (gathered cost (G*kl,), gathered rows (G*kl, nv),
    selected positions (k,)); gathered[sel] are the global elites in order.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n, nv = xi.shape
    kl = min(int(k), n)
    if kl * world < k:
        raise ValueError(f"k={k} elites need more than {world} x {n} candidates")
    lidx = topk_fn(cost, kl).long()
    pack = torch.empty((kl, nv + 1), dtype=xi.dtype, device=xi.device)
    pack[:, :nv] = xi.index_select(0, lidx)
    pack[:, nv] = cost.index_select(0, lidx)
    out = all_gather(pack, group).reshape(world * kl, nv + 1)
    g_cost = out[:, nv].contiguous()
    g_xi = out[:, :nv].contiguous()
    sel = topk_fn(g_cost, int(k))
    return g_cost, g_xi, sel


def allgather_min(values, group=None):
    """Elementwise NaN-propagating min over ranks (jnp.min semantics) of a
    small 1-D tensor; returned on the host as float32 numpy."""
    import torch
    import torch.distributed as dist

    a = all_gather(values, group).cpu().numpy()
    return np.where(np.isnan(a).any(axis=0), np.nan, np.nanmin(np.where(np.isnan(a), np.inf, a), axis=0)).astype(
        np.float32)


class RcclComm:
    """The C ABI's own RCCL communicator (``mpcr_comm_*``, include/mpcr.h):
    the same two exchanges as the torch.distributed functions above, for
    hosts that embed libmpcr.so without Python.  Device tensors only.

        uid = RcclComm.unique_id()            # rank 0, shared out of band
        comm = RcclComm(rank, nranks, uid, device)
    """

    ID_BYTES = 128

    @staticmethod
    def unique_id() -> bytes:
        import ctypes

        from . import _lib
        buf = ctypes.create_string_buffer(RcclComm.ID_BYTES)
        _lib.check(_lib.load().mpcr_comm_unique_id(buf))
        return buf.raw

    def __init__(self, rank: int, nranks: int, uid: bytes, device: int = 0):
        import ctypes

        from . import _lib
        if len(uid) != self.ID_BYTES:
            raise ValueError(f"unique id must be {self.ID_BYTES} bytes")
        self._lib = _lib.load()
        self.rank, self.nranks, self.device = rank, nranks, device
        h = ctypes.c_void_p()
        _lib.check(self._lib.mpcr_comm_init(rank, nranks, uid, device, ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            self._lib.mpcr_comm_free(self.handle)
            self.handle = None

    __del__ = close

    @staticmethod
    def _stream(t):
        import torch
        return ctypes_ptr(torch.cuda.current_stream(t.device).cuda_stream)

    def allreduce_min_key(self, key_tensor):
        """In-place global MIN of packed uint64 keys held in an int64 device tensor."""
        from . import _lib
        _lib.check(self._lib.mpcr_comm_allreduce_key(self.handle, key_tensor.data_ptr(), key_tensor.numel(),
                                                     self._stream(key_tensor)))
        return key_tensor

    def all_gather(self, x):
        """(nranks, *x.shape) rank-major all-gather of a float32 device tensor."""
        import torch

        from . import _lib
        src = x.contiguous()
        out = torch.empty((self.nranks,) + tuple(src.shape), dtype=torch.float32, device=src.device)
        _lib.check(self._lib.mpcr_comm_allgather(self.handle, src.data_ptr(), out.data_ptr(), src.numel(),
                                                 self._stream(src)))
        return out

    def gather_elites(self, cost, xi, k):
        """gather_elites above through mpcr_comm_gather_elites: returns
        (gathered cost, gathered rows, selected positions)."""
        import torch

        from . import _lib
        n, nv = xi.shape
        kl = min(int(k), n)
        rows = torch.empty((self.nranks * kl, nv + 1), dtype=torch.float32, device=xi.device)
        sel = torch.empty(int(k), dtype=torch.int32, device=xi.device)
        c, x = cost.contiguous(), xi.contiguous()
        _lib.check(self._lib.mpcr_comm_gather_elites(self.handle, c.data_ptr(), x.data_ptr(), n, nv, int(k),
                                                     rows.data_ptr(), sel.data_ptr(), self._stream(x)))
        return rows[:, nv].contiguous(), rows[:, :nv].contiguous(), sel


def ctypes_ptr(v: int):
    import ctypes
    return ctypes.c_void_p(v) if v else None

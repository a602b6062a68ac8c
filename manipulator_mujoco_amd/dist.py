"""Multi-GPU selection: one process per GPU, candidates sharded by rank.

The only exchange the rollout path needs is the global best candidate
(``idx_min = argmin(cost_batch[-1])``, SBP/mjx_planner.py:395).  Each rank's
rollout kernel atomically min-reduces a packed 64-bit key
``ordered(cost) << 32 | global_index`` (NaN first, ties to the lowest index:
jnp.argmin semantics); ranks then all-reduce that single int64 with MIN —
one 8-byte RCCL collective over xGMI (``nccl`` backend) or gloo on CPU.
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


def allreduce_min_key(key_tensor, group=None):
    """In-place global MIN of a 1-element int64 tensor holding an unsigned
    packed key (sign bit flipped around the signed reduction)."""
    import torch.distributed as dist

    key_tensor ^= SIGN
    dist.all_reduce(key_tensor, op=dist.ReduceOp.MIN, group=group)
    key_tensor ^= SIGN
    return key_tensor


def shard(n_total: int, rank: int, world: int):
    """Contiguous candidate shard [lo, hi) of rank."""
    per = (n_total + world - 1) // world
    lo = min(rank * per, n_total)
    return lo, min(lo + per, n_total)


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))

"""Multi-rank selection with gloo, world_size 2: each rank owns a
shard of candidates and contributes its packed best key; one MIN all-reduce
yields the global argmin with jnp.argmin semantics (NaN first, lowest index)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, costs, out):
    import torch
    import torch.distributed as dist

    from manipulator_mujoco_amd import dist as md

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = md.shard(len(costs), rank, world)
    local = min(md.ordered_key(c, lo + i) for i, c in enumerate(costs[lo:hi]))
    key = torch.tensor([local - (1 << 64) if local >= (1 << 63) else local], dtype=torch.int64)
    md.allreduce_min_key(key)
    out[rank] = int(key.item()) & 0xFFFFFFFFFFFFFFFF
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["plain", "nan", "ties"])
def test_global_best_two_ranks(case):
    rng = np.random.default_rng(1)
    costs = rng.uniform(1, 100, 101).astype(np.float32)
    if case == "nan":
        costs[70] = np.nan
        costs[90] = np.nan
    if case == "ties":
        costs[60] = costs[80] = costs.min() - 1
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, list(costs), out), nprocs=2, join=True)
    from manipulator_mujoco_amd import dist as md
    expect = int(np.argmin(costs))  # numpy: first NaN, else first minimum
    for r in range(2):
        idx, val = md.decode_key(out[r])
        assert idx == expect

"""The C ABI's RCCL exchange (mpcr_comm_*, csrc/comm.hip) on one MI355X: a
one-rank communicator exercises every path of the key all-reduce, the
all-gather and the sharded elite selection (pack -> all-gather -> top-k over
the gathered block).  Two ranks cannot share one GPU in an RCCL communicator,
so the multi-rank selection rule itself is covered by the gloo tests of
tests/test_distributed.py (same rule, manipulator_mujoco_amd/dist.py).

Bars: integer / index work bit-exact; gathered rows bit-identical copies."""
import numpy as np
import pytest

from manipulator_mujoco_amd import dist as md

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = md.RcclComm(0, 1, md.RcclComm.unique_id(), 0)
    yield c
    c.close()


def test_allreduce_key_is_identity_on_one_rank(comm):
    import torch
    keys = [md.ordered_key(3.5, 7), md.ordered_key(float("nan"), 9), md.ordered_key(-1.0, 2)]
    t = torch.tensor(np.array(keys, dtype=np.uint64).view(np.int64), device="cuda")  # the unsigned keys' bits
    ref = t.clone()
    comm.allreduce_min_key(t)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)


def test_allgather_copies_rank_major(comm):
    import torch
    x = torch.randn(5, 3, device="cuda")
    g = comm.all_gather(x)
    torch.cuda.synchronize()
    assert g.shape == (1, 5, 3) and torch.equal(g[0], x)


@pytest.mark.parametrize("n,k", [(4096, 204), (1000, 1000), (300, 17)])
def test_gather_elites_matches_single_gpu_selection(comm, n, k):
    import torch
    rng = np.random.default_rng(n + k)
    cost = rng.normal(0, 1, n).astype(np.float32)
    cost[rng.integers(0, n, 8)] = np.nan           # NaN sorts last
    cost[rng.integers(0, n, 40)] = cost[3]          # ties break by index
    xi = rng.normal(0, 1, (n, 66)).astype(np.float32)
    c_d, x_d = torch.tensor(cost, device="cuda"), torch.tensor(xi, device="cuda")
    g_cost, g_xi, sel = comm.gather_elites(c_d, x_d, k)
    torch.cuda.synchronize()
    ref = np.argsort(np.where(np.isnan(cost), np.inf, cost), kind="stable")[:k]
    got_rows = g_xi.cpu().numpy()[sel.cpu().numpy()]
    np.testing.assert_array_equal(got_rows, xi[ref])
    np.testing.assert_array_equal(g_cost.cpu().numpy()[sel.cpu().numpy()], cost[ref])

"""GPU parity of the CEM distribution step (csrc/cem.hip through the C ABI)
against the fp64 numpy oracle (oracle/cem_np.py, SBP/mjx_planner.py:180-335).

Tolerances (fp32 kernels vs fp64 oracle):
  projection    |gpu - oracle| <= 1e-4 + 1e-4 |oracle| per coefficient
  moments       mean within 1e-5 + 1e-5 |.|, cov within 1e-5 + 1e-4 |.|
  top-k         bit-exact indices (integer work)
"""
import numpy as np
import pytest

from manipulator_mujoco_amd import basis, models
from oracle import cem_np

pytestmark = pytest.mark.gpu

Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
BOUNDS = (0.8, 1.8, np.pi)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch


def _ctx(H, max_n, qinv=None):
    from manipulator_mujoco_amd.cem import CemContext
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    return CemContext(P, Pd, Pdd, 6, max_n, qinv=qinv), (P, Pd, Pdd)


def _oracle_mats(P, Pd, Pdd):
    f32 = np.float32
    A = cem_np.a_matrices(P.astype(f32), Pd.astype(f32), Pdd.astype(f32))
    return A, cem_np.q_inv(A)


def _state(n, rng, moving=False):
    st = np.zeros((n, 30))
    st[:, :6] = Q0
    if moving:
        st[:, 6:12] = rng.uniform(-0.5, 0.5, (n, 6))
        st[:, 12:18] = rng.uniform(-1.0, 1.0, (n, 6))
    return st


@pytest.mark.parametrize("H", [16, 50, 100])
def test_projection_parity(torch_cuda, H):
    torch = torch_cuda
    n = 512
    ctx, (P, Pd, Pdd) = _ctx(H, n)
    A, Qinv = _oracle_mats(P, Pd, Pdd)
    rng = np.random.default_rng(H)
    xi = rng.normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)
    st = _state(1, rng)
    ref = cem_np.projection_filter(xi.astype(np.float64), np.repeat(st, n, 0), A, Qinv, 10)
    beq = torch.tensor(cem_np.boundary_vec(st).astype(np.float32).reshape(-1), device="cuda")
    out = ctx.project(torch.tensor(xi, device="cuda"), beq, 10, BOUNDS).cpu().numpy()
    err = np.abs(out - ref)
    assert (err <= 1e-4 + 1e-4 * np.abs(ref)).all(), err.max()


def test_projection_per_candidate_beq(torch_cuda):
    """b_eq per candidate (beq_stride = 5 nd) with nonzero initial velocity/acceleration."""
    torch = torch_cuda
    n, H = 256, 50
    ctx, (P, Pd, Pdd) = _ctx(H, n)
    A, Qinv = _oracle_mats(P, Pd, Pdd)
    rng = np.random.default_rng(5)
    xi = rng.normal(0, 1.0, (n, 66)).astype(np.float32)
    st = _state(n, rng, moving=True)
    ref = cem_np.projection_filter(xi.astype(np.float64), st, A, Qinv, 10)
    beq = torch.tensor(cem_np.boundary_vec(st).astype(np.float32), device="cuda")
    out = ctx.project(torch.tensor(xi, device="cuda"), beq, 10, BOUNDS, beq_shared=False).cpu().numpy()
    err = np.abs(out - ref)
    assert (err <= 1e-4 + 1e-4 * np.abs(ref)).all(), err.max()


def test_projection_given_qinv_and_identity(torch_cuda):
    """An explicit KKT inverse gives the same result; maxiter = 0 returns the input bit-exactly."""
    torch = torch_cuda
    n, H = 128, 50
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    _, Qinv = _oracle_mats(P, Pd, Pdd)
    ctx_a, _ = _ctx(H, n)
    ctx_b, _ = _ctx(H, n, qinv=Qinv)
    rng = np.random.default_rng(9)
    xi = torch.tensor(rng.normal(0, 3, (n, 66)).astype(np.float32), device="cuda")
    beq = torch.tensor(cem_np.boundary_vec(_state(1, rng)).astype(np.float32).reshape(-1), device="cuda")
    a = ctx_a.project(xi, beq, 10, BOUNDS).cpu().numpy()
    b = ctx_b.project(xi, beq, 10, BOUNDS).cpu().numpy()
    # the two inverses differ only by the fp32 Gram blocks' summation order
    assert (np.abs(a - b) <= 1e-4 + 1e-4 * np.abs(b)).all(), np.abs(a - b).max()
    same = ctx_a.project(xi, beq, 0, BOUNDS)
    assert torch.equal(same, xi)


def test_projection_full_size_properties(torch_cuda):
    """C3 size (4096 x 66, H = 50): the KKT solve enforces the boundary
    equalities every iteration, and projecting twice from the same input is
    bitwise deterministic."""
    torch = torch_cuda
    n, H = 4096, 50
    ctx, (P, Pd, Pdd) = _ctx(H, n)
    A, _ = _oracle_mats(P, Pd, Pdd)
    rng = np.random.default_rng(3)
    xi = torch.tensor(rng.normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32), device="cuda")
    st = _state(1, rng)
    beq_np = cem_np.boundary_vec(st).reshape(-1)
    beq = torch.tensor(beq_np.astype(np.float32), device="cuda")
    out = ctx.project(xi, beq, 10, BOUNDS)
    out2 = ctx.project(xi, beq, 10, BOUNDS)
    assert torch.equal(out, out2)
    o = out.cpu().numpy().astype(np.float64)
    eq = o @ A["A_eq"].T
    assert np.abs(eq - beq_np).max() < 1e-3


def test_sampling_statistics_and_fusion(torch_cuda):
    """xi = mean + z L^T: empirical moments match (mean, cov + reg I); the fused
    sample+project equals projecting the returned samples; seeds are
    reproducible and counters decorrelate."""
    torch = torch_cuda
    n, H = 65536, 50
    ctx, (P, Pd, Pdd) = _ctx(H, n)
    rng = np.random.default_rng(1)
    B = rng.normal(0, 0.3, (66, 66))
    cov = (B @ B.T + np.eye(66)).astype(np.float32)
    mean = rng.normal(0, 1, 66).astype(np.float32)
    tc, tm = torch.tensor(cov, device="cuda"), torch.tensor(mean, device="cuda")
    ctx.factor(tc, 0.003)
    beq = torch.tensor(cem_np.boundary_vec(_state(1, rng)).astype(np.float32).reshape(-1), device="cuda")
    samples = torch.empty((n, 66), device="cuda")
    filt = ctx.sample_project(n, tm, seed=1234, counter=7, b_eq=beq, maxiter=10, bounds=BOUNDS, xi_samples=samples)
    s = samples.cpu().numpy().astype(np.float64)
    target = cov.astype(np.float64) + 0.003 * np.eye(66)
    sd = np.sqrt(np.diag(target))
    assert (np.abs(s.mean(0) - mean) < 5 * sd / np.sqrt(n)).all()
    emp = np.cov(s.T)
    corr_err = np.abs(emp - target) / np.outer(sd, sd)
    assert corr_err.max() < 6 / np.sqrt(n) * 2, corr_err.max()
    # fused == project(samples)
    again = ctx.project(samples, beq, 10, BOUNDS)
    assert torch.equal(filt, again)
    # reproducible, counter-dependent
    s2 = torch.empty_like(samples)
    ctx.sample_project(n, tm, seed=1234, counter=7, b_eq=beq, maxiter=0, bounds=BOUNDS, xi_samples=s2)
    assert torch.equal(samples, s2)
    ctx.sample_project(n, tm, seed=1234, counter=8, b_eq=beq, maxiter=0, bounds=BOUNDS, xi_samples=s2)
    assert not torch.equal(samples, s2)


def test_factor_matches_numpy_cholesky(torch_cuda):
    """Diagonal + low-rank covariance: samples reconstruct L through z = (xi - mean) L^-T
    being standard normal; checked via the factor's action on the identity draw."""
    torch = torch_cuda
    n = 8192
    ctx, _ = _ctx(50, n)
    rng = np.random.default_rng(2)
    B = rng.normal(0, 0.5, (66, 66))
    cov = (B @ B.T + 0.5 * np.eye(66)).astype(np.float32)
    L = np.linalg.cholesky(cov.astype(np.float64) + 0.003 * np.eye(66))
    ctx.factor(torch.tensor(cov, device="cuda"), 0.003)
    zero = torch.zeros(66, device="cuda")
    s = torch.empty((n, 66), device="cuda")
    ctx.sample_project(n, zero, seed=5, counter=0, b_eq=None, maxiter=0, bounds=BOUNDS, xi_samples=s)
    x = s.cpu().numpy().astype(np.float64)
    z = np.linalg.solve(L, x.T).T  # whitened with the fp64 factor
    assert np.abs(z.mean(0)).max() < 5 / np.sqrt(n)
    assert np.abs(np.cov(z.T) - np.eye(66)).max() < 8 / np.sqrt(n)


def _stable_argsort(c):
    return np.argsort(c, kind="stable")  # NaN last, -0 == +0, ties by index


@pytest.mark.parametrize("n,k", [(1, 1), (7, 3), (1000, 50), (4096, 204), (4096, 4096), (32768, 1638),
                                 (100000, 4096)])
def test_topk_matches_stable_argsort(torch_cuda, n, k):
    torch = torch_cuda
    from manipulator_mujoco_amd.cem import topk
    from manipulator_mujoco_amd.engine import Engine
    rng = np.random.default_rng(n + k)
    c = rng.normal(100, 30, n).astype(np.float32)
    c[rng.integers(0, n, n // 10 + 1)] = np.round(c[rng.integers(0, n, n // 10 + 1)])  # ties
    c[rng.integers(0, n, n // 50 + 1)] = np.nan
    c[rng.integers(0, n, n // 50 + 1)] = -0.0
    c[rng.integers(0, n, n // 50 + 1)] = 0.0
    c[rng.integers(0, n, n // 100 + 1)] = -np.inf
    m = models.load("ur5e_hande_mjx", 0.05)
    _, _, Pd, _ = basis.planner_basis(10, 0.05)
    e = Engine(m, 10, max(n, 1), Pd)
    got = topk(e, torch.tensor(c, device="cuda"), k).cpu().numpy()
    assert np.array_equal(got, _stable_argsort(c)[:k])
    # strided view of a (n, 4) cost4-like array
    c4 = np.zeros((n, 4), np.float32)
    c4[:, 0] = c
    got4 = topk(e, torch.tensor(c4, device="cuda"), k, stride=4).cpu().numpy()
    assert np.array_equal(got4, got)


def test_topk_all_equal_and_all_nan(torch_cuda):
    torch = torch_cuda
    from manipulator_mujoco_amd.cem import topk
    from manipulator_mujoco_amd.engine import Engine
    m = models.load("ur5e_hande_mjx", 0.05)
    _, _, Pd, _ = basis.planner_basis(10, 0.05)
    e = Engine(m, 10, 3000, Pd)
    for c in (np.full(3000, 7.0, np.float32), np.full(3000, np.nan, np.float32)):
        got = topk(e, torch.tensor(c, device="cuda"), 100).cpu().numpy()
        assert np.array_equal(got, np.arange(100))


@pytest.mark.parametrize("n,frac", [(1000, 0.05), (4096, 0.05), (32768, 0.05)])
def test_cem_update_matches_oracle(torch_cuda, n, frac):
    torch = torch_cuda
    from manipulator_mujoco_amd.cem import topk
    from manipulator_mujoco_amd.engine import Engine
    ctx, _ = _ctx(50, n)
    m = models.load("ur5e_hande_mjx", 0.05)
    _, _, Pd, _ = basis.planner_basis(10, 0.05)
    e = Engine(m, 10, n, Pd)
    rng = np.random.default_rng(n)
    xi = rng.normal(0, 3, (n, 66)).astype(np.float32)
    cost = rng.gamma(2.0, 50.0, n).astype(np.float32)
    mean = rng.normal(0, 1, 66).astype(np.float32)
    cov = (10 * np.eye(66)).astype(np.float32)
    k = int(frac * n)
    x_ref, idx_ref, c_ref = cem_np.ellite(cost.astype(np.float64), xi.astype(np.float64), frac)
    m_ref, cov_ref = cem_np.mean_cov(c_ref, mean.astype(np.float64), cov.astype(np.float64), x_ref)
    tx, tcost = torch.tensor(xi, device="cuda"), torch.tensor(cost, device="cuda")
    idx = topk(e, tcost, k)
    assert np.array_equal(idx.cpu().numpy(), idx_ref[:k])
    tm, tcov = torch.tensor(mean, device="cuda"), torch.tensor(cov, device="cuda")
    ctx.update(tx, tcost, 1, idx, 10.0, 0.6, 0.6, tm, tcov)
    gm, gc = tm.cpu().numpy(), tcov.cpu().numpy()
    assert (np.abs(gm - m_ref) <= 1e-5 + 1e-5 * np.abs(m_ref)).all(), np.abs(gm - m_ref).max()
    assert (np.abs(gc - cov_ref) <= 1e-5 + 1e-4 * np.abs(cov_ref)).all(), np.abs(gc - cov_ref).max()
    assert np.array_equal(gc, gc.T)


def test_cem_iteration_parity(torch_cuda):
    """One cem_iter of the drop-in planner, stage by stage, against the oracle on
    the planner's own samples: projection (1e-4), elite indices (exact, from the
    GPU costs), moments (fp32 tolerance)."""
    from manipulator_mujoco_amd.planner import cem_planner
    N, H = 256, 16
    p = cem_planner(num_dof=6, num_batch=N, num_steps=H, timestep=0.05, maxiter_cem=1, num_elite=0.05,
                    w_pos=20.0, w_rot=3.0, w_col=80.0, maxiter_projection=10, verbose=False)
    PT, QT = np.array([-0.3, -0.3, 0.5]), np.array([0.0, 1.0, 0.0, 0.0])
    mean0 = np.zeros(p.nvar)
    out = p.compute_cem(mean0, Q0, np.zeros(6), np.zeros(6), PT, QT)
    xs = p._xs.cpu().numpy().astype(np.float64)
    xf = p._xf.cpu().numpy().astype(np.float64)
    A, Qinv = _oracle_mats(p.P, p.Pdot, p.Pddot)
    st = np.zeros((N, 30))
    st[:, :6] = Q0
    ref_f = cem_np.projection_filter(xs, st, A, Qinv, 10)
    assert (np.abs(xf - ref_f) <= 1e-4 + 1e-4 * np.abs(ref_f)).all()
    # elites + moments from the GPU's own costs (thetadot/theta of iteration 0 are returned)
    td = out[7][0].astype(np.float64)  # thetadot N x 6H
    import oracle
    o = oracle.rollout(p.model, td, Q0, np.array([20.0, 3.0, 80.0]), PT, QT)
    cost = o["cost4"][:, 0]
    x_e, idx, c_e = cem_np.ellite(cost, xs, 0.05)
    m_ref, _ = cem_np.mean_cov(c_e, mean0, 10 * np.eye(p.nvar), x_e)
    assert np.abs(out[6] - m_ref).max() < 1e-3 * max(1.0, np.abs(m_ref).max())
    # the selected candidate's cost components best_cost_g / _r / _c
    # (SBP/mjx_planner.py:395-402) against the oracle's at the same index, to
    # 1e-4 or the candidate's own conditioning (8 fp32-sized probes)
    k = np.where((out[7][-1] == out[4].T.reshape(-1)).all(axis=1))[0]
    assert k.size >= 1
    i = int(k[0])
    W3 = np.array([20.0, 3.0, 80.0])
    ref = o["cost4"][i]
    sens = np.zeros(4)
    for sd in range(1, 9):
        b = oracle.rollout(p.model, td[i:i + 1], Q0, W3, PT, QT, want_theta=False, noise=1e-6, seed=sd)["cost4"][0]
        sens = np.maximum(sens, np.abs(b - ref) / np.maximum(np.abs(ref), 1e-12))
    got = np.array([out[0][-1], out[1], out[2], out[3]], dtype=np.float64)
    for c in range(4):
        if ref[c] == 0 and got[c] == 0:
            continue
        rel = abs(got[c] - ref[c]) / max(abs(ref[c]), 1e-12)
        assert rel < max(1e-4, 2 * sens[c]), (c, got, ref, sens)

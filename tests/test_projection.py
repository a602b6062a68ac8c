"""A12: the device projection filter (projection.py, here on CPU torch as host
logic) vs the numpy transliteration of compute_projection (SBP/mjx_planner.py:180-249)."""
import numpy as np
import torch

from manipulator_mujoco_amd import basis
from manipulator_mujoco_amd.projection import ProjectionFilter, kkt_inverse
from oracle import cem_np


def _setup(H):
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    return P, Pd, Pdd


def test_kkt_inverse_matches_transliteration():
    P, Pd, Pdd = _setup(16)
    A = cem_np.a_matrices(P, Pd, Pdd)
    np.testing.assert_allclose(kkt_inverse(P, Pd, Pdd), cem_np.q_inv(A), rtol=1e-10, atol=1e-6)


def test_projection_matches_and_enforces_bounds():
    H, n = 50, 64
    P, Pd, Pdd = _setup(H)
    A = cem_np.a_matrices(P, Pd, Pdd)
    Qi = cem_np.q_inv(A)
    rng = np.random.default_rng(20250629 + 3)
    xi = rng.normal(0, np.sqrt(10.003), (n, 66))
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    st = np.tile(np.concatenate([q0, np.zeros(24)]), (n, 1))
    ref = cem_np.projection_filter(xi, st, A, Qi, 10)
    f = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
    got = f(torch.tensor(xi, dtype=torch.float32), f.boundary(q0, np.zeros(6), np.zeros(6), n), 10).numpy()
    # fp32 vs fp64 on a KKT system with cond ~1e6: compare in the trajectory space
    v_ref = (A["A_thetadot"] @ ref.T).T
    v_got = (A["A_thetadot"] @ got.T).T
    assert np.abs(v_got - v_ref).max() < 2e-3 * max(1.0, np.abs(v_ref).max())
    # boundary: theta(0) = q0 and near-zero end velocity
    p0 = (A["A_theta"] @ got.T).T[:, ::H]
    np.testing.assert_allclose(p0, np.tile(q0, (n, 1)), atol=2e-3)
    assert np.abs(v_ref).max() < 1.2  # 10 ADMM iterations pull |thetadot| towards 0.8

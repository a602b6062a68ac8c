"""numpy transliterations of the reference planner's pure array algebra.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Each function follows the
cited lines of SBP/mjx_planner.py (sampling_based_planner/mjx_planner.py)
statement by statement, in fp64 unless ``dtype`` says otherwise.
"""

from __future__ import annotations

import numpy as np


def a_matrices(P, Pdot, Pddot, num_dof=6):
    """get_A_traj / get_A_p / get_A_v / get_A_a / get_A_eq (:140-164)."""
    I = np.identity(num_dof)
    A_theta = np.kron(I, P)
    A_thetadot = np.kron(I, Pdot)
    A_thetaddot = np.kron(I, Pddot)
    A_p_ineq = np.kron(I, np.vstack((P, -P)))
    A_v_ineq = np.kron(I, np.vstack((Pdot, -Pdot)))
    A_a_ineq = np.kron(I, np.vstack((Pddot, -Pddot)))
    A_eq = np.kron(I, np.vstack((P[0], Pdot[0], Pddot[0], Pdot[-1], Pddot[-1])))
    return dict(A_theta=A_theta, A_thetadot=A_thetadot, A_thetaddot=A_thetaddot, A_p_ineq=A_p_ineq,
                A_v_ineq=A_v_ineq, A_a_ineq=A_a_ineq, A_eq=A_eq)


def q_inv(A, rho_ineq=1.0, gram_dtype=np.float32):
    """get_Q_inv (:166-172): the Gram blocks are jnp.dot of fp32 arrays in the
    reference (x64 off), promoted to fp64 by np.hstack with the fp64 A_eq."""
    nvar = A["A_v_ineq"].shape[1]
    Av, Aa, Ap = (A[k].astype(gram_dtype) for k in ("A_v_ineq", "A_a_ineq", "A_p_ineq"))
    Q = (np.identity(nvar) + rho_ineq * (Av.T @ Av).astype(np.float64) + rho_ineq * (Aa.T @ Aa).astype(np.float64)
         + rho_ineq * (Ap.T @ Ap).astype(np.float64))
    Aeq = A["A_eq"]
    K = np.vstack((np.hstack((Q, Aeq.T)), np.hstack((Aeq, np.zeros((Aeq.shape[0], Aeq.shape[0]))))))
    return np.linalg.inv(K)


def boundary_vec(state_term, num_dof=6):
    """compute_boundary_vec_single (:174-178), batched."""
    n = state_term.shape[0]
    return state_term.reshape(n, 5, num_dof).transpose(0, 2, 1).reshape(n, 5 * num_dof)


def projection_filter(xi, state_term, A, Qinv, maxiter, v_max=0.8, a_max=1.8, p_max=np.pi, rho=1.0):
    """compute_projection_filter + compute_projection (:180-249)."""
    n, nvar = xi.shape
    m2 = A["A_v_ineq"].shape[0]
    b_eq = boundary_vec(state_term)
    s_v = np.zeros((n, m2)); s_a = np.zeros((n, m2)); s_p = np.zeros((n, m2))
    l_v = np.zeros((n, nvar)); l_a = np.zeros((n, nvar)); l_p = np.zeros((n, nvar))
    b_v = v_max * np.ones((n, m2)); b_a = a_max * np.ones((n, m2)); b_p = p_max * np.ones((n, m2))
    Av, Aa, Ap = A["A_v_ineq"], A["A_a_ineq"], A["A_p_ineq"]
    primal = xi
    for _ in range(maxiter):
        lincost = (-l_v - l_a - l_p - rho * xi - rho * (Av.T @ (b_v - s_v).T).T
                   - rho * (Aa.T @ (b_a - s_a).T).T - rho * (Ap.T @ (b_p - s_p).T).T)
        sol = (Qinv @ np.hstack((-lincost, b_eq)).T).T
        primal = sol[:, :nvar]
        s_v = np.maximum(0, -(Av @ primal.T).T + b_v)
        res_v = (Av @ primal.T).T - b_v + s_v
        s_a = np.maximum(0, -(Aa @ primal.T).T + b_a)
        res_a = (Aa @ primal.T).T - b_a + s_a
        s_p = np.maximum(0, -(Ap @ primal.T).T + b_p)
        res_p = (Ap @ primal.T).T - b_p + s_p
        l_v = l_v - rho * (Av.T @ res_v.T).T
        l_a = l_a - rho * (Aa.T @ res_a.T).T
        l_p = l_p - rho * (Ap.T @ res_p.T).T
    return primal


def cost_single(eef_pos, eef_rot, collision, target_pos, target_rot, w, y=0.005):
    """compute_cost_single (:276-303) for one candidate.
    eef_pos (H,3), eef_rot (H,4), collision (H,S)."""
    cg_ = np.linalg.norm(eef_pos - target_pos, axis=1)
    cost_g = cg_[-1] + np.sum(cg_[:-1])
    q = eef_rot / np.linalg.norm(eef_rot, axis=1, keepdims=True)
    dot = np.abs(q @ (target_rot / np.linalg.norm(target_rot)))
    cr_ = 2 * np.arccos(np.clip(dot, -1.0, 1.0))
    cost_r = cr_[-1] + np.sum(cr_[:-1])
    c = collision.T
    g = -c[:, 1:] + c[:, :-1] - y * c[:, :-1]
    cost_c = np.sum(np.maximum(g, 0)) + np.sum(c < 0)
    cost = w[0] * cost_g + w[1] * cost_r + w[2] * cost_c
    return cost, cost_g, cost_r, cost_c


def ellite(cost, xi, num_elite_frac):
    """compute_ellite_samples (:305-310): stable argsort, NaN last."""
    e = int(num_elite_frac * cost.shape[0])
    idx = np.argsort(cost, kind="stable")
    return xi[idx[:e]], idx, cost[idx[:e]]


def mean_cov(cost_ellite, mean_prev, cov_prev, xi_ellite, lamda=10.0, alpha_mean=0.6, alpha_cov=0.6):
    """compute_mean_cov + comp_prod (:318-335)."""
    w = np.exp(-(1.0 / lamda) * (cost_ellite - np.min(cost_ellite)))
    sw = np.sum(w)
    mean = (1 - alpha_mean) * mean_prev + alpha_mean * (np.sum(xi_ellite * w[:, None], axis=0) / sw)
    d = xi_ellite - mean
    prod = np.einsum("e,ei,ej->ij", w, d, d)
    cov = (1 - alpha_cov) * cov_prev + alpha_cov * prod / sw + 0.0001 * np.identity(mean.shape[0])
    return mean, cov

"""ADMM projection filter (SBP/mjx_planner.py:180-249) on the device.

Projects sampled Bernstein coefficients xi onto |Pdot xi| <= v_max,
|Pddot xi| <= a_max, |P xi| <= p_max with the boundary equalities
(theta0, thetadot0, thetaddot0 at t=0; zero velocity/acceleration at t=H-1)
through the precomputed KKT inverse Q_inv.  Same iteration as the reference
(rho = 1, zero-initialised slacks and multipliers, ``maxiter_projection``
unrolled updates), computed in fp32 like the reference (JAX x64 off).

The kron(I_6, [X; -X]) structure of A_{v,a,p}_ineq is applied as a per-joint
(N*6) x 11 x H product instead of the reference's dense 12H x 66 GEMMs (the
same sums, 6x fewer flops); Q_inv stays a dense 96 x 96 GEMM.
"""

from __future__ import annotations

import numpy as np
import torch


def kkt_inverse(P, Pdot, Pddot, num_dof=6, rho_ineq=1.0):
    """get_Q_inv (SBP/mjx_planner.py:166-172): fp32 Gram blocks, fp64 inverse."""
    I = np.identity(num_dof)
    A = {k: np.kron(I, np.vstack((X, -X))).astype(np.float32) for k, X in (("p", P), ("v", Pdot), ("a", Pddot))}
    nvar = A["v"].shape[1]
    Q = np.identity(nvar) + sum(rho_ineq * (A[k].T @ A[k]).astype(np.float64) for k in ("v", "a", "p"))
    Aeq = np.kron(I, np.vstack((P[0], Pdot[0], Pddot[0], Pdot[-1], Pddot[-1])))
    K = np.vstack((np.hstack((Q, Aeq.T)), np.hstack((Aeq, np.zeros((Aeq.shape[0], Aeq.shape[0]))))))
    return np.linalg.inv(K)


class ProjectionFilter:
    def __init__(self, P, Pdot, Pddot, num_dof, device, v_max=0.8, a_max=1.8, p_max=np.pi, rho=1.0):
        self.num_dof = num_dof
        self.nb = P.shape[1]
        self.H = P.shape[0]
        self.nvar = num_dof * self.nb
        self.device = device
        f32 = dict(dtype=torch.float32, device=device)
        self.P = torch.as_tensor(np.asarray(P, np.float32), **f32)
        self.Pdot = torch.as_tensor(np.asarray(Pdot, np.float32), **f32)
        self.Pddot = torch.as_tensor(np.asarray(Pddot, np.float32), **f32)
        self.Qinv = torch.as_tensor(kkt_inverse(P, Pdot, Pddot, num_dof, rho).astype(np.float32), **f32)
        self.bounds = (float(v_max), float(a_max), float(p_max))
        self.rho = float(rho)

    def _fwd(self, X, xi):  # A_ineq xi -> (N, dof, 2H)
        v = xi @ X.T
        return torch.cat((v, -v), dim=2)

    def _adj(self, X, y):  # A_ineq^T y, y (N, dof, 2H) -> (N, dof, nb)
        return (y[:, :, : self.H] - y[:, :, self.H:]) @ X

    def boundary(self, init_pos, init_vel, init_acc, n):
        """b_eq per candidate (compute_cem state_term -> compute_boundary_vec_single, :174-178, :374-384)."""
        d = self.num_dof
        st = torch.zeros((d, 5), dtype=torch.float32, device=self.device)
        st[:, 0] = torch.as_tensor(np.asarray(init_pos, np.float32)[:d], device=self.device)
        st[:, 1] = torch.as_tensor(np.asarray(init_vel, np.float32)[:d], device=self.device)
        st[:, 2] = torch.as_tensor(np.asarray(init_acc, np.float32)[:d], device=self.device)
        return st.reshape(1, 5 * d).expand(n, 5 * d)

    @torch.no_grad()
    def __call__(self, xi_samples, b_eq, maxiter):
        n = xi_samples.shape[0]
        d, nb, H = self.num_dof, self.nb, self.H
        xi = xi_samples.reshape(n, d, nb)
        mats = (self.Pdot, self.Pddot, self.P)
        s = [torch.zeros((n, d, 2 * H), dtype=torch.float32, device=self.device) for _ in range(3)]
        lam = [torch.zeros((n, d, nb), dtype=torch.float32, device=self.device) for _ in range(3)]
        primal = xi
        for _ in range(maxiter):
            lincost = -lam[0] - lam[1] - lam[2] - self.rho * xi
            for k in range(3):
                lincost = lincost - self.rho * self._adj(mats[k], self.bounds[k] - s[k])
            rhs = torch.cat((-lincost.reshape(n, d * nb), b_eq), dim=1)
            sol = rhs @ self.Qinv.T
            primal = sol[:, : d * nb].reshape(n, d, nb)
            for k in range(3):
                ax = self._fwd(mats[k], primal)
                s[k] = torch.clamp_min(self.bounds[k] - ax, 0.0)
                res = ax - self.bounds[k] + s[k]
                lam[k] = lam[k] - self.rho * self._adj(mats[k], res)
        return primal.reshape(n, d * nb).contiguous()

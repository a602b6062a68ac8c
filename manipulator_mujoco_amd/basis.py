"""Bernstein basis of order n and its time derivatives (host, fp64).

Restates ``bernstein_coeff_ordern_new`` (SBP/bernstein_coeff_ordern_arbitinterval.py:4-28),
which the planner calls at SBP/mjx_planner.py:40 with n = 10 on the grid
``linspace(0, H*dt, H)`` (:36).  The closed-form order-10 variant
(SBP/bernstein_coeff_order10_arbitinterval.py:13-103) is the same function.
Checked against golden vectors generated from the reference
(tests/golden/basis.npz, tools/make_golden.py).
"""

from __future__ import annotations

from math import comb

import numpy as np


def _b(n, i, t):
    if i < 0 or i > n:
        return np.zeros_like(t)
    return comb(n, i) * (1.0 - t) ** (n - i) * t ** i


def bernstein(n: int, tmin: float, tmax: float, t) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """P, Pdot, Pddot, each (len(t), n+1), on the normalised time (t - tmin)/(tmax - tmin)."""
    t = np.asarray(t, dtype=np.float64).reshape(-1)
    l = float(tmax - tmin)
    x = (t - tmin) / l
    P = np.stack([_b(n, i, x) for i in range(n + 1)], axis=1)
    # d/dx B_{n,i} = n (B_{n-1,i-1} - B_{n-1,i})
    Pd = np.stack([n * (_b(n - 1, i - 1, x) - _b(n - 1, i, x)) for i in range(n + 1)], axis=1) / l
    # d2/dx2 B_{n,i} = n (n-1) (B_{n-2,i-2} - 2 B_{n-2,i-1} + B_{n-2,i})
    Pdd = np.stack([n * (n - 1) * (_b(n - 2, i - 2, x) - 2 * _b(n - 2, i - 1, x) + _b(n - 2, i, x))
                    for i in range(n + 1)], axis=1) / (l * l)
    return P, Pd, Pdd


def planner_basis(num_steps: int, timestep: float, order: int = 10):
    """The planner's time grid and basis (SBP/mjx_planner.py:34-46)."""
    t_fin = num_steps * timestep
    tot_time = np.linspace(0.0, t_fin, num_steps)
    P, Pd, Pdd = bernstein(order, tot_time[0], tot_time[-1], tot_time)
    return tot_time, P, Pd, Pdd

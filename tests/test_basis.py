"""A1: Bernstein basis vs golden vectors generated from the reference
(SBP/bernstein_coeff_ordern_arbitinterval.py:4-28, order-10 file :13-103)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from manipulator_mujoco_amd import basis

G = np.load(os.path.join(GOLDEN, "basis.npz"))


@pytest.mark.parametrize("H", [10, 16, 20, 50, 100])
def test_basis_matches_reference(H):
    t, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    np.testing.assert_allclose(t, G[f"H{H}_t"], rtol=0, atol=1e-15)
    for got, key in ((P, "P"), (Pd, "Pdot"), (Pdd, "Pddot")):
        ref = G[f"H{H}_{key}"]
        scale = np.abs(ref).max()
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * scale)
        # the closed-form order-10 module is the same function
        np.testing.assert_allclose(G[f"H{H}_{key}10"], ref, rtol=0, atol=1e-11 * scale)


def test_partition_of_unity_and_derivatives():
    t, P, Pd, Pdd = basis.planner_basis(50, 0.05)
    np.testing.assert_allclose(P.sum(1), 1.0, atol=1e-13)
    np.testing.assert_allclose(Pd.sum(1), 0.0, atol=1e-11)
    np.testing.assert_allclose(Pdd.sum(1), 0.0, atol=1e-9)

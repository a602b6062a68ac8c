"""Hull support ties: the support of a convex hull must
not depend on where its hill climb starts.  A direction normal to a hull
edge or face makes every vertex of it a maximum; the climb's end then
depends on its start (the support start table's cell, the pair's hint) and
on the last bits of the dot products.  The tie rule (oracle hull_tie, the
kernel's sup_finish / tie_round) walks from the climb's end to the tie's
lowest vertex index, so a start table whose every cell points at a random
vertex of its hull gives bitwise the same rollouts -- a table resolution is
a performance choice, not a parity change.  Without the rule (tie band 0)
the same batch changes (the test's teeth).  CPU only: the fp64 oracle and
its fp32 build over a dual-arm batch (URD/dual_arm_gripper_scene.xml)."""
import ctypes
import os
import sys

import numpy as np
import pytest

import oracle
from manipulator_mujoco_amd import models

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
ARGS = (Q0, [20.0, 3.0, 80.0], [-0.3, -0.3, 0.5], [0.0, 1.0, 0.0, 0.0])


@pytest.fixture(scope="module")
def batch():
    from diag_f32 import batch as make
    m = models.load("dual_arm", 0.05)
    return m, make(m, 256, 100, 4)


def _costs(m, td, prec, scramble):
    """cost4 of the batch; scramble: the oracle's start tables name hashed
    vertices of each hull (oracle_set_start_scramble) instead of the extreme one."""
    L = oracle.lib_f32() if prec == "fp32" else oracle.lib()
    L.oracle_set_start_scramble.argtypes = [ctypes.c_ulonglong]
    L.oracle_set_start_scramble(1 if scramble else 0)
    try:
        if prec == "fp64":
            return oracle.rollout(m, td, *ARGS, want_theta=False, workers=8)["cost4"]
        r = oracle.Runner(m, 8, *ARGS, precision="fp32", exact_mask=4)
        try:
            return r.rollout(td).astype(np.float64)
        finally:
            r.close()
    finally:
        L.oracle_set_start_scramble(0)


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_support_is_start_independent(batch, prec):
    m, td = batch
    L = oracle.lib_f32() if prec == "fp32" else oracle.lib()
    L.oracle_set_hull_tie.argtypes = [ctypes.c_float if prec == "fp32" else ctypes.c_double]
    try:
        for tie, same in ((1e-7, True), (0.0, False)):
            L.oracle_set_hull_tie(tie)
            L.oracle_set_hint_ge(1 if same else 0)  # the teeth: the plain climb (the table's start on equal values)
            a = _costs(m, td, prec, False)
            b = _costs(m, td, prec, True)
            if same:
                np.testing.assert_array_equal(a, b, err_msg=f"{prec}: the start table moved a rollout")
            else:  # teeth: without the rule the random starts end on other tied vertices
                assert (a[:, 0] != b[:, 0]).any(), prec
    finally:
        L.oracle_set_hull_tie(1e-7)
        L.oracle_set_hint_ge(1)

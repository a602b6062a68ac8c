"""A8: quaternion helpers vs golden outputs of SBP/quat_math.py; the oracle's
rotation cost term (SBP/mjx_planner.py:281-283) uses the same distance."""
import os

import numpy as np

from conftest import GOLDEN
from manipulator_mujoco_amd import quat_math as qm
from oracle import cem_np

Z = np.load(os.path.join(GOLDEN, "quat.npz"))


def test_distance_multiply_rotation():
    d = np.array([qm.quaternion_distance(a, b) for a, b in zip(Z["q1"], Z["q2"])])
    np.testing.assert_array_equal(d, Z["distance"])
    mul = np.array([qm.quaternion_multiply(a, b) for a, b in zip(Z["q1"], Z["q2"])])
    np.testing.assert_array_equal(mul, Z["multiply"])
    rot = np.array([qm.rotation_quaternion(a, x) for a, x in zip(Z["angle_deg"], Z["axis"])])
    np.testing.assert_array_equal(rot, Z["rotation"])
    assert np.all(d[:8] < 1e-6)  # identical and antipodal pairs


def test_cost_rotation_term_is_quaternion_distance():
    H = len(Z["q1"])
    eef_rot = Z["q1"] * 3.0  # unnormalised: the cost normalises
    _, _, cr, _ = cem_np.cost_single(np.zeros((H, 3)), eef_rot, np.ones((H, 1)), np.zeros(3), Z["q2"][0] * 2.0,
                                     (1, 1, 1))
    ref = sum(qm.quaternion_distance(q, Z["q2"][0]) for q in Z["q1"])
    np.testing.assert_allclose(cr, ref, rtol=1e-12)

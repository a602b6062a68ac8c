"""Quaternion helpers with the reference's API (SBP/quat_math.py:1-23).

The in-kernel rotation cost uses the same distance on normalised quaternions
(SBP/mjx_planner.py:281-283); these host versions serve the MPC driver's
logging (SBP/mpc_planner.py:184).
"""

from __future__ import annotations

import numpy as np


def quaternion_distance(q1, q2):
    d = np.abs(np.dot(q1, q2))
    d = np.clip(d, -1.0, 1.0)
    return 2 * np.arccos(d)


def rotation_quaternion(angle_deg, axis):
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.linalg.norm(axis)
    half = np.deg2rad(angle_deg) / 2
    w = np.cos(half)
    x, y, z = axis * np.sin(half)
    return (round(w, 5), round(x, 5), round(y, 5), round(z, 5))


def quaternion_multiply(q1, q2):
    """The reference's product, which is the Hamilton product q2 * q1
    (scalar w1 w2 - v1.v2, vector w1 v2 + w2 v1 + v2 x v1), rounded to 5 digits."""
    a = np.asarray(q1, dtype=np.float64)
    b = np.asarray(q2, dtype=np.float64)
    w = a[0] * b[0] - np.dot(a[1:], b[1:])
    v = a[0] * b[1:] + b[0] * a[1:] + np.cross(b[1:], a[1:])
    return tuple(round(float(c), 5) for c in (w, v[0], v[1], v[2]))

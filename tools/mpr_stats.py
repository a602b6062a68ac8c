"""MPR work profile of the dual-arm rollouts on the fp64 oracle (diagnostic):
calls, support pairs and hull-climb rounds per step, the histogram of
support pairs per call, and the same per 64-lane flush chunk model.

    python tools/mpr_stats.py [n] [H]
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.projection import ProjectionFilter  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
H = int(sys.argv[2]) if len(sys.argv) > 2 else 100
m = models.load("dual_arm", 0.05)
_, P, Pd, Pdd = basis.planner_basis(H, 0.05)
Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
f = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
xi = f(torch.tensor(np.random.default_rng(20250629 + 4).normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)),
       f.boundary(Q0, np.zeros(6), np.zeros(6), n), 10).numpy()
td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
L = oracle.lib()
L.oracle_mpr_stats.argtypes = [ctypes.POINTER(ctypes.c_long), ctypes.c_int]
st = (ctypes.c_long * 64)()
L.oracle_mpr_stats(st, 1)
oracle.rollout(m, td, Q0, [20, 3, 80], [-0.3, -0.3, 0.5], [0, 1, 0, 0], want_theta=False, workers=1)
L.oracle_mpr_stats(st, 0)
steps = n * H
s = np.array(st[:])
print(f"per step: mpr calls {s[0] / steps:.1f}, hits {s[4] / steps:.2f}, support pairs {s[1] / steps:.1f}, "
      f"climb rounds {s[2] / steps:.1f}, neighbour evals {s[3] / steps:.1f}")
h = s[16:64]
print("support pairs per call: " + " ".join(f"{k}:{v}" for k, v in enumerate(h) if v))
print(f"per call: support pairs {s[1] / max(s[0], 1):.2f}, climb rounds per support {s[2] / max(2 * s[1], 1):.2f}")
if s[8]:
    print(f"polyhedron manifold per step: calls {s[8] / steps:.2f}, reaching the clip {s[11] / steps:.2f}; per call: "
          f"candidate faces {s[9] / s[8]:.1f} (support-vertex faces {s[15] / s[8]:.1f}), faces scanned "
          f"{s[10] / s[8]:.0f}; per clip: reference vertices {s[12] / max(s[11], 1):.1f}, incident vertices "
          f"{s[13] / max(s[11], 1):.1f}, climb rounds {s[14] / max(s[11], 1):.1f}; clips keeping no point "
          f"{s[5] / steps:.3f} per step")

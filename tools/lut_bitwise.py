"""The C4 shard's cost4 from the library in argv[1] (a build at some
-DMPCR_LUT_R; the engine builds its start table), saved to argv[2]: a bitwise
comparison between support start-table resolutions (diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from manipulator_mujoco_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
import torch  # noqa: E402

from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine  # noqa: E402
from test_gpu_parity import PT, Q0, QT, W, projected_xi  # noqa: E402

n, H = 4096, 100
m = models.load("dual_arm", 0.05)
_, P, Pd, _ = basis.planner_basis(H, 0.05)
xi = projected_xi(n, H, 20250629 + 4, torch.device("cuda:0"))
e = Engine(m, H, n, Pd)
a = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT).cpu().numpy()
np.save(sys.argv[2], a)
print(sys.argv[1], float(a[:, 0].sum()))

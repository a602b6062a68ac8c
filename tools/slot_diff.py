"""Per-step masked contact-slot distances of one candidate from the kernel
(Engine.trace), saved for a CPU comparison with the oracle's (diagnostic).
The batch is tests/test_gpu_parity.py::test_parity_small's thetadot layout.

    python tools/slot_diff.py planner_scene 30 gpurun_out/slots.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401

from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_THETADOT, Engine  # noqa: E402
from parity_util import PT, Q0, QT, W  # noqa: E402

name, cand, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
n, H = 64, 20
m = models.load(name, 0.05)
_, P, Pd, _ = basis.planner_basis(H, 0.05)
rng = np.random.default_rng(11)
t = np.arange(H) * 0.05
inp = (rng.uniform(-0.7, 0.7, (n, 6, 1)) * np.sin(rng.uniform(0.2, 2, (n, 6, 1)) * t)).reshape(n, 6 * H)
inp = inp.astype(np.float32)
e = Engine(m, H, n, Pd)
g = e.trace(inp, MPCR_LAYOUT_THETADOT, Q0, W, PT, QT)
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
np.savez(out, cost4=g["cost4"][cand], slots=g["slots"][cand], theta=g["theta"][cand], inp=inp[cand])
print(name, cand, g["cost4"][cand])

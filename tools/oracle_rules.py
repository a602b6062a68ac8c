"""What each of the oracle's rules moves:
oracle vs oracle on the dual-arm C4 batch (seed 20250629 + 4, projected on
the CPU), every rule MuJoCo-exact except the one under test, which runs at
the kernel's value.  Prints, per rule, how many well-conditioned candidates
(probe A < 1e-5, tests/parity_util.py) move by more than 1e-4.  CPU only.

    python tools/oracle_rules.py [n=1024] [H=100]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import oracle  # noqa: E402
import parity_util as pu  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.projection import ProjectionFilter  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
H = int(sys.argv[2]) if len(sys.argv) > 2 else 100
m = models.load("dual_arm", 0.05)
_, P, Pd, Pdd = basis.planner_basis(H, 0.05)
f = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
rng = np.random.default_rng(20250629 + 4)
xi = f(torch.tensor(rng.normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)),
       f.boundary(pu.Q0, np.zeros(6), np.zeros(6), n), 10).numpy()
td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
KERNEL = (1e-6, 1e-5, 1e-6, 1e-5)  # the round-2 kernel's Newton floor, climb band, axis tie, MPR tolerance


def run(mask, floors):
    with oracle.exact(mask, floors):
        return oracle.rollout(m, td, pu.Q0, pu.W, pu.PT, pu.QT, want_theta=False, workers=pu.WORKERS)["cost4"][:, 0]


with oracle.exact(31):
    _, sens = pu.conditioning(m, td)
well = sens < pu.TOL / 10
ex = run(31, None)
print(f"{n} x {H}: {int(well.sum())} well-conditioned")
for name, bit, k in (("Newton stop floor", 1, 0), ("line-search bracket floor", 2, None), ("MPR tolerance", 4, 3),
                     ("hull climb band", 8, 1), ("support axis tie", 8, 2), ("manifold picks", 16, None)):
    fl = [0.0, 0.0, -1.0, 1e-6]  # exact values: no floors, strict climb, mju_sign tie, ccd_tolerance
    if k is not None:
        fl[k] = KERNEL[k]
    c = run(31 & ~bit, fl)
    r = np.abs(c - ex) / np.abs(ex)
    print(f"{name:28s} moves {int((well & (r > 1e-4)).sum()):4d} well-conditioned candidates by > 1e-4")

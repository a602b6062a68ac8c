"""Which stage's fp32 precision moves the dual arm's trajectories?  (CPU
experiment)  The fp64 oracle with the outputs of chosen stages rounded to
fp32 every step (oracle_set_round32, mpcr_oracle.c forward / euler), against
the plain fp64 oracle: well-conditioned candidates (tests/parity_util.py)
moved by more than 1e-4, per stage.

    python tools/stage_precision.py [model=dual_arm] [n=4096] [H=100] [seed=4] [--xi=gpurun_out/xi_....npy]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import oracle  # noqa: E402
import parity_util as pu  # noqa: E402
from diag_f32 import batch  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402

STAGES = [(1, "kinematics (poses)"), (2, "COM / cinert / cdof"), (4, "mass matrix"), (8, "contacts"),
          (16, "velocities"), (32, "passive + bias + actuator forces"), (64, "constraint rows J, D, aref"),
          (128, "qacc_smooth"), (256, "qacc (solver output)"), (512, "Euler state (qpos, qvel, warm start)"),
          (1023, "all of the above")]


def main():
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    name = a[0] if a else "dual_arm"
    n = int(a[1]) if len(a) > 1 else 4096
    H = int(a[2]) if len(a) > 2 else 100
    seed = int(a[3]) if len(a) > 3 else 4
    m = models.load(name, 0.05)
    xs = [x for x in sys.argv if x.startswith("--xi=")]
    if xs:
        xi = np.load(xs[0][5:])[:n]
        _, _, Pd, _ = basis.planner_basis(H, 0.05)
        td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
    else:
        td = batch(m, n, H, seed)
    L = oracle.lib()
    L.oracle_set_round32.argtypes = [ctypes.c_int]
    with oracle.exact(4):
        o, sens = pu.conditioning(m, td)
        well = (sens < pu.TOL / 10) & ~pu.grazing(m, o)
        oc = o["cost4"][:, 0]
        print(f"{name} {n} x {H}: well {int(well.sum())}, probe B {int((well & (o['probe_b'] >= pu.TOL)).sum())}, "
              f"probe F (fp32 build) {int((well & (o['probe_f4'][:, 0] >= pu.TOL)).sum())}")
        for bit, label in STAGES:
            L.oracle_set_round32(bit)
            try:
                c = oracle.rollout(m, td, pu.Q0, pu.W, pu.PT, pu.QT, want_theta=False, workers=pu.WORKERS)["cost4"][:, 0]
            finally:
                L.oracle_set_round32(0)
            r = np.abs(c - oc) / np.abs(oc)
            print(f"  fp32 outputs of {label:40s} well-conditioned misses {int((well & (r >= pu.TOL)).sum()):4d}  "
                  f"all {(r >= pu.TOL).mean():.3f}  median {np.median(r):.1e}")


if __name__ == "__main__":
    main()

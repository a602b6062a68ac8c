"""Narrow-phase calls executed per step, by pair function, on the fp64 oracle
(after the bounding-sphere / plane culls; robot-masked pairs always run for
cost_c's slot distances).  bench/flops_model.json credits the executed calls
only (culled pairs were credited at full cost).  CPU only.

    python tools/narrow_stats.py [model=scene_mjx] [n=256] [H=50] [seed=3]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle  # noqa: E402
from diag_f32 import batch  # noqa: E402
from manipulator_mujoco_amd import models  # noqa: E402

NAMES = {0: "plane_capsule", 1: "plane_box", 2: "capsule_capsule", 3: "capsule_box", 4: "box_box", 9: "convex",
         10: "plane_convex"}


def main():
    a = sys.argv[1:]
    name = a[0] if a else "scene_mjx"
    n = int(a[1]) if len(a) > 1 else 256
    H = int(a[2]) if len(a) > 2 else 50
    seed = int(a[3]) if len(a) > 3 else 3
    m = models.load(name, 0.05)
    td = batch(m, n, H, seed)
    L = oracle.lib()
    L.oracle_narrow_stats.argtypes = [ctypes.POINTER(ctypes.c_long), ctypes.c_int]
    st = (ctypes.c_long * 16)()
    L.oracle_narrow_stats(st, 1)
    oracle.rollout(m, td, [1.5, -1.8, 1.75, -1.25, -1.6, 0.0], [20, 3, 80], [-0.3, -0.3, 0.5], [0, 1, 0, 0],
                   want_theta=False, workers=1)
    L.oracle_narrow_stats(st, 0)
    steps = n * H
    tot = {f: int(np.sum(np.asarray(m.pair_func) == f)) for f in NAMES}
    out = {NAMES[f]: round(st[f] / steps, 3) for f in NAMES if tot[f]}
    print(f"{name} {n} x {H}: executed narrow-phase calls per step {out}; pairs {({NAMES[f]: tot[f] for f in NAMES if tot[f]})}")


if __name__ == "__main__":
    main()

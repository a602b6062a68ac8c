"""Probe F (fp32 restatement vs the fp64 oracle) on a dual-arm batch with and
without the hull support tie rule (diagnostic): how many
well-conditioned candidates fp32 arithmetic alone moves past 1e-4, per cost
component.

    python tools/tie_probe_f.py [n=1024] [H=100] [seed=4]
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
from manipulator_mujoco_amd import models  # noqa: E402

kw = dict(a.split("=") for a in sys.argv[1:])
n, H, seed = int(kw.get("n", 1024)), int(kw.get("H", 100)), int(kw.get("seed", 4))
ties = [float(x) for x in kw.get("ties", "0,1e-7").split(",")]
m = models.load("dual_arm", 0.05)
td = batch(m, n, H, seed)
L, L32 = oracle.lib(), oracle.lib_f32()
L.oracle_set_hull_tie.argtypes = [ctypes.c_double]
L32.oracle_set_hull_tie.argtypes = [ctypes.c_float]
for t in ties:
    L.oracle_set_hull_tie(t)
    L32.oracle_set_hull_tie(t)
    o, sens = pu.conditioning(m, td, seed=7)
    out = []
    for k, name in enumerate(("total", "g", "r")):
        s4, pf, pb = o["sens4"][:, k], o["probe_f4"][:, k], o["probe_b4"][:, k]
        well = s4 < pu.TOL / 10
        out.append(f"{name}: well {well.sum()} F-miss {(well & (pf >= pu.TOL)).sum()} B-miss "
                   f"{(well & (pb >= pu.TOL)).sum()} worst-F {pf[well].max():.2e} all-F {(pf >= pu.TOL).sum()}")
    print(f"hull tie {t:g}: " + "; ".join(out), flush=True)

"""Is the hull support independent of where its climb starts?  (diagnostic,
VERDICT r5 item 1)

Rolls a dual-arm batch out with the fp64 oracle twice: with the model's
support start table, and with every table cell pointing at a random vertex
of its hull (the climb then starts somewhere else for every query).  With
the hull tie rule (oracle hull_tie, HULL_TIE) the costs should agree bit for
bit; without it (oracle_set_hull_tie(0)) ties end on whichever tied vertex
the climb reaches first.

    python tools/tie_start_independence.py [n=128] [H=50] [tie=1e-7]
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from manipulator_mujoco_amd import cmodel, models  # noqa: E402
from diag_f32 import batch  # noqa: E402  (tools/)

kw = dict(a.split("=") for a in sys.argv[1:])
n, H, tie = int(kw.get("n", 128)), int(kw.get("H", 50)), float(kw.get("tie", 1e-7))
m = models.load("dual_arm", 0.05)
td = batch(m, n, H, 4)
L = oracle.lib()
L.oracle_set_hull_tie.argtypes = [ctypes.c_double]
L.oracle_set_exact.argtypes = [ctypes.c_int]
L.oracle_set_exact(4)  # the kernel's rules (tests/parity_util.py)
orig = cmodel.hull_luts


def scrambled(mm, seed=1):
    adr, lut = orig(mm)
    lut = np.array(lut, copy=True)
    rng = np.random.default_rng(seed)
    R = cmodel.LUT_R
    for g in range(len(mm.geom_type)):
        if mm.geom_hulladr[g] >= 0 and mm.geom_hullnum[g] > 0 and adr[g] >= 0:
            lut[adr[g]:adr[g] + 6 * R * R] = mm.geom_hulladr[g] + rng.integers(0, mm.geom_hullnum[g], 6 * R * R)
    return adr, lut


Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
ARGS = (Q0, [20.0, 3.0, 80.0], [-0.3, -0.3, 0.5], [0.0, 1.0, 0.0, 0.0])
L32 = oracle.lib_f32()
L32.oracle_set_hull_tie.argtypes = [ctypes.c_float]
for prec in ("fp64", "fp32"):
    for t in (0.0, tie):
        (L32 if prec == "fp32" else L).oracle_set_hull_tie(t)
        (L32 if prec == "fp32" else L).oracle_set_hint_ge(1 if t > 0 else 0)  # no rule: the plain climb's start
        res = []
        for scr in (False, True):
            cmodel.hull_luts = scrambled if scr else orig
            t0 = time.time()
            if prec == "fp64":
                res.append(oracle.rollout(m, td, *ARGS, want_theta=False, workers=8)["cost4"])
            else:
                r = oracle.Runner(m, 8, *ARGS, precision="fp32", exact_mask=4)
                res.append(r.rollout(td).astype(np.float64))
                r.close() if hasattr(r, "close") else None
        cmodel.hull_luts = orig
        (L32 if prec == "fp32" else L).oracle_set_hint_ge(1)
        a, b = res
        rel = np.abs(a[:, 0] - b[:, 0]) / np.abs(a[:, 0])
        print(f"{prec} hull tie {t:g}: candidates differing {(a[:, 0] != b[:, 0]).sum()}/{n}, >1e-6 "
              f"{(rel > 1e-6).sum()}, >1e-4 {(rel > 1e-4).sum()}, worst {rel.max():.2e}", flush=True)

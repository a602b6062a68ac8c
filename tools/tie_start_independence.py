"""Is the hull support independent of where its climb starts?  (diagnostic,
VERDICT r5 item 1)

Rolls a dual-arm batch out with the fp64 oracle twice: with its support
start table, and with every table cell pointing at a hashed vertex of its
hull (oracle_set_start_scramble) (the climb then starts somewhere else for every query).  With
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
from manipulator_mujoco_amd import models  # noqa: E402
from diag_f32 import batch  # noqa: E402  (tools/)

kw = dict(a.split("=") for a in sys.argv[1:])
n, H, tie = int(kw.get("n", 128)), int(kw.get("H", 50)), float(kw.get("tie", 1e-7))
m = models.load("dual_arm", 0.05)
td = batch(m, n, H, 4)
L = oracle.lib()
L.oracle_set_hull_tie.argtypes = [ctypes.c_double]
L.oracle_set_exact.argtypes = [ctypes.c_int]
L.oracle_set_exact(4)  # the kernel's rules (tests/parity_util.py)


Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
ARGS = (Q0, [20.0, 3.0, 80.0], [-0.3, -0.3, 0.5], [0.0, 1.0, 0.0, 0.0])
L32 = oracle.lib_f32()
L32.oracle_set_hull_tie.argtypes = [ctypes.c_float]
for lib in (L, L32):
    lib.oracle_set_start_scramble.argtypes = [ctypes.c_ulonglong]
for prec in ("fp64", "fp32"):
    for t in (0.0, tie):
        (L32 if prec == "fp32" else L).oracle_set_hull_tie(t)
        (L32 if prec == "fp32" else L).oracle_set_hint_ge(1 if t > 0 else 0)  # no rule: the plain climb's start
        res = []
        for scr in (False, True):
            (L32 if prec == "fp32" else L).oracle_set_start_scramble(1 if scr else 0)
            t0 = time.time()
            if prec == "fp64":
                res.append(oracle.rollout(m, td, *ARGS, want_theta=False, workers=8)["cost4"])
            else:
                r = oracle.Runner(m, 8, *ARGS, precision="fp32", exact_mask=4)
                res.append(r.rollout(td).astype(np.float64))
                r.close() if hasattr(r, "close") else None
        (L32 if prec == "fp32" else L).oracle_set_start_scramble(0)
        (L32 if prec == "fp32" else L).oracle_set_hint_ge(1)
        a, b = res
        rel = np.abs(a[:, 0] - b[:, 0]) / np.abs(a[:, 0])
        print(f"{prec} hull tie {t:g}: candidates differing {(a[:, 0] != b[:, 0]).sum()}/{n}, >1e-6 "
              f"{(rel > 1e-6).sum()}, >1e-4 {(rel > 1e-4).sum()}, worst {rel.max():.2e}", flush=True)

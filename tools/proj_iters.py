"""Projection kernel time against its ADMM iteration count (diagnostic):
    python tools/proj_iters.py [n] [H]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench_cem import ev_time  # noqa: E402
from manipulator_mujoco_amd.planner import cem_planner  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
H = int(sys.argv[2]) if len(sys.argv) > 2 else 50
p = cem_planner(num_dof=6, num_batch=n, num_steps=H, timestep=0.05, maxiter_cem=1, num_elite=0.05, w_pos=20.0,
                w_rot=3.0, w_col=80.0, maxiter_projection=10, verbose=False)
p.compute_cem(np.zeros(66), np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0]), np.zeros(6), np.zeros(6),
              np.array([-0.3, -0.3, 0.5]), np.array([0.0, 1.0, 0.0, 0.0]))
bounds = (0.8, 1.8, np.pi)
for it in (0, 1, 2, 5, 10):
    t = ev_time(lambda: p.cem.project(p._xs, p._beq, it, bounds, out=p._xf))
    print(f"n {n} H {H} maxiter {it}: {t:.4f} ms")

"""Time the CEM distribution-step kernels and one whole compute_cem tick.

    python tools/bench_cem.py [--n 4096] [--H 50] [--iters 3]

Per-kernel durations come from HIP events on the launch stream (median of
repeats); the tick is wall time around compute_cem (host sync included).
Prints one JSON line.  Diagnostic only (not the bench.py contract).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ev_time(fn, reps=20):
    import torch
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--H", type=int, default=50)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--model", default="scene_mjx")
    args = ap.parse_args()
    import torch

    from manipulator_mujoco_amd.cem import topk
    from manipulator_mujoco_amd.planner import cem_planner
    from manipulator_mujoco_amd.projection import ProjectionFilter
    n, H = args.n, args.H
    p = cem_planner(num_dof=6, num_batch=n, num_steps=H, timestep=0.05, maxiter_cem=args.iters, num_elite=0.05,
                    w_pos=20.0, w_rot=3.0, w_col=80.0, maxiter_projection=10, model_path=args.model, verbose=False)
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    pt, qt = np.array([-0.3, -0.3, 0.5]), np.array([0.0, 1.0, 0.0, 0.0])
    p.compute_cem(np.zeros(p.nvar), q0, np.zeros(6), np.zeros(6), pt, qt)  # warm-up
    bounds = (p.v_max, p.a_max, p.p_max)
    res = {"n": n, "H": H, "model": args.model}
    res["factor_ms"] = ev_time(lambda: p.cem.factor(p._cov, 0.003))
    res["sample_project_ms"] = ev_time(lambda: p.cem.sample_project(n, p._mean, 1, 0, p._beq, 10, bounds,
                                                                     xi_samples=p._xs, out=p._xf))
    res["project_only_ms"] = ev_time(lambda: p.cem.project(p._xs, p._beq, 10, bounds, out=p._xf))
    cost4 = torch.empty((n, 4), device=p.device)
    res["rollout_ms"] = ev_time(lambda: p.engine.rollout_cost(p._xf, 0, q0, (20, 3, 80), pt, qt, cost4=cost4),
                                reps=5)
    res["topk_ms"] = ev_time(lambda: topk(p.engine, cost4, p.ellite_num, stride=4, out=p._idx))
    m0, c0 = p._mean.clone(), p._cov.clone()

    def upd():
        p._mean.copy_(m0)
        p._cov.copy_(c0)
        p.cem.update(p._xs, cost4, 4, p._idx, 10.0, 0.6, 0.6, p._mean, p._cov)
    res["update_ms_incl_2_copies"] = ev_time(upd)
    # the torch-op projection this replaces (projection.py), same inputs
    f = ProjectionFilter(p.P, p.Pdot, p.Pddot, 6, p.device)
    beq = f.boundary(q0, np.zeros(6), np.zeros(6), n)
    res["torch_projection_ms"] = ev_time(lambda: f(p._xs, beq, 10), reps=5)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        p.compute_cem(np.zeros(p.nvar), q0, np.zeros(6), np.zeros(6), pt, qt)
        ts.append((time.perf_counter() - t0) * 1e3)
    res["compute_cem_ms"] = float(np.median(ts))
    res["iters"] = args.iters
    print(json.dumps(res))


if __name__ == "__main__":
    main()

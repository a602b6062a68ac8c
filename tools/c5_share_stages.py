"""Per-stage times of the C5 tick at one rank's share on 8 GPUs (VERDICT r5
item 3): the 8192 x 50 x 3 closed loop split over 8 ranks gives each rank
1024 candidates per CEM iteration while the elite set stays the global one
(5 % of 8192 = 409 rows).  One GPU times every device stage of that share
with HIP events on the launch stream (median of repeats):

  per CEM iteration (x 3): Cholesky factor, MVN sample + projection (1024),
  rollout + cost (1024 x 50, the two-wave dual-arm kernel), local top-E
  (409 of 1024), [elite all-gather: 8 x 409 rows of (xi, cost)], global
  top-E (409 of 8 x 409), mean / cov update (409 elites);
  per tick: the plant step (one environment, n = 1, H = 1).

The all-gather itself needs 8 ranks (RCCL over xGMI, 8 x 409 x 67 floats =
877 KB per iteration); it is reported by its size only.  The tick is then
3 x (iteration) + plant, against the 1-GPU tick of bench.py --config c5.
Diagnostic only.

    python tools/c5_share_stages.py [--n 1024] [--ranks 8]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from bench_cem import ev_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--H", type=int, default=50)
    args = ap.parse_args()
    import torch

    from manipulator_mujoco_amd.cem import topk
    from manipulator_mujoco_amd.engine import Plant
    from manipulator_mujoco_amd.planner import cem_planner
    n, H, G = args.n, args.H, args.ranks
    E = int(0.05 * n * G)  # the global elite count
    p = cem_planner(num_dof=6, num_batch=n, num_steps=H, timestep=0.05, maxiter_cem=3, num_elite=E / n, w_pos=20.0,
                    w_rot=3.0, w_col=80.0, maxiter_projection=10, model_path="dual_arm", verbose=False)
    assert p.ellite_num == E, (p.ellite_num, E)
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    pt, qt = np.array([-0.3, -0.3, 0.5]), np.array([0.0, 1.0, 0.0, 0.0])
    p.compute_cem(np.zeros(p.nvar), q0, np.zeros(6), np.zeros(6), pt, qt)  # warm-up, realistic mean / cov
    bounds = (p.v_max, p.a_max, p.p_max)
    res = {"share": n, "ranks": G, "global_batch": n * G, "H": H, "global_elites": E}
    res["factor_ms"] = ev_time(lambda: p.cem.factor(p._cov, 0.003))
    res["sample_project_ms"] = ev_time(lambda: p.cem.sample_project(n, p._mean, 1, 0, p._beq, 10, bounds,
                                                                     xi_samples=p._xs, out=p._xf))
    cost4 = torch.empty((n, 4), device=p.device)
    res["rollout_ms"] = ev_time(lambda: p.engine.rollout_cost(p._xf, 0, q0, (20, 3, 80), pt, qt, cost4=cost4),
                                reps=7)
    res["local_topk_ms"] = ev_time(lambda: topk(p.engine, cost4, E, stride=4, out=p._idx))
    gathered = torch.rand(G * E, device=p.device)
    sel = torch.empty(E, dtype=torch.int32, device=p.device)
    res["global_topk_ms"] = ev_time(lambda: topk(p.engine, gathered, E, stride=1, out=sel))
    m0, c0 = p._mean.clone(), p._cov.clone()

    def upd():
        p._mean.copy_(m0)
        p._cov.copy_(c0)
        p.cem.update(p._xs, cost4, 4, p._idx, 10.0, 0.6, 0.6, p._mean, p._cov)
    res["update_ms_incl_2_copies"] = ev_time(upd)
    res["allgather_bytes"] = G * E * (p.nvar + 1) * 4
    plant = Plant(p.model)
    qp = plant.qpos.copy()
    qp[:6] = q0
    plant.set_state(qpos=qp)
    plant.forward()
    v = np.zeros(6)
    import time
    ts = []
    for _ in range(12):
        t0 = time.perf_counter()
        plant.step(v)  # blocks until done (mpcr_plant_step)
        ts.append(1e3 * (time.perf_counter() - t0))
    res["plant_step_ms_wall"] = float(np.median(ts[2:]))
    it = (res["factor_ms"] + res["sample_project_ms"] + res["rollout_ms"] + res["local_topk_ms"] +
          res["global_topk_ms"] + res["update_ms_incl_2_copies"])
    res["iteration_device_ms"] = round(it, 3)
    res["tick_device_ms"] = round(3 * it + res["plant_step_ms_wall"], 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

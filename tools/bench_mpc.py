"""C5-style closed-loop benchmark: receding-horizon MPC ticks of the drop-in
planner (SBP/mpc_planner.py:151-233 loop body, headless) with the CEM
iterations of every tick replayed from HIP graphs.

    python tools/bench_mpc.py [--model dual_arm] [--n 8192] [--H 50] [--iters 3] [--ticks 30]
    torchrun --nproc-per-node G tools/bench_mpc.py ...   (candidates sharded, num_batch global)

Per tick: compute_cem (graph replay of every iteration: factor, sample +
project, rollout + cost, top-E, moments; the 9-tuple copied to the host)
+ the plant step on the GPU + the host bookkeeping of the reference loop.
Reports the median tick (graph) next to the same loop with eager launches.
Prints one JSON line (rank 0).  Diagnostic, not the bench.py contract.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(model, n, H, iters, ticks, graph, device, group):
    from manipulator_mujoco_amd.engine import Plant
    from manipulator_mujoco_amd.planner import cem_planner
    p = cem_planner(num_dof=6, num_batch=n, num_steps=H, timestep=0.05, maxiter_cem=iters, num_elite=0.05,
                    w_pos=20.0, w_rot=3.0, w_col=80.0, maxiter_projection=10, model_path=model, device=device,
                    graph=graph, group=group, return_rollouts=False, verbose=False)
    plant = Plant(p.model, device=device)
    qpos = plant.qpos.copy()
    qpos[:6] = [1.5, -1.8, 1.75, -1.25, -1.6, 0.0]
    plant.set_state(qpos=qpos)
    plant.forward()
    pt, qt = np.array([-0.3, -0.3, 0.5]), np.array([0.0, 1.0, 0.0, 0.0])
    xi_mean = np.zeros(p.nvar)
    ts, dist = [], []
    for k in range(ticks + 2):  # 2 warm-up ticks (graph capture happens in the first)
        t0 = time.perf_counter()
        out = p.compute_cem(xi_mean, plant.qpos[:6], plant.qvel[:6], plant.qacc[:6], pt, qt)
        xi_mean = out[6]
        plant.step(np.mean(out[4][1:H - 2], axis=0))
        if k >= 2:
            ts.append((time.perf_counter() - t0) * 1e3)
            dist.append(float(np.linalg.norm(plant.site_xpos_tcp - pt)))
    return ts, dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="dual_arm")
    ap.add_argument("--n", type=int, default=8192, help="global candidates per CEM iteration")
    ap.add_argument("--H", type=int, default=50)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--ticks", type=int, default=30)
    ap.add_argument("--no-eager", action="store_true")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    group = None
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        group = dist.group.WORLD
    res = {"model": args.model, "candidates": args.n, "horizon": args.H, "cem_iters": args.iters,
           "ticks": args.ticks, "ranks": world}
    ts, d = run(args.model, args.n, args.H, args.iters, args.ticks, True, local, group)
    res["tick_ms_graph"] = round(float(np.median(ts)), 3)
    res["rollouts_per_s_graph"] = round(args.n * args.iters / (np.median(ts) * 1e-3), 1)
    res["eef_dist_first_last"] = [round(d[0], 4), round(d[-1], 4)]
    if not args.no_eager:
        te, _ = run(args.model, args.n, args.H, args.iters, args.ticks, False, local, group)
        res["tick_ms_eager"] = round(float(np.median(te)), 3)
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

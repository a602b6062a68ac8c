"""Benchmark: candidate rollouts/s of the fused HIP hot path (basis -> H
MuJoCo-semantics steps -> cost -> best) on 1..8 MI355X, one process per GPU.

Workload (BASELINE.json configs[2], the largest single-GPU config, named in
the metric "UR5e scene"): URD/scene_mjx.xml (UR5e + Hand-E + object.xml free
box resting on the table), 4096 candidates x 50 steps per GPU (weak scaling:
N x 4096 candidates in total), order-10 Bernstein, dt = 0.05, Newton solver.
A step = one rollout_cost launch over the rank's batch (inputs resident in
HBM, theta/thetadot/cost4 written back like the reference's outputs) + the
global best-candidate selection (fused atomic-min key; for N > 1 one 8-byte
RCCL MIN all-reduce).  Synthetic inputs: xi ~ N(0, 10.003 I) (seed
20250629 + 3 + rank), projected with 10 ADMM iterations before timing.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "candidate rollouts/sec (N×H steps) UR5e scene, 1/2/4/8 MI355X"
Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
W = (20.0, 3.0, 80.0)
PT = (-0.3, -0.3, 0.5)
QT = (0.0, 1.0, 0.0, 0.0)
PEAK_F32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = f32-MFMA dense peak
PEAK_HBM_GBS = 8000.0

# BASELINE.json configs; c3 is the metric's workload (default)
CONFIGS = {
    "c2": dict(model="ur5e_hande_mjx", n=1024, H=50,
               desc="URD/ur5e_1_robotiq_hande_mjx.xml arm alone, Newton(1 it, 5 ls)"),
    "c3": dict(model="scene_mjx", n=4096, H=50,
               desc="UR5e+Hand-E arm + object.xml box (URD/scene_mjx.xml), Newton(1 it, 5 ls)"),
    "c4": dict(model="dual_arm", n=4096, H=100,
               desc="dual-arm gripper scene (implicitfast, 14 actuators, connect equalities, convex-hull "
                    "meshes), Newton(100 it, 50 ls); C4 = 8 GPUs x 4096"),
}


def flops_per_step(m, nefc_mean, ncon_pairs=None):
    fm = json.load(open(os.path.join(ROOT, "bench", "flops_model.json")))
    nb_moving = int(sum(1 for b in range(1, m.nbody) if m.body_weldid[b] != 0))
    names = {0: "plane_capsule", 1: "plane_box", 2: "capsule_capsule", 3: "capsule_box", 4: "box_box", 9: "convex",
             10: "plane_convex"}
    coll = sum(fm["collision_per_pair"][names[int(f)]] for f in m.pair_func)
    sp = fm["solve_per_row"]
    nv = m.nv
    solve = fm["solve_base"] + nefc_mean * (sp["row_setup"] + sp["jacobian_per_dof"] * nv
                                            + sp["hessian_per_dof2"] * nv * nv + sp["matvec_per_dof"] * nv
                                            + sp["linesearch"])
    f = (fm["basis_per_coeff"] * m.nctrl * 11 + fm["kinematics_per_moving_body"] * nb_moving
         + fm["dynamics_per_dof"] * nv + coll + solve + fm["cost_base"] + fm["cost_per_slot"] * m.nslot)
    return float(f)


def pmc_traffic(path, kernel="rollout_kernel"):
    """HBM bytes per dispatch from a committed rocprofv3 --pmc CSV (FETCH_SIZE
    doubled per the gfx950 note in MI355X_MICROARCH.md §HBM, plus WRITE_SIZE)."""
    import csv
    if not os.path.exists(path):
        return None
    fetch, write = [], []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            name = row.get("Counter_Name", "")
            val = float(row.get("Counter_Value", 0))
            if name == "FETCH_SIZE":
                fetch.append(val)
            elif name == "WRITE_SIZE":
                write.append(val)
    if not fetch and not write:
        return None
    kb = 2.0 * (np.mean(fetch) if fetch else 0.0) + (np.mean(write) if write else 0.0)
    return kb * 1024.0


def cpu_baseline(m, xi, H, Pd, workers):
    """fp64 scalar C oracle on host cores over a bounded sample of the same workload."""
    import oracle
    from concurrent.futures import ProcessPoolExecutor
    oracle.build()
    n = xi.shape[0]
    td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
    chunks = np.array_split(np.arange(n), workers)
    t0 = time.perf_counter()
    if workers == 1:
        oracle.rollout(m, td, Q0, np.array(W), np.array(PT), np.array(QT), want_theta=False)
    else:
        with ProcessPoolExecutor(workers) as ex:
            list(ex.map(_oracle_chunk, [(td[c], m.bundle_name) for c in chunks]))
    return n / (time.perf_counter() - t0)


def _oracle_chunk(args):
    import oracle
    from manipulator_mujoco_amd import models
    td, name = args
    m = models.load(name, 0.05)
    oracle.rollout(m, td, Q0, np.array(W), np.array(PT), np.array(QT), want_theta=False)
    return td.shape[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3",
                    help="BASELINE.json config preset (c3 = the metric's workload, the default)")
    ap.add_argument("--n", type=int, default=None, help="candidates per GPU (default: the config's)")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--model", default=None)
    ap.add_argument("--cpu-sample", type=int, default=4096)
    ap.add_argument("--cpu-workers", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default=None,
                    help="rocprofv3 --pmc CSV of this workload (default: the committed C3 one for c3, else none)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    args.model = args.model or cfg["model"]
    args.n = args.n or cfg["n"]
    args.horizon = args.horizon or cfg["H"]

    import torch
    import torch.distributed as dist

    from manipulator_mujoco_amd import basis, models
    from manipulator_mujoco_amd import dist as md
    from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine
    from manipulator_mujoco_amd.projection import ProjectionFilter

    rank, world, local = md.env_rank()
    if world == 1 and args.gpus > 1:
        raise SystemExit("launch N>1 with torch.distributed.run (one process per GPU)")

    H, n = args.horizon, args.n
    m = models.load(args.model, 0.05)
    m.bundle_name = args.model
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    # synthetic inputs, generated on the host (same bytes on every run)
    rng = np.random.default_rng(20250629 + 3 + rank)
    cpu = torch.device("cpu")
    proj = ProjectionFilter(P, Pd, Pdd, 6, cpu)
    xi_host = proj(torch.tensor(rng.normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)),
                   proj.boundary(Q0, np.zeros(6), np.zeros(6), n), 10)
    cpu_rec = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # host-core baseline first: its worker processes are forked before
        # this process initialises the GPU
        workers = args.cpu_workers or min(16, os.cpu_count() or 1)
        sample = xi_host[: args.cpu_sample].numpy()
        v1 = cpu_baseline(m, sample[: max(64, args.cpu_sample // 16)], H, Pd, 1)
        vp = cpu_baseline(m, sample, H, Pd, workers)
        cpu_rec = {"value": round(vp, 1), "unit": "rollouts/s", "cores": workers, "kind": "port",
                   "sample": f"{sample.shape[0]} of the same {args.config.upper()} candidates x {H} steps, fp64 "
                             f"scalar C oracle "
                             f"(oracle/mpcr_oracle.c), {workers} processes; 1 core: {v1:.1f} rollouts/s",
                   "one_core": round(v1, 1)}

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    xi = xi_host.to(dev)
    eng = Engine(m, H, n, Pd, device=local)
    cost4 = torch.empty((n, 4), dtype=torch.float32, device=dev)
    theta = torch.empty((n, 6 * H), dtype=torch.float32, device=dev)
    thetadot = torch.empty((n, 6 * H), dtype=torch.float32, device=dev)
    key = torch.empty(1, dtype=torch.int64, device=dev)
    status = torch.zeros(n, dtype=torch.int32, device=dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        eng.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, cost4=cost4, theta=theta, thetadot=thetadot,
                         best_key=key, index_base=rank * n, status=status)
        if ev is not None:
            ev[1].record()
        if world > 1:
            md.allreduce_min_key(key)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    idx, best = md.decode_key(int(key.item()))
    trunc = int((status & 1).sum().item())
    nefc_mean = float((status >> 8).double().mean().item()) / H

    if rank == 0:
        total = n * world
        value = total * args.steps / elapsed
        # algorithmic work of the dominant kernel per launch
        fps = flops_per_step(m, nefc_mean)  # mean constraint rows/step measured by the kernel
        flops_launch = fps * H * n
        achieved_tf = flops_launch / (kern_ms * 1e-3) / 1e12
        hbm_launch = n * (66 * 4 + 16 + 2 * 6 * H * 4 + 4)  # xi in; cost4, theta, thetadot, status out
        pmc = args.pmc or (os.path.join(ROOT, "profiles", "r01_pmc_rollout.csv") if args.config == "c3" else None)
        traffic = pmc_traffic(pmc) if pmc else None
        rec = {
            "metric": METRIC, "value": round(value, 1), "unit": "rollouts/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (xi ~ N(0, 10.003 I), 10-iteration ADMM projection; seed 20250629+3+rank)",
            "config": {"workload": f"{args.config.upper()} {args.model}: {cfg['desc']}, {n} candidates x {H} "
                                   f"steps per GPU, order-10 Bernstein, dt 0.05",
                       "candidates_per_gpu": n, "horizon": H, "global_batch": total,
                       "parallelism": f"dp{world} (candidate shards, 8-byte RCCL MIN all-reduce)"},
            "roofline": {"bound": "mfma", "achieved": round(achieved_tf, 3), "peak": PEAK_F32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_F32_TFLOPS, 5),
                         "traffic": None if traffic is None else round(traffic),
                         "kernel": "rollout_kernel", "kernel_ms": round(kern_ms, 4),
                         "flops_per_step": fps, "hbm_algorithmic_bytes": hbm_launch,
                         "hbm_achieved_GBs": round(hbm_launch / (kern_ms * 1e-3) / 1e9, 2),
                         "hbm_frac": round(hbm_launch / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 6)},
            "best": {"index": idx, "cost": best}, "truncated_candidates": trunc,
            "mean_constraint_rows": round(nefc_mean, 2),
        }
        if cpu_rec is not None:
            rec["cpu_baseline"] = cpu_rec
        print(json.dumps(rec))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

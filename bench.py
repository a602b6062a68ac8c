"""Benchmark: candidate rollouts/s of the fused HIP hot path (basis -> H
MuJoCo-semantics steps -> cost -> best) on 1..8 MI355X, one process per GPU.

Workload (BASELINE.json configs[2], the largest single-GPU config, named in
the metric "UR5e scene"): URD/scene_mjx.xml (UR5e + Hand-E + object.xml free
box resting on the table), 4096 candidates x 50 steps per GPU, order-10
Bernstein, dt = 0.05, Newton solver.  A step = one rollout_cost launch over
the rank's batch (inputs resident in HBM, theta/thetadot/cost4 written back
like the reference's outputs) + the global selection: the fused atomic-min
best key (N > 1: one 8-byte RCCL MIN all-reduce) or, with --exchange elite
(the C4 default), the sharded CEM's elite exchange as well (local top-E,
RCCL all-gather of (xi row, cost), global top-E).  Synthetic inputs:
xi ~ N(0, 10.003 I) (seed 20250629 + 3 + shard), projected with 10 ADMM
iterations before timing.

Scaling: --scaling weak (default): every rank owns --n candidates (N x 4096
in total); --scaling strong: --n is the global batch, split over the ranks
(C3's 4096 x 50 on 1..8 GPUs).  The default line (C3, weak) also carries two
sub-records measured by the same ranks in the same run: "strong" (C3's 4096
x 50 global batch split over the ranks) and "c5" (BASELINE configs[4]: the
closed-loop dual-arm MPC tick, 3 CEM iterations over a global 8192 x 50 batch
split over the ranks, graph replay) -- the strong-scaling curves beside the
weak one.  --config c5 makes the C5 tick the line itself.

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4|c5] [--scaling strong] [--no-sub]
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
PEAK_F32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector (FMA) peak
PEAK_HBM_GBS = 8000.0
PROFILE_TAG = "r06j"  # the final round-6 build (source 77733f95)

# BASELINE.json configs; c3 is the metric's workload (default)
CONFIGS = {
    "c2": dict(model="ur5e_hande_mjx", n=1024, H=50, exchange="key",
               desc="URD/ur5e_1_robotiq_hande_mjx.xml arm alone, Newton(1 it, 5 ls)"),
    "c3": dict(model="scene_mjx", n=4096, H=50, exchange="key",
               desc="UR5e+Hand-E arm + object.xml box (URD/scene_mjx.xml), Newton(1 it, 5 ls)"),
    "c4": dict(model="dual_arm", n=4096, H=100, exchange="elite",
               desc="dual-arm gripper scene (implicitfast, 14 actuators, connect equalities, convex-hull "
                    "meshes), Newton(100 it, 50 ls); C4 = 8 GPUs x 4096, elite exchange per step"),
    # C5: a closed-loop MPC tick = compute_cem (3 CEM iterations over the GLOBAL
    # 8192-candidate batch split over the ranks, graph replay) + the plant step
    "c5": dict(model="dual_arm", n=8192, H=50, exchange="elite", iters=3,
               desc="closed-loop receding-horizon MPC tick on the dual-arm scene: compute_cem with 3 CEM "
                    "iterations (factor, MVN sample + projection, rollout + cost, elites, mean/cov) over a "
                    "global 8192-candidate batch split over the ranks, HIP-graph replay, + the plant step"),
}


def flops_per_step(m, nefc_mean, model_name=None):
    fm = json.load(open(os.path.join(ROOT, "bench", "flops_model.json")))
    nb_moving = int(sum(1 for b in range(1, m.nbody) if m.body_weldid[b] != 0))
    names = {0: "plane_capsule", 1: "plane_box", 2: "capsule_capsule", 3: "capsule_box", 4: "box_box", 9: "convex_cull",
             10: "plane_convex"}
    nex = fm.get("narrow_executed_per_step", {}).get(model_name) if model_name else None
    if nex:  # executed primitive narrow-phase calls only (culled pairs are not credited)
        coll = sum(fm["collision_per_pair"][k] * v for k, v in nex.items())
        coll += sum(fm["collision_per_pair"][names[int(f)]] for f in m.pair_func if names[int(f)] not in nex)
    else:
        coll = sum(fm["collision_per_pair"][names[int(f)]] for f in m.pair_func)
    ex = fm["convex_executed_per_step"].get(model_name) if model_name else None
    if ex:  # executed MPR solves and polyhedron manifolds only (culled pairs are not credited)
        coll += ex["mpr_calls"] * fm["collision_per_pair"]["convex"] + ex["hits"] * fm["poly_manifold_per_hit"]
    sp = fm["solve_per_row"]
    nv = m.nv
    solve = fm["solve_base"] + nefc_mean * (sp["row_setup"] + sp["jacobian_per_dof"] * nv
                                            + sp["hessian_per_dof2"] * nv * nv + sp["matvec_per_dof"] * nv
                                            + sp["linesearch"])
    f = (fm["basis_per_coeff"] * m.nctrl * 11 + fm["kinematics_per_moving_body"] * nb_moving
         + fm["dynamics_per_dof"] * nv + coll + solve + fm["cost_base"] + fm["cost_per_slot"] * m.nslot)
    return float(f)


def _pmc_rows(path, kernel="rollout_kernel"):
    import csv
    out = {}
    if not path or not os.path.exists(path):
        return out
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            out.setdefault(row.get("Counter_Name", ""), []).append(float(row.get("Counter_Value", 0)))
    return out


def pmc_traffic(path, dispatches=1):
    """HBM bytes per rollout call from a committed rocprofv3 --pmc CSV
    (FETCH_SIZE doubled per the gfx950 note in MI355X_MICROARCH.md §HBM, plus
    WRITE_SIZE; both KiB): the mean per dispatch times the call's dispatches
    (Engine.dispatches: the dual-arm shard runs as horizon segments)."""
    c = _pmc_rows(path)
    if "FETCH_SIZE" not in c and "WRITE_SIZE" not in c:
        return None
    kb = 2.0 * float(np.mean(c.get("FETCH_SIZE", [0.0]))) + float(np.mean(c.get("WRITE_SIZE", [0.0])))
    return kb * 1024.0 * dispatches


def pmc_valu(path, n, H, flops_step, dispatches=1):
    """VALU instructions per candidate-step (over all of a candidate's waves:
    the two-wave variant runs two, a segmented call one per segment) and the
    lane-flop efficiency flops / (64 x VALU instructions) from a committed SQ
    counter CSV of the same workload (per-dispatch means times the call's
    dispatches)."""
    c = _pmc_rows(path)
    if "SQ_INSTS_VALU" not in c:
        return None
    insts = float(np.mean(c["SQ_INSTS_VALU"])) * dispatches
    wpd = float(np.mean(c.get("SQ_WAVES", [n])))
    per = insts / (n * H)
    #  waves per candidate *per call* summed over a segmented
    # call's dispatches (a 7-step segment is one wave per candidate), and the
    # waves of one dispatch, reported apart: round 4's "waves_per_candidate"
    # meant the former for segmented calls and waves per candidate otherwise
    rec = {"valu_insts_per_candidate_step": round(per, 1), "waves_per_candidate_per_call": round(wpd * dispatches / n, 2),
           "waves_per_dispatch": round(wpd, 1), "dispatches_per_call": dispatches,
           "lane_flop_efficiency": round(flops_step / (64.0 * per), 4), "source": os.path.relpath(path, ROOT)}
    if "SQ_ACTIVE_INST_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        # SQ_ACTIVE_INST_VALU counts quad-cycles; GRBM_GUI_ACTIVE is summed over
        # the 8 XCDs (MI355X_MICROARCH.md); 1024 SIMDs
        busy = (4.0 * float(np.mean(c["SQ_ACTIVE_INST_VALU"])) / 1024.0
                / (float(np.mean(c["GRBM_GUI_ACTIVE"])) / 8.0))
        rec["valu_busy"] = round(busy, 3)
    return rec


def _cgroup_cpus():
    """The cgroup v2 CPU quota in CPUs (cpu.max "quota period"), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def _host_cpu():
    """(usable host cores, machine cpu count, model name, affinity cores, cgroup
    quota).  Usable = the CPUs this process may run on AND the cgroup lets it
    use: the GPU box's affinity mask shows the whole machine (256) while its
    cgroup quota is the box's share."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = _cgroup_cpus()
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return usable, os.cpu_count() or 1, model, aff, quota


EXACT_MPR = 4  # oracle/mpcr_oracle.c: ccd_tolerance exact; Newton / line-search floors as in the kernel


def cpu_baseline(m, xi, H, Pd, threads, reps=5, precision="fp32"):
    """The scalar C oracle (oracle/mpcr_oracle.c, a restatement of the
    reference's rollout + cost, SBP/mjx_planner.py:123-124; precision "fp32"
    = oracle_f32.c, every double as float, the reference's own precision) on
    host threads: pool started and model converted before the clock; median
    of `reps` timed repetitions of the rollout compute only.  The fp32 build
    runs the kernel's stop rules (EXACT_MPR only: the fp32 Newton /
    line-search floors), the fp64 build MuJoCo's.  Returns rollouts/s."""
    import oracle
    oracle.build()
    n = xi.shape[0]
    td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
    run = oracle.Runner(m, threads, Q0, W, PT, QT, precision=precision,
                        exact_mask=EXACT_MPR if precision == "fp32" else None)
    run.rollout(td[: max(1, min(n, threads))])  # warm-up (page in, first-touch)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run.rollout(td)
        ts.append(time.perf_counter() - t0)
    run.close()
    return n / float(np.median(ts)), [round(n / t, 1) for t in ts]


def _free_port():
    """A free port below the ephemeral range (32768..), where no client
    socket of the ranks can take it before rank 0's rendezvous binds it."""
    import random
    import socket
    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
        return p
    raise RuntimeError("no free port in 20000..32000")


def launch_ranks(nproc, argv, grace_s=30.0):
    """`python bench.py --gpus N` outside torch.distributed.run: start N fresh
    child processes of this script, one per GPU (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT in their environment), and return
    the worst child's exit code.  Called before anything imports torch, so the
    parent never touches the GPU; the children inherit stdout, and rank 0's
    JSON line is the run's output.  When a rank fails, the others get
    `grace_s` seconds to end on their own (a collective's error reaches them)
    and are then killed by PID."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   GROUP_RANK="0", MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    deadline = None
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        if deadline is None and any(rc not in (None, 0) for rc in rcs):
            deadline = time.monotonic() + grace_s
        if deadline is not None and time.monotonic() > deadline:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.05)
    # a signal death (negative returncode) maps to the shell's 128 + signal
    codes = [rc if rc >= 0 else 128 - rc for rc in (p.returncode for p in procs)]
    return max(codes)


def launch_selftest():
    """--launch-selftest: the spawn path's plumbing without a GPU (CPU test,
    tests/test_bench_launch.py): each rank joins a gloo group and all-reduces;
    rank 0 prints one JSON line; MPCR_SELFTEST_FAIL_RANK=r makes rank r exit 3."""
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    if os.environ.get("MPCR_SELFTEST_FAIL_RANK") == str(rank):
        sys.exit(3)
    dist.init_process_group("gloo")
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}
    if rank == 0:
        print(json.dumps({"world": world, "sum_ranks_plus_1": int(t.item()), "env": env}))
    dist.destroy_process_group()


def committed_counters(kind, sfx):
    """A committed rocprof counter CSV (profiles/<tag>_pmc_<kind><sfx>.csv) and
    its provenance, attached only when the profile manifest
    (profiles/<tag>_pmc_manifest.json) records the same libmpcr.so source hash
    as this checkout -- a profile of an earlier build is not this run's."""
    from manipulator_mujoco_amd import build as b
    path = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_pmc_{kind}{sfx}.csv")
    man = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_pmc_manifest.json")
    if not (os.path.exists(path) and os.path.exists(man)):
        return None, None
    rec = json.load(open(man)).get(os.path.basename(path))
    if not rec or rec.get("source_hash") != b.source_hash():
        return None, "stale (profile of another build, not attached)"
    return path, "committed 1-GPU profile of this build (" + os.path.relpath(path, ROOT) + ")"


def synthetic_xi(n, H, seed):
    """The bench's synthetic candidates: xi ~ N(0, 10.003 I), 10-iteration ADMM
    projection (host, before any timing)."""
    import torch

    from manipulator_mujoco_amd import basis
    from manipulator_mujoco_amd.projection import ProjectionFilter
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    proj = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
    rng = np.random.default_rng(seed)
    return proj(torch.tensor(rng.normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)),
                proj.boundary(Q0, np.zeros(6), np.zeros(6), n), 10)


def _timed(step, steps, warmup, world, dev):
    """warmup untimed steps, then `steps` timed between barrier + synchronize
    on both sides; (wall seconds, median per-step ms of the HIP events) as the
    max over ranks."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kms = [a.elapsed_time(b) for a, b in events]
    t = torch.tensor([elapsed, float(np.median(kms))], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(t[1]), kms


def strong_subrecord(eng, dev, rank, world, H, steps, warmup, n_global=4096):
    """C3's fixed global batch (4096 x 50, BASELINE configs[2]) split over the
    ranks in the same run: the strong-scaling reading of
    the multi-GPU line beside its weak one.  Same candidates as
    `--scaling strong` (the global draw, this rank's rows), selection by the
    8-byte MIN all-reduce of the best key."""
    import torch

    from manipulator_mujoco_amd import dist as md
    from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI
    lo, hi = md.shard(n_global, rank, world)
    n = hi - lo
    xi = synthetic_xi(n_global, H, 20250629 + 3)[lo:hi].contiguous().to(dev)
    cost4 = torch.empty((n, 4), dtype=torch.float32, device=dev)
    theta = torch.empty((n, 6 * H), dtype=torch.float32, device=dev)
    thetadot = torch.empty((n, 6 * H), dtype=torch.float32, device=dev)
    key = torch.empty(1, dtype=torch.int64, device=dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        eng.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, cost4=cost4, theta=theta, thetadot=thetadot,
                         best_key=key, index_base=lo)
        if ev is not None:
            ev[1].record()
        if world > 1:
            md.allreduce_min_key(key)

    elapsed, kern_ms, _ = _timed(step, steps, warmup, world, dev)
    idx, best = md.decode_key(int(key.item()))
    return {"scaling": "strong", "workload": f"C3 scene_mjx, {n_global} candidates x {H} steps in total, split "
                                             f"over {world} GPU(s)",
            "global_batch": n_global, "candidates_per_gpu": n, "steps": steps, "warmup": warmup,
            "value": round(n_global * steps / elapsed, 1), "unit": "rollouts/s",
            "ms_per_step": round(1e3 * elapsed / steps, 4), "kernel_ms": round(kern_ms, 4),
            "best": {"index": idx, "cost": best}}


def c5_run(rank, world, gpu, dev, n_global, H, iters, ticks, warmup, capture_exchange):
    """C5 (BASELINE configs[4]): closed-loop MPC ticks on the dual-arm scene.
    A tick = compute_cem (SBP/mjx_planner.py:364-406: `iters` CEM iterations
    over the global batch, each rank its n_global / world share, sampling
    keyed by the global index, elites exchanged; the iterations replayed from
    HIP graphs) + the plant step with the mean of best_vels[1:H-2]
    (SBP/mpc_planner.py:151-233, headless).  Returns the timing and, for the
    roofline, the rollout call timed eagerly on the last tick's samples."""
    import torch
    import torch.distributed as dist

    from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Plant
    from manipulator_mujoco_amd.planner import cem_planner
    p = cem_planner(num_dof=6, num_batch=n_global, num_steps=H, timestep=0.05, maxiter_cem=iters, num_elite=0.05,
                    w_pos=W[0], w_rot=W[1], w_col=W[2], maxiter_projection=10, model_path="dual_arm", device=gpu,
                    graph=True, group=dist.group.WORLD if world > 1 else None, return_rollouts=False,
                    capture_exchange=capture_exchange, verbose=False)
    plant = Plant(p.model, device=gpu)
    qpos = plant.qpos.copy()
    qpos[:6] = Q0
    plant.set_state(qpos=qpos)
    plant.forward()
    state = {"mean": np.zeros(p.nvar), "out": None}

    def tick(ev=None):
        if ev is not None:
            ev[0].record()
        out = p.compute_cem(state["mean"], plant.qpos[:6], plant.qvel[:6], plant.qacc[:6], PT, QT)
        state["mean"] = out[6]
        plant.step(np.mean(out[4][1:H - 2], axis=0))
        if ev is not None:
            ev[1].record()
        state["out"] = out

    elapsed, tick_ms, tick_each = _timed(tick, ticks, warmup, world, dev)
    # the dominant kernel: the rank's rollout call on the last iteration's
    # samples, eagerly, HIP events on its stream (graph replays cannot be split)
    n = p.n_local
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    kms = []
    for k in range(ticks + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        p.engine.rollout_cost_dp(p._xf, MPCR_LAYOUT_XI, p._par, p._costs[0], theta=p._theta[0],
                                 thetadot=p._thetadot[0], index_base=p.index_base, status=st)
        b.record()
        torch.cuda.synchronize()
        if k:
            kms.append(a.elapsed_time(b))
    out = state["out"]
    nefc_mean = float((st >> 11).double().mean().item()) / H
    return {"elapsed": elapsed, "tick_ms": tick_ms, "tick_ms_each": [round(x, 3) for x in tick_each],
            "kernel_ms": float(np.median(kms)), "n_local": n,
            "nefc_mean": nefc_mean, "model": p.model, "engine": p.engine,
            "best_cost": [float(x) for x in np.asarray(out[0])],
            "best_cost_grc": [float(out[1]), float(out[2]), float(out[3])],
            "eef_dist": float(np.linalg.norm(plant.site_xpos_tcp - np.asarray(PT))),
            "capture": "the whole tick, RCCL all-gathers included" if (world > 1 and capture_exchange and
                                                                        dist.get_backend() == "nccl")
            else ("each CEM iteration's device segment; the elite exchange eager between replays" if world > 1
                  else "the whole tick (one rank: no exchange)")}


def c5_subrecord(rank, world, gpu, dev, steps, warmup):
    """C5 beside the default line: the global 8192 x 50 x 3
    tick over however many ranks this run has -- the strong-scaling curve the
    north star's ">= 6x further at 8 GPUs" is about.  The exchange runs
    eagerly between graph replays here (the RCCL-captured tick is
    `--config c5 --c5-capture-exchange`)."""
    cfg = CONFIGS["c5"]
    r = c5_run(rank, world, gpu, dev, cfg["n"], cfg["H"], cfg["iters"], steps, warmup, capture_exchange=False)
    return {"scaling": "strong", "workload": f"C5 dual_arm closed-loop tick: {cfg['iters']} CEM iterations over "
                                             f"{cfg['n']} candidates x {cfg['H']} steps in total, split over "
                                             f"{world} GPU(s), + the plant step",
            "global_batch": cfg["n"], "candidates_per_gpu": r["n_local"], "ticks": steps, "warmup": warmup,
            "value": round(cfg["n"] * cfg["iters"] * steps / r["elapsed"], 1), "unit": "rollouts/s",
            "ms_per_tick": round(1e3 * r["elapsed"] / steps, 3), "rollout_kernel_ms": round(r["kernel_ms"], 3),
            "best_cost": r["best_cost"], "graph": r["capture"]}


def init_device(args, world, local):
    """This rank's GPU (local rank; with --backend gloo ranks may share one)
    and, for world > 1, the process group."""
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > 1 and local >= ndev:
        raise SystemExit(f"local rank {local} has no GPU of its own ({ndev} visible); use --backend gloo to share")
    gpu = local % max(ndev, 1)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    backend = None
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        backend = dist.get_backend()
    return gpu, dev, ndev, backend


def main_c5(args, cfg):
    """--config c5: the closed-loop tick as the line (strong scaling: the
    global batch is fixed, split over the ranks)."""
    import torch.distributed as dist

    from manipulator_mujoco_amd import basis, models
    from manipulator_mujoco_amd import dist as md
    rank, world, local = md.env_rank()
    n_global, H, iters = args.n or cfg["n"], args.horizon or cfg["H"], cfg["iters"]
    cpu_rec = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the scalar C restatement on host cores, a bounded sample of the
        # workload's rollouts (the dual arm is ~100x C3's CPU cost per rollout)
        usable, ncpu, model, aff, quota = _host_cpu()
        threads = args.cpu_threads or usable
        sample = synthetic_xi(args.cpu_sample or 256, H, 20250629 + 5).numpy()
        m = models.load(cfg["model"], 0.05)
        _, _, Pd, _ = basis.planner_basis(H, 0.05)
        v32, reps = cpu_baseline(m, sample, H, Pd, threads, reps=3, precision="fp32")
        cpu_rec = {"value": round(v32, 1), "unit": "rollouts/s", "cores": threads, "kind": "port",
                   "sample": f"{sample.shape[0]} dual-arm candidates x {H} steps (rollout + cost only, no CEM "
                             f"step); fp32 scalar C restatement (oracle/oracle_f32.c), {threads} threads, median "
                             f"of {len(reps)} repetitions",
                   "reps": reps, "host": {"usable_cores": usable, "affinity_cores": aff, "cgroup_cpu_quota": quota,
                                          "nproc": ncpu, "cpu_model": model}}
    gpu, dev, ndev, backend = init_device(args, world, local)
    r = c5_run(rank, world, gpu, dev, n_global, H, iters, args.steps, args.warmup, args.c5_capture_exchange)
    if rank == 0:
        coll = {"nccl": "RCCL (xGMI)", "gloo": "gloo (host-staged)"}.get(backend, str(backend))
        fps = flops_per_step(r["model"], r["nefc_mean"], "dual_arm")
        achieved_tf = fps * H * r["n_local"] / (r["kernel_ms"] * 1e-3) / 1e12
        hbm_launch = r["n_local"] * (66 * 4 + 16 + 2 * 6 * H * 4 + 4)
        rec = {
            "metric": METRIC, "value": round(n_global * iters * args.steps / r["elapsed"], 1), "unit": "rollouts/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * r["elapsed"] / args.steps, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic closed loop (CEM from a zero mean, Philox samples keyed by the global candidate "
                    "index; target (-0.3, -0.3, 0.5), qt (0, 1, 0, 0))",
            "config": {"workload": f"C5 {cfg['model']}: {cfg['desc']}; {n_global} x {H} x {iters} per tick",
                       "global_batch": n_global, "candidates_per_gpu": r["n_local"], "horizon": H, "cem_iters": iters,
                       "parallelism": f"dp{world} (candidate shards; elite exchange)", "world_size_seen": world,
                       "backend": backend or "single process", "gpus_visible": ndev,
                       "graph": r["capture"],
                       "exchange": "none (one rank)" if world == 1 else
                       f"local top-E + {coll} all-gather of (xi, cost) rows + global top-E per iteration; "
                       f"best key MIN all-reduce + broadcast of the best row per tick"},
            "roofline": {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": PEAK_F32_VALU_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_F32_VALU_TFLOPS, 5), "traffic": None,
                         "traffic_source": "not profiled in this run", "kernel": "rollout_kernel",
                         "kernel_ms": round(r["kernel_ms"], 4),
                         "kernel_timing": "the rank's rollout call on the last tick's samples, eager, HIP events "
                                          "(graph replays are timed whole)",
                         "flops_per_step": fps, "hbm_algorithmic_bytes": hbm_launch},
            "best": {"cost_per_iteration": r["best_cost"], "cost_grc": r["best_cost_grc"]},
            "eef_dist_after": r["eef_dist"], "mean_constraint_rows": round(r["nefc_mean"], 2),
            "ticks": {"timed": args.steps, "warmup": args.warmup, "ms_each": r["tick_ms_each"],
                      "note": "consecutive closed-loop ticks: each starts from the plant state the previous left"},
        }
        if cpu_rec is not None:
            rec["cpu_baseline"] = cpu_rec
        print(json.dumps(rec))
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ticks", type=int, default=None,
                    help="--config c5: closed-loop ticks timed (BASELINE configs[4] runs 30); overrides --steps")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3",
                    help="BASELINE.json config preset (c3 = the metric's workload, the default)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: --n candidates per GPU; strong: --n candidates in total, split over the GPUs")
    ap.add_argument("--exchange", choices=("key", "elite"), default=None,
                    help="per-step selection: best-key MIN all-reduce, or also the CEM elite exchange")
    # --candidates: torch.distributed.run's argparse takes a bare "--n" after the
    # script name for an abbreviation of its own options
    ap.add_argument("--candidates", "--n", dest="n", type=int, default=None,
                    help="candidates (per GPU for weak, total for strong)")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--model", default=None)
    ap.add_argument("--cpu-sample", type=int, default=0, help="candidates timed on the host (0 = the whole batch)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every usable host core (affinity mask capped by the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-contact-report", action="store_true")
    ap.add_argument("--pmc", default=None, help="rocprofv3 FETCH/WRITE CSV of this workload")
    ap.add_argument("--pmc-sq", default=None, help="rocprofv3 SQ counter CSV of this workload")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="N > 1: nccl (= RCCL over xGMI, one GPU per rank) or gloo (host-staged; ranks may share "
                         "a GPU, device = local rank mod the visible GPUs: rehearses the multi-rank path on one GPU)")
    ap.add_argument("--no-sub", action="store_true",
                    help="default line only: skip the strong (C3 4096 global) and C5 sub-records")
    ap.add_argument("--c5-capture-exchange", action="store_true",
                    help="c5: capture the RCCL elite all-gathers in the tick's graph (default: eager between replays)")
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # not under torch.distributed.run: one fresh process per GPU, spawned
        # before this process imports torch (it never initialises the GPU)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launch_selftest:
        return launch_selftest()
    cfg = CONFIGS[args.config]
    if args.config == "c5":
        if args.ticks:
            args.steps = args.ticks
        return main_c5(args, cfg)
    args.model = args.model or cfg["model"]
    args.n = args.n or cfg["n"]
    args.horizon = args.horizon or cfg["H"]
    args.exchange = args.exchange or cfg["exchange"]

    import torch
    import torch.distributed as dist

    from manipulator_mujoco_amd import basis, models
    from manipulator_mujoco_amd import dist as md
    from manipulator_mujoco_amd.cem import topk
    from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine

    rank, world, local = md.env_rank()

    H = args.horizon
    if args.scaling == "strong":
        lo, hi = md.shard(args.n, rank, world)
        n, n_total, base = hi - lo, args.n, lo
    else:
        n, n_total, base = args.n, args.n * world, rank * args.n
    m = models.load(args.model, 0.05)
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    # synthetic inputs, generated on the host (same bytes on every run); strong
    # scaling draws the global batch and takes this rank's rows
    n_draw = n_total if args.scaling == "strong" else n
    xi_all = synthetic_xi(n_draw, H, 20250629 + 3 + (0 if args.scaling == "strong" else rank))
    xi_host = xi_all[base:base + n] if args.scaling == "strong" else xi_all
    cpu_rec = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # host-core baseline before the process initialises the GPU
        usable, ncpu, model, aff, quota = _host_cpu()
        threads = args.cpu_threads or usable
        sample = xi_host[: args.cpu_sample or n].numpy()
        one = sample[: max(32, sample.shape[0] // 16)]
        v32, reps = cpu_baseline(m, sample, H, Pd, threads, precision="fp32")
        v32_1, _ = cpu_baseline(m, one, H, Pd, 1, precision="fp32")
        v64, reps64 = cpu_baseline(m, sample, H, Pd, threads, precision="fp64")
        v64_1, _ = cpu_baseline(m, one, H, Pd, 1, precision="fp64")
        # the affinity mask may show more CPUs than the cgroup quota grants (the
        # GPU box: 256 vs 16): one run with a thread per affinity CPU shows
        # the quota binding (not the reported value)
        v32_aff = None
        if aff > threads and not args.cpu_threads:
            v32_aff, _ = cpu_baseline(m, sample, H, Pd, aff, reps=3, precision="fp32")
        cpu_rec = {"value": round(v32, 1), "unit": "rollouts/s", "cores": threads, "kind": "port",
                   "sample": f"{sample.shape[0]} of the same {args.config.upper()} candidates x {H} steps; fp32 "
                             f"scalar C restatement of the reference rollout + cost (oracle/oracle_f32.c = "
                             f"oracle/mpcr_oracle.c in float, not CPU-MJX), {threads} threads = every usable core "
                             f"(affinity {aff}, cgroup quota {quota}), median of {len(reps)} timed repetitions "
                             f"(pool and model set up before the clock); 1 thread: {v32_1:.1f} rollouts/s; fp64 "
                             f"build: {v64:.1f} ({threads} threads), {v64_1:.1f} (1 thread)",
                   "precision": "fp32", "one_core": round(v32_1, 1), "reps": reps,
                   "stop_rules": "fp32: the kernel's (ccd_tolerance 1e-6, fp32 Newton / line-search floors); "
                                 "fp64: MuJoCo's (ccd_tolerance 1e-6, scale*dcost < tol, no bracket floor)",
                   "affinity_threads": None if v32_aff is None else {"threads": aff, "value": round(v32_aff, 1)},
                   "fp64": {"value": round(v64, 1), "one_core": round(v64_1, 1), "reps": reps64},
                   "host": {"usable_cores": usable, "affinity_cores": aff, "cgroup_cpu_quota": quota, "nproc": ncpu,
                            "cpu_model": model}}

    gpu, dev, ndev, backend = init_device(args, world, local)
    xi = xi_host.to(dev)
    eng = Engine(m, H, n, Pd, device=gpu)
    cost4 = torch.empty((n, 4), dtype=torch.float32, device=dev)
    theta = torch.empty((n, 6 * H), dtype=torch.float32, device=dev)
    thetadot = torch.empty((n, 6 * H), dtype=torch.float32, device=dev)
    key = torch.empty(1, dtype=torch.int64, device=dev)
    status = torch.zeros(n, dtype=torch.int32, device=dev)
    n_elite = int(0.05 * n_total)
    topk_fn = (lambda c, k: topk(eng, c, k))

    elites = {}

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        eng.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, cost4=cost4, theta=theta, thetadot=thetadot,
                         best_key=key, index_base=base, status=status)
        if ev is not None:
            ev[1].record()
        if args.exchange == "elite":
            c = cost4[:, 0].contiguous()
            if world > 1:
                g_cost, _, sel = md.gather_elites(c, xi, n_elite, topk_fn)
                elites["cost"] = g_cost.index_select(0, sel.long())
            else:
                elites["cost"] = c.index_select(0, topk_fn(c, n_elite).long())
            elites["count"] = elites.get("count", 0) + 1
        if world > 1:
            md.allreduce_min_key(key)

    for _ in range(args.warmup):
        step()
    elites["count"] = 0
    elapsed, kern_ms, kms = _timed(step, args.steps, 0, world, dev)
    idx, best = md.decode_key(int(key.item()))
    trunc = int((status & 1).sum().item())
    nefc_mean = float((status >> 11).double().mean().item()) / H

    contact = None
    if rank == 0 and not args.no_contact_report and m.nslot:
        # SURVEY §8d asks whether contacts activate (C2 "no contacts"): the
        # masked robot slots of this batch, traced outside the timed region
        tr = eng.trace(xi_host.numpy(), MPCR_LAYOUT_XI, Q0, W, PT, QT)
        act = (tr["slots"] < 0).any(axis=2)
        first = np.where(act.any(axis=1), act.argmax(axis=1), -1)
        contact = {"candidates_with_active_robot_contact": int(act.any(axis=1).sum()), "of": int(n),
                   "first_active_step_median": float(np.median(first[first >= 0])) if (first >= 0).any() else None}

    # the default line (C3, weak) also carries the strong-scaling reading of
    # the same ranks and the C5 tick
    subs = {}
    if args.config == "c3" and args.scaling == "weak" and args.n == cfg["n"] and not args.no_sub:
        subs["strong"] = strong_subrecord(eng, dev, rank, world, H, args.steps, args.warmup)
        subs["c5"] = c5_subrecord(rank, world, gpu, dev, min(args.steps, 5), 2)

    if rank == 0:
        coll = {"nccl": "RCCL (xGMI)", "gloo": "gloo (host-staged)"}.get(backend, str(backend))
        value = n_total * args.steps / elapsed
        fps = flops_per_step(m, nefc_mean, args.model)  # mean constraint rows/step measured by the kernel
        flops_launch = fps * H * n
        achieved_tf = flops_launch / (kern_ms * 1e-3) / 1e12
        hbm_launch = n * (66 * 4 + 16 + 2 * 6 * H * 4 + 4)  # xi in; cost4, theta, thetadot, status out
        # counters: the CSVs passed explicitly (--pmc / --pmc-sq, a profile of
        # this command), else the committed 1-GPU passes of this exact workload
        # (the config's own batch, weak mode, one rank) when they were taken
        # from this build: C3 <tag>_pmc_rollout.csv / _sq.csv, the other
        # configs the same names suffixed _c2 / _c4.  A multi-rank line gets
        # none: no rank of it was profiled.
        default_prof = args.n == cfg["n"] and args.scaling == "weak" and world == 1
        sfx = "" if args.config == "c3" else "_" + args.config
        pmc, pmc_src = (args.pmc, "--pmc " + args.pmc) if args.pmc else (
            committed_counters("rollout", sfx) if default_prof else (None, None))
        pmc_sq, sq_src = (args.pmc_sq, "--pmc-sq " + args.pmc_sq) if args.pmc_sq else (
            committed_counters("sq", sfx) if default_prof else (None, None))
        ndisp = eng.dispatches(n)  # kernel dispatches per rollout call (horizon segments)
        traffic = pmc_traffic(pmc, ndisp) if pmc else None
        valu = pmc_valu(pmc_sq, n, H, fps, ndisp) if pmc_sq else None
        if valu is not None:
            valu["source"] = sq_src
        rec = {
            "metric": METRIC, "value": round(value, 1), "unit": "rollouts/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (xi ~ N(0, 10.003 I), 10-iteration ADMM projection; seed 20250629+3"
                    + ("" if args.scaling == "strong" else "+rank") + ")",
            "config": {"workload": f"{args.config.upper()} {args.model}: {cfg['desc']}, {n} candidates x {H} "
                                   f"steps per GPU, order-10 Bernstein, dt 0.05",
                       "candidates_per_gpu": n, "horizon": H, "global_batch": n_total,
                       "parallelism": f"dp{world} (candidate shards; {args.exchange} exchange)",
                       "world_size_seen": world, "backend": backend or "single process",
                       "gpus_visible": ndev,
                       "launcher": ("torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ
                                    else "bench.py self-launch" if world > 1 else "single process"),
                       "exchange": ("none (one rank: the fused atomic-min key is the global best"
                                    + ("; the local top-E is the global top-E)" if args.exchange == "elite" else ")")
                                    if world == 1 else f"8-byte {coll} MIN all-reduce of the best key" + (
                                        f"; local top-E + {coll} all-gather of (xi, cost) rows + global top-E"
                                        if args.exchange == "elite" else ""))},
            "roofline": {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": PEAK_F32_VALU_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_F32_VALU_TFLOPS, 5),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": pmc_src if traffic is not None else pmc_src or "not profiled in this run",
                         "kernel": "rollout_kernel", "dispatches_per_call": ndisp, "kernel_ms": round(kern_ms, 4),
                         "kernel_ms_mean": round(float(np.mean(kms)), 4),
                         "flops_per_step": fps, "hbm_algorithmic_bytes": hbm_launch,
                         "hbm_achieved_GBs": round(hbm_launch / (kern_ms * 1e-3) / 1e9, 2),
                         "hbm_frac": round(hbm_launch / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 6)},
            "best": {"index": idx, "cost": best}, "truncated_candidates": trunc,
            "mean_constraint_rows": round(nefc_mean, 2),
        }
        if traffic is not None:
            rec["roofline"]["traffic_over_algorithmic"] = round(traffic / hbm_launch, 3)
        if "cost" in elites:
            ec = elites["cost"].double().cpu().numpy()
            # the global top-E of the last timed step: equal to one GPU's on the
            # same global batch (tests/test_gpu_bench.py)
            rec["elites"] = {"k": n_elite, "exchanges_timed": elites["count"], "cost_sum": float(ec.sum()),
                             "first": [float(x) for x in ec[:4]]}
        if valu is not None:
            rec["roofline"]["valu"] = valu
        if contact is not None:
            rec["contacts"] = contact
        if cpu_rec is not None:
            rec["cpu_baseline"] = cpu_rec
        rec.update(subs)
        print(json.dumps(rec))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

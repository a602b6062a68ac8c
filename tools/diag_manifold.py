"""Diagnostic: the plane-mesh manifold on a dual-arm candidate whose large
hulls touch the table (candidate 2989 of the seed-20250632 C4 batch; 2986,
the slowest before the wave-cooperative manifold, until round 4's capsule-box
rule changed its trajectory).  Plant (GPU, wide kernel) vs
oracle, re-synced to the oracle's fp64 state every step: active contacts of
the plane-mesh pairs and qacc."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import Plant  # noqa: E402
from manipulator_mujoco_amd.projection import ProjectionFilter  # noqa: E402


def candidate_td(idx, H=100, n=4096, seed=20250632):
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    proj = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    raw = np.random.default_rng(seed).normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)[idx:idx + 1]
    xi = proj(torch.tensor(raw), proj.boundary(q0, np.zeros(6), np.zeros(6), 1), 10).numpy()
    return q0, np.einsum("tk,jk->jt", Pd.astype(np.float32), xi.reshape(6, 11)).astype(np.float64)


def run(idx=2989, H=100):
    m = models.load("dual_arm", 0.05)
    q0, td = candidate_td(idx, H)
    big = {g for g in range(m.ngeom) if int(m.geom_type[g]) == 7 and int(m.geom_hullnum[g]) >= 600}
    mesh_pairs = {p for p in range(m.npair) if int(m.pair_func[p]) == 10 and int(m.pair_geom2[p]) in big}
    qpos = m.qpos_init[:m.nq].copy()
    qpos[np.asarray(m.ctrl_qposadr[:m.nctrl])] = q0
    qvel, ws = m.qvel_init[:m.nv].copy(), np.zeros(m.nv)
    plant = Plant(m)
    rows = []
    for t in range(H):
        qv = qvel.copy()
        qv[np.asarray(m.ctrl_dofadr[:m.nctrl])] = td[:, t]
        plant.set_state(qpos=qpos, qvel=qv, qacc_warmstart=ws)
        kd = plant.step_debug(td[:, t])
        o = oracle.step(m, qpos, qv, ws)
        scale = max(1.0, np.abs(o["qacc"]).max())
        kp = sorted((int(p), tuple(np.round(x, 4))) for p, x in zip(kd["con_pair"], kd["con_pos"]) if p in mesh_pairs)
        row = dict(t=t)
        # the fp64 oracle, and the fp32 build as the second reference (probe F):
        # a flush mesh-mesh contact (the gripper linkage) can take MPR's other
        # portal under fp32 rounding, the fp32 oracle the same way as the kernel
        for tag, prec in (("", "fp64"), ("_f32", "fp32")):
            od = oracle.step_debug(m, qpos, qv, ws, precision=prec)
            op = sorted((int(p), tuple(np.round(x, 4))) for p, x in zip(od["con_pair"], od["con_pos"]) if p in mesh_pairs)
            row["n_mesh" + tag] = len(op)
            row["same" + tag] = len(kp) == len(op) and all(
                a[0] == b[0] and np.abs(np.array(a[1]) - np.array(b[1])).max() <= 2e-4 for a, b in zip(kp, op))
            row["qacc_err" + tag] = float(np.abs(plant.qacc - od["qacc"]).max() / scale)
        rows.append(row)
        qpos, qvel, ws = o["qpos"], o["qvel"], o["qacc_warmstart"]
    return rows, sorted(big), sorted(mesh_pairs)


if __name__ == "__main__":
    rows, big, pairs = run(int(sys.argv[1]) if len(sys.argv) > 1 else 2989)
    act = [r for r in rows if r["n_mesh"] > 0]
    best = [min(r["qacc_err"], r["qacc_err_f32"]) for r in rows]
    print(f"big hulls {big}, their plane pairs {pairs}; steps with big-hull plane contacts {len(act)}, "
          f"max contacts {max([r['n_mesh'] for r in act], default=0)}, identical contact sets "
          f"{sum(r['same'] for r in act)}/{len(act)} (fp32 oracle {sum(r['same_f32'] for r in act)}); "
          f"max qacc err/scale {max(r['qacc_err'] for r in rows):.2e} vs fp64, {max(best):.2e} vs the nearer, "
          f"median {np.median(best):.2e}")
    for r in rows:
        if r["qacc_err"] > 5e-3 or (r["n_mesh"] and not r["same"]):
            print("  differs:", r)

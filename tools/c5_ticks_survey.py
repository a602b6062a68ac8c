"""How often does a closed-loop tick select a candidate the fp64 oracle
prices differently?  (diagnostic; the 30-tick test checks one trajectory)

Runs the C5 loop (8192 x 50 x 3 CEM iterations per tick on the dual arm,
graph-replayed, the plant stepping the applied velocities) for each planner
seed -- a different Philox key, so a different trajectory -- and checks
every tick's selected candidate (its best_vels from the tick's start) against
the fp64 oracle: a miss is rel >= max(1e-4, 2 x probe-A sensitivity, as the
test), and a miss is fp32-conditioned when the fp32 restatement
(oracle_f32.c, the kernel's stop rules) misses too.

    python tools/c5_ticks_survey.py [seeds=0,1,2,3] [ticks=30]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402,F401

import oracle  # noqa: E402
import parity_util as pu  # noqa: E402
from manipulator_mujoco_amd.engine import Plant  # noqa: E402
from manipulator_mujoco_amd.planner import cem_planner  # noqa: E402

kw = dict(a.split("=") for a in sys.argv[1:])
seeds = [int(s) for s in kw.get("seeds", "0,1,2,3").split(",")]
ticks, n, H = int(kw.get("ticks", 30)), 8192, 50
PT, QT, Q0 = pu.PT, pu.QT, pu.Q0
tot = dict(ticks=0, miss=0, f32=0)
for seed in seeds:
    p = cem_planner(num_dof=6, num_batch=n, num_steps=H, timestep=0.05, maxiter_cem=3, num_elite=0.05, w_pos=20.0,
                    w_rot=3.0, w_col=80.0, maxiter_projection=10, verbose=False, model_path="dual_arm", graph=True,
                    seed=seed)
    m = p.model
    plant = Plant(m)
    qpos = plant.qpos.copy()
    qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
    qpos[qa] = Q0
    plant.set_state(qpos=qpos)
    plant.forward()
    xi_mean, rows = np.zeros(p.nvar), []
    for t in range(ticks):
        q0 = plant.qpos[qa].copy()
        out = p.compute_cem(xi_mean, q0, plant.qvel[da], plant.qacc[da], PT, QT)
        xi_mean = out[6]
        td = np.asarray(out[4], dtype=np.float64).T.reshape(1, 6 * H)
        a = oracle.rollout(m, td, q0, pu.W, PT, QT, want_theta=False)["cost4"][0, 0]
        sens = max(abs(a - oracle.rollout(m, td, q0, pu.W, PT, QT, want_theta=False, noise=1e-6, seed=sd)["cost4"][0, 0])
                   / abs(a) for sd in range(1, 9))
        rel = abs(float(out[0][-1]) - a) / abs(a)
        bar = max(pu.TOL, 2 * sens)
        if rel >= bar:
            r32 = oracle.Runner(m, 1, q0, pu.W, PT, QT, precision="fp32", exact_mask=4)
            c32 = float(r32.rollout(td)[0][0])
            r32.close()
            f32 = abs(c32 - a) / abs(a) >= bar
            rows.append((t, rel, sens, f32))
            if os.environ.get("MPCR_DUMP_DIR"):  # tools/c5_tick_triage.py input
                os.makedirs(os.environ["MPCR_DUMP_DIR"], exist_ok=True)
                np.savez(os.path.join(os.environ["MPCR_DUMP_DIR"], f"c5_seed{seed}_tick{t}.npz"), q0=q0,
                         best_vels=np.asarray(out[4]), gpu_cost=float(out[0][-1]), oracle_cost=a, rel=rel, sens=sens,
                         fp32_cost=c32)
        plant.step(np.mean(out[4][1:H - 2], axis=0))
    nf = sum(r[3] for r in rows)
    tot["ticks"] += ticks
    tot["miss"] += len(rows)
    tot["f32"] += nf
    print(f"seed {seed}: {len(rows)}/{ticks} selected candidates miss the fp64 oracle ({nf} fp32-conditioned): "
          + ", ".join(f"tick {t} {rel:.1e}{' f32' if f else ''}" for t, rel, s, f in rows), flush=True)
    del p, plant
print(f"total: {tot['miss']} of {tot['ticks']} selections miss, {tot['f32']} of them fp32-conditioned "
      f"(the fp32 restatement misses too), {tot['miss'] - tot['f32']} well-conditioned", flush=True)

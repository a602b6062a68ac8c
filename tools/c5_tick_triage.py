"""Triage a closed-loop tick dumped by tests/test_gpu_planner.py
(MPCR_DUMP_DIR): the selected candidate (the tick's start, best_vels)
replayed in fp64 step by step, every step evaluated from the same fp64 state
by the oracle and by the kernel (the plant's step_debug, n = 1, H = 1) --
the outlier step and the contacts that differ there name the mechanism, as
tools/diag_f32.py does for the parity batches (diagnostic).

    python tools/c5_tick_triage.py [--own] build_variants/c5t/c5_tick24.npz [...]

--own: the states are the kernel's own trajectory (the plant stepping the
candidate's velocities in fp32), each evaluated by the oracle from the
plant's state -- for a miss whose fp64 states show no outlier step.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402,F401

import oracle  # noqa: E402
import parity_util as pu  # noqa: E402
from diag_f32 import contact_diffs, pair_kind  # noqa: E402
from manipulator_mujoco_amd import models  # noqa: E402
from manipulator_mujoco_amd.engine import Plant  # noqa: E402

H = 50
m = models.load("dual_arm", 0.05)
plant = Plant(m)
qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
own = "--own" in sys.argv
for f in [a for a in sys.argv[1:] if not a.startswith("--")]:
    d = np.load(f)
    v = np.asarray(d["best_vels"], dtype=np.float32).astype(np.float64).T  # 6 x H
    qpos = np.array(m.qpos_init[:m.nq], dtype=np.float64)
    qpos[qa] = d["q0"]
    qvel = np.array(m.qvel_init[:m.nv], dtype=np.float64)
    ws = np.zeros(m.nv)
    print(f"{os.path.basename(f)}: GPU {float(d['gpu_cost']):.4f} oracle {float(d['oracle_cost']):.4f}", flush=True)
    evals = []
    with oracle.exact(4):
        if own:
            plant.set_state(qpos=qpos, qvel=qvel, qacc_warmstart=ws)
        for t in range(H):
            if own:  # the plant's fp32 state before this step
                qpos, qvel, ws = plant.qpos.copy(), plant.qvel.copy(), plant.qacc.copy()
            qv = qvel.copy()
            qv[da] = v[:, t]
            d64 = oracle.step_debug(m, qpos, qv, ws)
            if f"{os.path.basename(f)}:{t}" in os.environ.get("DUMP_STEPS", "").split(","):
                os.makedirs(os.path.join(ROOT, "gpurun_out", "c5t"), exist_ok=True)
                np.savez(os.path.join(ROOT, "gpurun_out", "c5t", f"state_{os.path.basename(f)[:-4]}_{t}.npz"),
                         qpos=qpos, qvel=qv, ws=ws, v=v[:, t])
            if not own:
                plant.set_state(qpos=qpos, qvel=qv, qacc_warmstart=ws)
            dg = plant.step_debug(v[:, t])
            d32 = oracle.step_debug(m, qpos, qv, ws, precision="fp32")
            scale = max(1.0, np.abs(d64["qacc"]).max())
            eg = np.abs(dg["qacc"] - d64["qacc"]).max() / scale
            e32 = np.abs(d32["qacc"] - d64["qacc"]).max() / scale
            evals.append((t, eg, e32, d64, dg))
            if not own:
                st = oracle.step(m, qpos, qv, ws)
                qpos, qvel, ws = st["qpos"], st["qvel"], st["qacc_warmstart"]
    floor = float(np.median([e[1] for e in evals]))
    for t, eg, e32, d64, dg in evals:
        if eg > max(1e-5, 10 * floor):
            print(f"  step {t}: GPU qacc err {eg:.1e} (fp32 oracle {e32:.1e}, floor {floor:.1e}), ncon {d64['ncon']}/"
                  f"{dg['ncon']}, nefc {d64['nefc']}/{dg['nefc']}, iters {d64['info'][0]:.0f}/{dg['info'][0]:.0f}")
            culprits = contact_diffs(m, d64, dg)
            print("   ->", ", ".join(sorted({pair_kind(m, p) for p in culprits})) or "solver only", flush=True)

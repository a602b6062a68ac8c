"""Where does a candidate's GPU rollout leave the oracle's?  (diagnostic)

For each listed candidate of a projected batch: the fp64 oracle's rollout is
replayed step by step (oracle.step, qvel[:6] overridden as in
SBP/mjx_planner.py:254), and the GPU plant is re-synced to the oracle's state
before every step; the per-step qacc disagreement, the row count and the
active contacts show which step (and which constraint state) breaks parity.

    python tools/diag_parity.py scene_mjx 4096 50 3 188 327 ...
Writes gpurun_out/diag_<model>.json and prints a summary.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import oracle  # noqa: E402
import parity_util as pu  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine, Plant  # noqa: E402
from manipulator_mujoco_amd.projection import ProjectionFilter  # noqa: E402


def main():
    name, n, H, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    cands = [int(x) for x in sys.argv[5:]]
    m = models.load(name, 0.05)
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    f = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cuda:0"))
    rng = np.random.default_rng(20250629 + seed)
    xi = torch.tensor(rng.normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32), device="cuda:0")
    xi = f(xi, f.boundary(pu.Q0, np.zeros(6), np.zeros(6), n), 10).cpu().numpy()[cands]
    k = len(cands)
    td = np.einsum("tk,njk->njt", Pd, xi.reshape(k, 6, 11).astype(np.float64)).reshape(k, 6 * H)
    e = Engine(m, H, k, Pd)
    g = e.trace(xi, MPCR_LAYOUT_XI, pu.Q0, pu.W, pu.PT, pu.QT)
    o = oracle.rollout(m, td, pu.Q0, pu.W, pu.PT, pu.QT, want_slots=m.nslot > 0, want_eef=True)
    qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
    plant = Plant(m)
    out = []
    for j, c in enumerate(cands):
        rec = {"cand": c, "xi": xi[j].tolist(), "cost_gpu": float(g["cost4"][j, 0]), "cost_oracle": float(o["cost4"][j, 0]),
               "parts_gpu": g["cost4"][j].tolist(), "parts_oracle": o["cost4"][j].tolist()}
        th_g, th_o = g["theta"][j].reshape(6, H), o["theta"][j].reshape(6, H)
        dth = np.abs(th_g - th_o).max(axis=0)
        rec["theta_err_by_step"] = dth.tolist()
        rec["first_step_theta_err_gt_1e-5"] = int(np.argmax(dth > 1e-5)) if (dth > 1e-5).any() else -1
        if m.nslot:
            ds = np.abs(g["slots"][j] - o["slots"][j]).max(axis=1)
            rec["slot_err_by_step"] = ds.tolist()
        # oracle replay with per-step re-synced plant
        qpos = np.array(m.qpos_init[:m.nq], dtype=np.float64)
        qpos[qa] = pu.Q0
        qvel = np.array(m.qvel_init[:m.nv], dtype=np.float64)
        ws = np.zeros(m.nv)
        v = td[j].reshape(6, H)
        steps = []
        for t in range(H):
            qv = qvel.copy()
            qv[da] = v[:, t]
            plant.set_state(qpos=qpos, qvel=qv, qacc_warmstart=ws)
            plant.step(v[:, t])
            st = oracle.step(m, qpos, qv, ws)
            # the oracle's own sensitivity to the state rounded to fp32 (what the plant is given)
            r32 = [np.asarray(x, dtype=np.float32).astype(np.float64) for x in (qpos, qv, ws)]
            sr = oracle.step(m, *r32)
            err = np.abs(plant.qacc - st["qacc"])
            scale = max(1.0, np.abs(st["qacc"]).max())
            dd = np.abs(st["dist"][st["dist"] < 1e29])
            steps.append({"t": t, "nefc": int(st["nefc"]), "nefc_r32": int(sr["nefc"]), "qacc_err": float(err.max()),
                          "qacc_err_r32": float(np.abs(sr["qacc"] - st["qacc"]).max()), "qacc_scale": float(scale),
                          "ncon_active": int((st["dist"] < 0).sum()),
                          "near0": float(dd.min()) if len(dd) else 1.0,
                          "min_dist": float(st["dist"].min()) if len(st["dist"]) else 0.0})
            qpos, qvel, ws = st["qpos"], st["qvel"], st["qacc_warmstart"]
        rec["steps"] = steps
        worst = sorted(steps, key=lambda s: -s["qacc_err"] / s["qacc_scale"])[:4]
        # the worst step in detail: contacts that differ between the plant and the oracle
        tw = int(os.environ.get("DIAG_STEP", worst[0]["t"]))  # DIAG_STEP: inspect that step instead
        qpos = np.array(m.qpos_init[:m.nq], dtype=np.float64)
        qpos[qa] = pu.Q0
        qvel = np.array(m.qvel_init[:m.nv], dtype=np.float64)
        ws = np.zeros(m.nv)
        for t in range(tw):
            qv = qvel.copy()
            qv[da] = v[:, t]
            st = oracle.step(m, qpos, qv, ws)
            qpos, qvel, ws = st["qpos"], st["qvel"], st["qacc_warmstart"]
        qv = qvel.copy()
        qv[da] = v[:, tw]
        od = oracle.step_debug(m, qpos, qv, ws)
        plant.set_state(qpos=qpos, qvel=qv, qacc_warmstart=ws)
        gd = plant.step_debug(v[:, tw])
        G = m.names["geom"]
        print(f"  step {tw}: ncon g {gd['ncon']} o {od['ncon']}, solver g {np.round(gd['info'], 4)} o {np.round(od['info'], 4)}")
        for k in range(min(gd["ncon"], od["ncon"])):
            dn = np.abs(gd["con_normal"][k] - od["con_normal"][k]).max()
            dp = np.abs(gd["con_pos"][k] - od["con_pos"][k]).max()
            if dn > 1e-3 or dp > 1e-4 or gd["con_pair"][k] != od["con_pair"][k]:
                p_ = int(od["con_pair"][k])
                print(f"    con {k} pair g{gd['con_pair'][k]} o{p_} ({G[m.pair_geom1[p_]]}:{m.geom_type[m.pair_geom1[p_]]}-"
                      f"{G[m.pair_geom2[p_]]}:{m.geom_type[m.pair_geom2[p_]]} func {m.pair_func[p_]}) "
                      f"d g {gd['con_dist'][k]:.6e} o {od['con_dist'][k]:.6e} n g {np.round(gd['con_normal'][k], 4)} "
                      f"o {np.round(od['con_normal'][k], 4)} pos g {np.round(gd['con_pos'][k], 5)} o {np.round(od['con_pos'][k], 5)}")
        print(f"cand {c}: gpu {rec['cost_gpu']:.6f} oracle {rec['cost_oracle']:.6f} "
              f"parts g{np.round(rec['parts_gpu'], 5)} o{np.round(rec['parts_oracle'], 5)} "
              f"first theta err step {rec['first_step_theta_err_gt_1e-5']}; worst resynced steps "
              + "; ".join(f"t{s['t']} err {s['qacc_err']:.2e}/{s['qacc_scale']:.1f} (r32 {s['qacc_err_r32']:.1e}) "
                          f"nefc {s['nefc']}/{s['nefc_r32']} act {s['ncon_active']} near0 {s['near0']:.1e}"
                          for s in worst))
        out.append(rec)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"diag_{name}.json"), "w") as fh:
        json.dump(out, fh)


if __name__ == "__main__":
    main()

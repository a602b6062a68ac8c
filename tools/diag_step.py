"""Compare one step of the GPU plant with the oracle in detail (diagnostic):
contacts, constraint rows, qacc_smooth, qacc, from the oracle's state at
step T of a candidate recorded by tools/diag_parity.py.

    python tools/diag_step.py scene_mjx 932 31 [H]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
import parity_util as pu  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import Plant  # noqa: E402


def main():
    name, cand, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    H = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    m = models.load(name, 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    rec = [r for r in json.load(open(os.path.join(ROOT, "diag", f"diag_{name}.json"))) if r["cand"] == cand][0]
    xi = np.array(rec["xi"], dtype=np.float32)
    td = np.einsum("tk,jk->jt", Pd, xi.reshape(6, 11).astype(np.float64))
    qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
    qpos = np.array(m.qpos_init[:m.nq], dtype=np.float64)
    qpos[qa] = pu.Q0
    qvel, ws = np.array(m.qvel_init[:m.nv], dtype=np.float64), np.zeros(m.nv)
    for t in range(T):
        qv = qvel.copy()
        qv[da] = td[:, t]
        st = oracle.step(m, qpos, qv, ws)
        qpos, qvel, ws = st["qpos"], st["qvel"], st["qacc_warmstart"]
    qv = qvel.copy()
    qv[da] = td[:, T]
    o = oracle.step_debug(m, qpos, qv, ws)
    plant = Plant(m)
    plant.set_state(qpos=qpos, qvel=qv, qacc_warmstart=ws)
    g = plant.step_debug(td[:, T])
    G = m.names["geom"]
    np.set_printoptions(precision=6, suppress=True, linewidth=160)
    print(f"{name} cand {cand} step {T}: ncon g {g['ncon']} o {o['ncon']}  nefc g {g['nefc']} o {o['nefc']}")
    for k in range(max(g["ncon"], o["ncon"])):
        def fmt(d):
            if k >= len(d["con_pair"]):
                return "-"
            p = d["con_pair"][k]
            return (f"pair {p:3d} {G[m.pair_geom1[p]]}-{G[m.pair_geom2[p]]} d {d['con_dist'][k]: .6e} "
                    f"pos {d['con_pos'][k]} n {d['con_normal'][k]}")
        print(f"  con {k}: g {fmt(g)}\n          o {fmt(o)}")
    n = min(g["nefc"], o["nefc"])
    for key in ("efc_D", "efc_aref", "efc_vel"):
        a, b = g[key][:n], o[key][:n]
        rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-9)
        print(f"  {key}: max rel {rel.max():.2e} at row {int(np.argmax(rel))}  (g {a[np.argmax(rel)]:.6g} o {b[np.argmax(rel)]:.6g})")
    print("  qacc_smooth g", g["qacc_smooth"], "\n              o", o["qacc_smooth"])
    print("  qacc        g", g["qacc"], "\n              o", o["qacc"])
    print("  solver [ws taken, cost ws, cost smooth, p0 cost, alpha, ls passes, bracket best, iters]\n"
          "            g", g["info"], "\n            o", o["info"])
    print("  grad   g", g["grad"], "\n         o", o["grad"])
    print("  search g", g["search"], "\n         o", o["search"])


if __name__ == "__main__":
    main()

"""Quick GPU-vs-oracle parity probe (development aid; tests/ hold the real gates)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_THETADOT, MPCR_LAYOUT_XI, Engine  # noqa: E402

Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
W = np.array([20.0, 3.0, 80.0])
PT = np.array([-0.3, -0.3, 0.5])
QT = np.array([0.0, 1.0, 0.0, 0.0])


def run(name, n, H, layout):
    m = models.load(name, 0.05)
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    rng = np.random.default_rng(0)
    if layout == MPCR_LAYOUT_XI:
        xi = rng.normal(0, 0.05, (n, 6 * 11)).astype(np.float32)
        td = np.einsum("tk,njk->njt", Pd.astype(np.float32), xi.reshape(n, 6, 11)).reshape(n, 6 * H)
        inp = xi
    else:
        t = np.arange(H) * 0.05
        amp = rng.uniform(-0.6, 0.6, (n, 6, 1))
        fr = rng.uniform(0.2, 2.0, (n, 6, 1))
        td = (amp * np.sin(fr * t[None, None, :])).reshape(n, 6 * H).astype(np.float32)
        inp = td
    e = Engine(m, H, n, Pd)
    t0 = time.time()
    g = e.trace(inp, layout, Q0, W, PT, QT)
    t1 = time.time()
    o = oracle.rollout(m, td.astype(np.float64), Q0, W, PT, QT, want_slots=True, want_eef=True)
    t2 = time.time()
    gc, oc = g["cost4"].astype(np.float64), o["cost4"]
    rel = np.abs(gc - oc) / np.maximum(np.abs(oc), 1e-6)
    print(f"== {name} n={n} H={H} layout={layout}: gpu {t1-t0:.3f}s oracle {t2-t1:.3f}s")
    print("  cost rel err: max", rel.max(0), "median", np.median(rel, 0))
    print("  theta max abs err", np.abs(g["theta"] - o["theta"]).max())
    print("  eef max abs err", np.abs(g["eef"] - o["eef"]).max())
    if m.nslot:
        print("  slots max abs err", np.abs(g["slots"] - o["slots"]).max())
    bad = np.argsort(-rel[:, 0])[:3]
    for b in bad:
        print("  worst", b, gc[b], oc[b])
    return rel


if __name__ == "__main__":
    for name in ("planner_scene", "ur5e_hande_mjx", "scene_mjx"):
        run(name, 64, 20, MPCR_LAYOUT_THETADOT)
        run(name, 64, 20, MPCR_LAYOUT_XI)

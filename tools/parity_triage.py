"""Which candidates break the parity bar, and on what?  (diagnostic)

Runs one batch of the GPU parity tests (projected xi, tests/test_gpu_parity.py)
through the kernel trace, measures the oracle's conditioning exactly as
tests/parity_util.py does, and lists the candidates that are
well-conditioned for the total or a component yet miss 1e-4, plus those
whose integer #{c < 0} count differs on a stable candidate.  Saves the GPU
outputs and the oracle's statistics to gpurun_out/triage_<label>.npz and the
candidate indices to gpurun_out/triage_<label>.txt (one line, for
tools/diag_parity.py).

    python tools/parity_triage.py scene_mjx 4096 50 3 [label]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import parity_util as pu  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine  # noqa: E402
from test_gpu_parity import projected_xi  # noqa: E402


def main():
    name, n, H, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    label = sys.argv[5] if len(sys.argv) > 5 else f"{name}_{n}x{H}"
    # ORACLE_EXACT=1: every rule MuJoCo-exact (support tie by mju_sign too);
    # ORACLE_MASK / ORACLE_FLOORS ("newton,band,tie,mpr"): a kernel variant's
    # rules (tools/build_variant.py); default: the oracle's defaults
    import oracle
    mask = 31 if os.environ.get("ORACLE_EXACT") == "1" else int(os.environ.get("ORACLE_MASK", oracle.DEFAULT_EXACT))
    floors = os.environ.get("ORACLE_FLOORS")
    floors = [float(x) for x in floors.split(",")] if floors else None
    m = models.load(name, 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + seed, torch.device("cuda:0")).cpu().numpy()
    e = Engine(m, H, n, Pd)
    g = e.trace(xi, MPCR_LAYOUT_XI, pu.Q0, pu.W, pu.PT, pu.QT)
    td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
    import oracle
    with oracle.exact(mask, floors):
        o, sens = pu.conditioning(m, td)
    g4 = g["cost4"].astype(np.float64)
    graze = pu.grazing(m, o)
    picks = []
    for k, cname in enumerate(pu.COMPONENTS):
        oc = o["cost4"][:, k]
        zero = (oc == 0) & (g4[:, k] == 0)
        rel = np.where(zero, 0, np.abs(g4[:, k] - oc) / np.maximum(np.abs(oc), 1e-12))
        s = np.where(zero, 0, o["sens4"][:, k])
        well = (s < pu.TOL / 10) & ~graze
        bad = np.where(well & (rel >= pu.TOL))[0]
        pb = int((well & (o["probe_b4"][:, k] >= pu.TOL)).sum())
        pf = int((well & (o["probe_f4"][:, k] >= pu.TOL)).sum())
        print(f"{label} {cname}: well {int(well.sum())}, misses {bad.size} (probe B {pb}, F {pf}); worst "
              + ", ".join(f"{i}:{rel[i]:.2e}(sens {s[i]:.1e})" for i in bad[np.argsort(-rel[bad])][:8]))
        picks += [int(i) for i in bad[np.argsort(-rel[bad])][:4]]
    if m.nslot:
        gn = (g["slots"] < 0).sum(axis=(1, 2))
        stable = ~graze & ~o["nneg_unstable"]
        badn = np.where(stable & (gn != o["nneg"]))[0]
        print(f"{label} nneg: stable {int(stable.sum())}, mismatched "
              + ", ".join(f"{i}:{int(gn[i])}/{int(o['nneg'][i])}(sens {sens[i]:.1e})" for i in badn[:8]))
        picks += [int(i) for i in badn[:4]]
    picks = list(dict.fromkeys(picks))[:8]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"triage_{label}.npz"), xi=xi, cost4_gpu=g["cost4"],
                        cost4_oracle=o["cost4"], sens4=o["sens4"], probe_b4=o["probe_b4"], probe_f4=o["probe_f4"],
                        graze=graze,
                        nneg_oracle=o["nneg"], nneg_unstable=o["nneg_unstable"],
                        nneg_gpu=(g["slots"] < 0).sum(axis=(1, 2)) if m.nslot else np.zeros(n, int))
    with open(os.path.join(ROOT, "gpurun_out", f"triage_{label}.txt"), "w") as f:
        f.write(" ".join(str(i) for i in picks) + "\n")
    print(f"{label} picks: {picks}")


if __name__ == "__main__":
    main()

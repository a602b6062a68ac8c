"""Per-step error budget of the kernel against the fp32 restatement (GPU
diagnostic).  For the listed candidates of the GPU-projected batch of
`tools/diag_f32.py --gpu` (the parity tests' inputs), every
step is evaluated from the fp64 oracle's state three ways -- fp64 oracle,
fp32 oracle (oracle_f32.c), the GPU plant -- and the relative errors of
qacc_smooth (dynamics only), the constraint rows (D, aref) and qacc (after
the solver) against fp64 are summarised: which stage carries the GPU's
extra error where the fp32 restatement stays on the fp64 trajectory.

    python tools/step_errors.py dual_arm 4096 100 4 928 3593 3162 ...
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import oracle  # noqa: E402
from diag_f32 import replay  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import Plant  # noqa: E402


def rel(a, b, scale):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / scale) if len(a) else 0.0


def main():
    name, n, H, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    cands = [int(x) for x in sys.argv[5:]]
    m = models.load(name, 0.05)
    from diag_f32 import batch_xi
    xi, Pd = batch_xi(n, H, seed, "cuda:0")  # the GPU-projected batch (as diag_f32 --gpu and the parity tests)
    td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
    plant = Plant(m)
    with oracle.exact(4):
        for c in cands:
            states = replay(m, td[c], H)
            v = td[c].reshape(6, H)
            acc = {k: [] for k in ("qs_gpu", "qs_f32", "qa_gpu", "qa_f32", "D_gpu", "D_f32", "ar_gpu", "ar_f32")}
            for t, (qp, qv, ws) in enumerate(states):
                d64 = oracle.step_debug(m, qp, qv, ws)
                d32 = oracle.step_debug(m, qp, qv, ws, precision="fp32")
                plant.set_state(qpos=qp, qvel=qv, qacc_warmstart=ws)
                dg = plant.step_debug(v[:, t])
                sq = max(1.0, np.abs(d64["qacc_smooth"]).max())
                sa = max(1.0, np.abs(d64["qacc"]).max())
                acc["qs_gpu"].append(rel(dg["qacc_smooth"], d64["qacc_smooth"], sq))
                acc["qs_f32"].append(rel(d32["qacc_smooth"], d64["qacc_smooth"], sq))
                acc["qa_gpu"].append(rel(dg["qacc"], d64["qacc"], sa))
                acc["qa_f32"].append(rel(d32["qacc"], d64["qacc"], sa))
                if dg["nefc"] == d64["nefc"] == d32["nefc"]:
                    nr = d64["nefc"]
                    sD = max(1e-9, np.abs(d64["efc_D"][:nr]).max())
                    sA = max(1e-9, np.abs(d64["efc_aref"][:nr]).max())
                    acc["D_gpu"].append(rel(dg["efc_D"][:nr], d64["efc_D"][:nr], sD))
                    acc["D_f32"].append(rel(d32["efc_D"][:nr], d64["efc_D"][:nr], sD))
                    acc["ar_gpu"].append(rel(dg["efc_aref"][:nr], d64["efc_aref"][:nr], sA))
                    acc["ar_f32"].append(rel(d32["efc_aref"][:nr], d64["efc_aref"][:nr], sA))
            print(f"cand {c}: median / p90 relative error per step (GPU | fp32 oracle): "
                  + "  ".join(f"{k[:-4]} {np.median(acc[k]):.1e}/{np.percentile(acc[k], 90):.1e} | "
                              f"{np.median(acc[k[:-4] + '_f32']):.1e}/{np.percentile(acc[k[:-4] + '_f32'], 90):.1e}"
                              for k in ("qs_gpu", "D_gpu", "ar_gpu", "qa_gpu") if acc[k]))


if __name__ == "__main__":
    main()

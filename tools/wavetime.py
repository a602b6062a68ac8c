"""Diagnostic: per-wave start / end / cycles / hardware slot of the rollout
kernel (-DMPCR_WAVETIME build; never used for timing claims).  Answers how
much of a one-round launch (N = 4096: every candidate resident at once) is
load imbalance across SIMDs and the drain at the end.

    python tools/wavetime.py --build                 # here (CPU container)
    N=4096 python tools/wavetime.py scene_mjx out.json   # on the GPU box
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from manipulator_mujoco_amd import _lib, basis, build, models  # noqa: E402

SO = os.path.join(ROOT, "manipulator_mujoco_amd", "libmpcr_wavetime.so")


def slot_key(w):
    """(xcc, se, sh, cu, simd) from XCC_ID << 32 | HW_ID (gfx9 HW_ID fields)."""
    hw = w & 0xffffffff
    xcc = (w >> 32) & 0xf
    return (int(xcc), int((hw >> 13) & 7), int((hw >> 12) & 1), int((hw >> 8) & 15), int((hw >> 4) & 3))


def main():
    if "--build" in sys.argv:
        build.compile_lib(SO, ["-DMPCR_WAVETIME"])
        print(SO)
        return
    import torch
    torch.cuda.init()  # torch's HIP runtime first: loading libmpcr first would bind both to ROCm's
    _lib.LIB_PATH = SO
    lib = _lib.load()
    vp, P_ = ctypes.c_void_p, ctypes.POINTER
    lib.mpcr_rollout_wavetime.restype = ctypes.c_int
    lib.mpcr_rollout_wavetime.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, P_(ctypes.c_double),
                                          P_(ctypes.c_float), P_(ctypes.c_float), P_(ctypes.c_float), vp]
    import torch
    from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine
    from manipulator_mujoco_amd.projection import ProjectionFilter
    name = sys.argv[1] if len(sys.argv) > 1 else "scene_mjx"
    out = sys.argv[2] if len(sys.argv) > 2 else None
    n, H = int(os.environ.get("N", 4096)), int(os.environ.get("H", 50))
    m = models.load(name, 0.05)
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    proj = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    xi = proj(torch.tensor(np.random.default_rng(20250632).normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)),
              proj.boundary(q0, np.zeros(6), np.zeros(6), n), 10).numpy()
    e = Engine(m, H, n, Pd)
    f = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
    w, pt, qt = np.array([20, 3, 80.]), np.array([-0.3, -0.3, 0.5]), np.array([0, 1, 0, 0.])
    buf = np.zeros((n, 6), np.uint64)  # (n, 4) times / slots, then (n, 2) work counters
    for _ in range(3):  # warm; the last launch is analysed
        _lib.check(lib.mpcr_rollout_wavetime(e.handle, xi.ctypes.data, MPCR_LAYOUT_XI, n,
                                             q0.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), f(w), f(pt), f(qt),
                                             buf.ctypes.data))
    st = torch.zeros(n, dtype=torch.int32, device="cuda")  # per-candidate rows: max (bits 2-9), sum (10-)
    e.rollout_cost(torch.tensor(xi, device="cuda"), MPCR_LAYOUT_XI, q0, w, pt, qt, status=st)
    sv = st.cpu().numpy()
    rows_mean, rows_max = (sv >> 11) / H, (sv >> 2) & 255
    work = buf.reshape(-1)[4 * n:].reshape(n, 2)
    buf = buf.reshape(-1)[:4 * n].reshape(n, 4)
    newton, lsp, cvx = (work[:, 0] & 0xffffffff).astype(float), (work[:, 0] >> 32).astype(float), work[:, 1].astype(float)
    t0, t1, cyc = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64), buf[:, 2].astype(np.float64)
    base = t0.min()
    s, e_ = (t0 - base) * 0.01, (t1 - base) * 0.01  # us (100 MHz)
    dur = e_ - s
    span = e_.max()
    keys = [slot_key(int(v)) for v in buf[:, 3]]
    simds = {}
    for i, k in enumerate(keys):
        simds.setdefault(k, []).append(i)
    per_simd_end = np.array([e_[ix].max() for ix in simds.values()])
    per_simd_cnt = np.array([len(ix) for ix in simds.values()])
    per_simd_cyc = np.array([cyc[ix].sum() for ix in simds.values()])
    done = np.sort(e_)
    res = {
        "model": name, "n": n, "H": H, "span_us": float(span),
        "start_us": {"max": float(s.max()), "p50": float(np.median(s)), "p99": float(np.percentile(s, 99))},
        "wave_us": {"mean": float(dur.mean()), "cv": float(dur.std() / dur.mean()), "p01": float(np.percentile(dur, 1)),
                    "p50": float(np.median(dur)), "p99": float(np.percentile(dur, 99)), "max": float(dur.max())},
        "wave_cycles": {"mean": float(cyc.mean()), "cv": float(cyc.std() / cyc.mean()),
                        "p99": float(np.percentile(cyc, 99)), "max": float(cyc.max())},
        "finished_at_us": {f"p{q}": float(done[min(n - 1, int(q / 100 * n))]) for q in (10, 50, 90, 99)},
        "simds": len(simds), "waves_per_simd": {str(int(c)): int((per_simd_cnt == c).sum())
                                                for c in np.unique(per_simd_cnt)},
        "simd_end_us": {"min": float(per_simd_end.min()), "p50": float(np.median(per_simd_end)),
                        "max": float(per_simd_end.max())},
        "simd_cycles_cv": float(per_simd_cyc.std() / per_simd_cyc.mean()),
        "xccs": sorted({k[0] for k in keys}), "cus": len({k[:4] for k in keys}),
        "work_per_step": {"newton": float(newton.mean() / H), "ls_passes": float(lsp.mean() / H),
                          "convex_chunks": float(cvx.mean() / H)},
        "corr_cycles": {"newton": float(np.corrcoef(cyc, newton)[0, 1]) if newton.std() > 0 else None,
                        "ls_passes": float(np.corrcoef(cyc, lsp)[0, 1]) if lsp.std() > 0 else None,
                        "convex_chunks": float(np.corrcoef(cyc, cvx)[0, 1]) if cvx.std() > 0 else None},
        "slowest": [{"cand": int(i), "Mcycles": round(cyc[i] / 1e6, 1), "newton": int(newton[i]), "ls": int(lsp[i]),
                     "cvx": int(cvx[i])} for i in np.argsort(-cyc)[:6]],
        "corr_cycles_rows": {"mean": float(np.corrcoef(cyc, rows_mean)[0, 1]), "max": float(np.corrcoef(cyc, rows_max)[0, 1])},
        "rows_slowest_vs_all": {"slowest_mean_rows": float(rows_mean[np.argsort(-cyc)[:40]].mean()),
                                "all_mean_rows": float(rows_mean.mean()),
                                "slowest_max_rows": float(rows_max[np.argsort(-cyc)[:40]].mean()),
                                "all_max_rows": float(rows_max.mean())},
        "median_work": {"newton": float(np.median(newton)), "ls": float(np.median(lsp)), "cvx": float(np.median(cvx))},
    }
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)
        np.save(out.replace(".json", ".npy"), np.concatenate([buf, work], axis=1))


if __name__ == "__main__":
    main()

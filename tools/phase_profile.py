"""Diagnostic: per-phase cycle shares of the rollout kernel (s_memtime stamps).
Builds a separate -DMPCR_PROFILE library; never used for timing claims."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from manipulator_mujoco_amd import _lib, basis, build, models  # noqa: E402

PHASES = ["init+basis", "kinematics", "geom/com/eef", "cinert/cdof", "crb/vel/rne", "M/bias", "M solve",
          "coll: box-box", "constraint rows", "newton: line search", "euler", "coll: narrow", "coll: cost+compact",
          "newton: warm start", "newton: factor/solve"]
# slot 7 is the collision loop's tail (box-box moved to 16); 15 packs iteration counts
EXTRA = {29: "newton: jar/cost", 30: "newton: J^T f + grad", 31: "newton: Hessian", 16: "coll: box-box (wave)", 21: "coll: convex narrow (MPR)", 22: "coll: plane-mesh manifold",
         17: "coll: polyhedron manifold", 18: "coll: convex emit"}
COUNTS = {19: "hull-climb rounds (wave level)", 20: "MPR support pairs (wave level)"}


def main():
    so = os.environ.get("PROF_LIB") or os.path.join(ROOT, "manipulator_mujoco_amd", "libmpcr_prof.so")
    if "--build" in sys.argv:  # build here (CPU container), run on the GPU box; --counts: wave-level event counters
        build.compile_lib(so, ["-DMPCR_PROFILE"] + (["-DMPCR_PROFILE_COUNTS"] if "--counts" in sys.argv else []))
        print(so)
        return
    _lib.LIB_PATH = so
    lib = _lib.load()
    lib.mpcr_rollout_profile.restype = ctypes.c_int
    vp, P_ = ctypes.c_void_p, ctypes.POINTER
    lib.mpcr_rollout_profile.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, P_(ctypes.c_double),
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
    if os.environ.get("SUBSET"):  # profile chosen candidates of the batch only (comma-separated indices)
        xi = np.ascontiguousarray(xi[[int(i) for i in os.environ["SUBSET"].split(",")]])
        n = xi.shape[0]
    e = Engine(m, H, n, Pd)
    ph = (ctypes.c_ulonglong * 64)()
    f = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
    w, pt, qt = np.array([20, 3, 80.]), np.array([-0.3, -0.3, 0.5]), np.array([0, 1, 0, 0.])
    for _ in range(2):
        ph = (ctypes.c_ulonglong * 64)()
        _lib.check(lib.mpcr_rollout_profile(e.handle, xi.ctypes.data, MPCR_LAYOUT_XI, n,
                                            q0.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), f(w), f(pt), f(qt), ph))
    waves = [list(ph[:32])] + ([list(ph[32:64])] if any(ph[32:64]) else [])
    names = dict(enumerate(PHASES))
    names[7] = "coll: loop tail"
    names.update(EXTRA)
    res = {"model": name, "n": n, "H": H, "waves_per_candidate": len(waves)}
    for w_i, pw in enumerate(waves):
        # two waves per candidate: wave 0 runs kinematics, dynamics, Newton; wave
        # 1 the collision (and, with coll_rows, the constraint rows); the time a
        # wave waits at a barrier lands in the stamp after it (wave 0: "geom/com/
        # eef" waits for the previous step's collision, "constraint rows" / the
        # rows stamp for this step's; wave 1: "geom/com/eef" for wave 0's
        # Newton + kinematics)
        tot = sum(pw[:15]) + sum(pw[i] for i in EXTRA)
        tag = f" wave {w_i}" if len(waves) > 1 else ""
        print(f"{name}{tag}: n={n} H={H} cycles/wave-step {tot / n / H:.0f}")
        for i, p in names.items():
            if pw[i]:
                print(f"  {p:26s} {pw[i] / n / H:10.0f} cyc  {100 * pw[i] / tot:5.1f}%")
        sub = {23: "support vertices", 24: "cone face scan", 25: "SAT support queries", 26: "incident face + polygons",
               27: "clip", 28: "picks"}
        if any(pw[i] for i in sub):  # inside the polyhedron manifold (wave level, atomics per stamp)
            for i, p in sub.items():
                print(f"    poly: {p:24s} {pw[i] / n / H:10.0f} cyc")
        for i, p in COUNTS.items():
            print(f"  {p:34s} {pw[i] / n / H:8.2f} per wave-step")
        print(f"  Newton iterations per step: {(pw[15] & 0xFFFFFFFF) / n / H:.2f}, line-search passes per step: "
              f"{(pw[15] >> 32) / n / H:.2f} (steps with constraints only)")
        rec = {"cycles_per_wave_step": tot / n / H,
               "phases": {p: {"cycles": pw[i] / n / H, "share": pw[i] / tot} for i, p in names.items()},
               "counts": {p: pw[i] / n / H for i, p in COUNTS.items()},
               "newton_iters_per_step": (pw[15] & 0xFFFFFFFF) / n / H,
               "ls_passes_per_step": (pw[15] >> 32) / n / H}
        if len(waves) == 1:
            res.update(rec)
        else:
            res[f"wave{w_i}"] = rec
    if out:
        import json
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)

if __name__ == "__main__":
    main()

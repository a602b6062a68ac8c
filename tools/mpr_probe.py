"""MPR on one pair in fp64 and emulated fp32 (diagnostic, test infrastructure).

A numpy statement of the oracle's / kernel's Minkowski portal refinement
(oracle/mpcr_oracle.c mpr(), csrc/rollout.hip mpr_lane()) run with every
operation rounded to the chosen dtype, on the geom poses the oracle computes
at a given qpos.  Shows whether fp32 arithmetic alone moves MPR's answer.

    python tools/mpr_probe.py dual_arm <cand> <step> <pair> [H]
(the candidate's state is replayed from diag/diag_<model>.json's xi.)
"""
import ctypes
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

EPS = 1.1920929e-07
TOL = float(os.environ.get("MPR_TOL", "1e-5"))
SUP_TIE = 1e-6
SUP_BAND = float(os.environ.get("SUP_BAND", "1e-6"))


class Geom:
    def __init__(self, m, g, xpos, xmat, dt):
        self.m, self.g, self.dt = m, g, dt
        self.type = int(m.geom_type[g])
        self.size = np.asarray(m.geom_size[g], dtype=dt)
        self.pos = np.asarray(xpos, dtype=dt)
        self.R = np.asarray(xmat, dtype=dt).reshape(3, 3)
        if self.type == 7:
            a, n = int(m.geom_hulladr[g]), int(m.geom_hullnum[g])
            self.verts = np.asarray(m.hull_vert[a:a + n], dtype=dt)
            self.adj = [[int(u) - a for u in m.hull_adj[m.hull_adjadr[v]:m.hull_adjadr[v] + m.hull_adjnum[v]]]
                        for v in range(a, a + n)]
        self.hint = -1

    def support(self, d):
        dt = self.dt
        l = self.R.T @ np.asarray(d, dtype=dt)
        ln = dt(np.sqrt(l @ l))
        p = np.zeros(3, dtype=dt)
        sz = self.size

        def ts(x):
            return dt(0) if abs(x) < SUP_TIE * ln else (dt(1) if x >= 0 else dt(-1))
        if self.type in (2, 3):
            if ln > 0:
                p = sz[0] * l / ln
            if self.type == 3:
                p[2] += ts(l[2]) * sz[1]
        elif self.type == 5:
            r = dt(np.sqrt(l[0] * l[0] + l[1] * l[1]))
            if r > SUP_TIE * ln:
                p[0], p[1] = sz[0] * l[0] / r, sz[0] * l[1] / r
            p[2] = ts(l[2]) * sz[1]
        elif self.type == 6:
            p = np.array([ts(l[k]) * sz[k] for k in range(3)], dtype=dt)
        elif self.type == 7:
            lu = l / ln if ln > 0 else l
            v = self.hint if self.hint >= 0 else 0
            best = self.verts[v] @ lu
            while True:
                nb, bn = v, best + dt(SUP_BAND)
                for u in self.adj[v]:
                    du = self.verts[u] @ lu
                    if du > bn:
                        bn, nb = du + dt(SUP_BAND), u
                if nb == v:
                    break
                best, v = bn - dt(SUP_BAND), nb
            p = self.verts[v].copy()
            self.hint = v
        return self.R @ p + self.pos


def mpr(g1, g2, dt):
    def zero(x):
        return abs(x) < EPS

    def nrm(v):
        n = dt(np.sqrt(v @ v))
        return v / n if n > 0 else v

    hints = []

    def msup(d):
        a, b = g1.support(d), g2.support(-d)
        hints.append((g1.hint, g2.hint))
        return [a - b, a, b]

    def off_plane(x, c):
        return abs(x) >= EPS * np.sqrt(c @ c)

    trace = []
    p = [None] * 4
    p[0] = [g1.pos - g2.pos, g1.pos.copy(), g2.pos.copy()]
    d = nrm(-p[0][0])
    p[1] = msup(d)
    dd = p[1][0] @ d
    if zero(dd) or dd < 0:
        return None, trace
    d = np.cross(p[0][0], p[1][0])
    thr = EPS * (np.sqrt(p[0][0] @ p[0][0]) + np.sqrt(p[1][0] @ p[1][0]))
    if d @ d < thr * thr:
        trace.append("v1 on the v0 ray")
        return ("ray", np.sqrt(p[1][0] @ p[1][0]), nrm(p[1][0])), trace
    d = nrm(d)
    p[2] = msup(d)
    dd = p[2][0] @ d
    if zero(dd) or dd < 0:
        return None, trace
    d = nrm(np.cross(p[1][0] - p[0][0], p[2][0] - p[0][0]))
    if d @ p[0][0] > 0:
        p[1], p[2] = p[2], p[1]
        d = -d
    for guard in range(52):
        p[3] = msup(d)
        dd = p[3][0] @ d
        if zero(dd) or dd < 0:
            return None, trace
        va = np.cross(p[1][0], p[3][0])
        dd = va @ p[0][0]
        if dd < 0 and off_plane(dd, va):
            p[2] = p[3]
            trace.append("disc: v2<-v3")
            d = nrm(np.cross(p[1][0] - p[0][0], p[2][0] - p[0][0]))
            continue
        va = np.cross(p[3][0], p[2][0])
        dd = va @ p[0][0]
        if dd < 0 and off_plane(dd, va):
            p[1] = p[3]
            trace.append("disc: v1<-v3")
            d = nrm(np.cross(p[1][0] - p[0][0], p[2][0] - p[0][0]))
            continue
        break

    def pdir():
        return nrm(np.cross(p[2][0] - p[1][0], p[3][0] - p[1][0]))

    def reach(v4, d):
        d4 = v4[0] @ d
        t = min(d4 - p[1][0] @ d, d4 - p[2][0] @ d, d4 - p[3][0] @ d)
        trace.append(f"gap {float(t):.4e}")
        return t < TOL

    def expand(v4):
        x = np.cross(v4[0], p[0][0])
        if p[1][0] @ x > 0:
            if p[2][0] @ x > 0:
                p[1] = v4
            else:
                p[3] = v4
        else:
            if p[3][0] @ x > 0:
                p[2] = v4
            else:
                p[1] = v4

    it = 0
    while True:
        d = pdir()
        dd = d @ p[1][0]
        if zero(dd) or dd > 0:
            break
        v4 = msup(d)
        dd = v4[0] @ d
        if not (zero(dd) or dd > 0) or reach(v4, d) or it > 50:
            trace.append(f"refine: miss at {it}")
            return None, trace
        expand(v4)
        it += 1
    trace.append(f"refine {it}")
    it = 0
    while True:
        d = pdir()
        v4 = msup(d)
        if reach(v4, d) or it > 50:
            break
        expand(v4)
        it += 1
    trace.append(f"penetration {it}")
    trace.append(f"support hull vertices (local) {hints}")
    for i in range(4):
        trace.append(f"v{i} {np.round(p[i][0].astype(float), 6)}")
    # closest point of the portal triangle to the origin: Ericson 5.1.5 (what
    # the oracle and the kernel do) and the plane projection, for comparison
    a, b, c = p[1][0], p[2][0], p[3][0]
    w = tri_closest(a, b, c, dt)
    n = np.cross(b - a, c - a)
    wp = n * (n @ a) / (n @ n)
    trace.append(f"plane-projection depth {float(np.sqrt(wp @ wp)):.6e}")
    depth = np.sqrt(w @ w)
    return ("hit", depth, w / depth if depth > 0 else w), trace


def tri_closest(a, b, c, dt):
    ab, ac, ap, bp, cp = b - a, c - a, -a, -b, -c
    d1, d2 = ab @ ap, ac @ ap
    if d1 <= 0 and d2 <= 0:
        return a
    d3, d4 = ab @ bp, ac @ bp
    if d3 >= 0 and d4 <= d3:
        return b
    vc = d1 * d4 - d3 * d2
    if vc <= 0 and d1 >= 0 and d3 <= 0:
        return a + (d1 / (d1 - d3)) * ab
    d5, d6 = ab @ cp, ac @ cp
    if d6 >= 0 and d5 <= d6:
        return c
    vb = d5 * d2 - d1 * d6
    if vb <= 0 and d2 >= 0 and d6 <= 0:
        return a + (d2 / (d2 - d6)) * ac
    va = d3 * d6 - d5 * d4
    if va <= 0 and (d4 - d3) >= 0 and (d5 - d6) >= 0:
        return b + ((d4 - d3) / ((d4 - d3) + (d5 - d6))) * (c - b)
    n = np.cross(ab, ac)  # face region: the plane projection (as the oracle and the kernel now do)
    return n * ((n @ a) / (n @ n))


def main():
    name, cand, T, pair = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    H = int(sys.argv[5]) if len(sys.argv) > 5 else 100
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
    s = m.to_struct()
    xp, xm, mo = np.zeros((m.ngeom, 3)), np.zeros((m.ngeom, 9)), np.zeros(8)
    dp = ctypes.POINTER(ctypes.c_double)
    oracle.lib().oracle_geom_poses(ctypes.byref(s), qpos.ctypes.data_as(dp), xp.ctypes.data_as(dp),
                                   xm.ctypes.data_as(dp), pair, mo.ctypes.data_as(dp))
    g1, g2 = int(m.pair_geom1[pair]), int(m.pair_geom2[pair])
    print(f"oracle mpr: hit {mo[0]:.0f} depth {mo[1]:.6e} dir {np.round(mo[2:5], 5)}")
    for dt in (np.float64, np.float32):
        r, tr = mpr(Geom(m, g1, xp[g1], xm[g1], dt), Geom(m, g2, xp[g2], xm[g2], dt), dt)
        print(dt.__name__, "result", None if r is None else (r[0], float(r[1]), np.round(r[2].astype(float), 5)), tr)
    if "--gpu" in sys.argv:  # the kernel's MPR on the same pair, from the plant at this state
        from manipulator_mujoco_amd.engine import Plant
        plant = Plant(m)
        qv = qvel.copy()
        qv[da] = td[:, T]
        plant.set_state(qpos=qpos, qvel=qv, qacc_warmstart=ws)
        tr = plant.step_debug(td[:, T], mpr_pair=pair)["mpr"]
        print(f"kernel mpr: hit {tr[1]:.0f} depth {tr[2]:.6e} dir {np.round(tr[3:6], 5)} pos {np.round(tr[6:9], 5)} "
              f"phases {tr[9:12]}")
        for i in range(4):
            print(f"   v{i} {np.round(tr[12 + 9 * i:15 + 9 * i], 6)}")
        a1, a2 = int(m.geom_hulladr[g1]), int(m.geom_hulladr[g2])
        seq = [(int(tr[48 + 2 * q]) - a1 if m.geom_type[g1] == 7 else -1,
                int(tr[49 + 2 * q]) - a2 if m.geom_type[g2] == 7 else -1) for q in range(32)]
        print(f"   kernel support hull vertices (local) {seq}")
    # sensitivity: fp64 with the poses rounded to fp32
    r, tr = mpr(Geom(m, g1, xp[g1].astype(np.float32), xm[g1].astype(np.float32), np.float64),
                Geom(m, g2, xp[g2].astype(np.float32), xm[g2].astype(np.float32), np.float64), np.float64)
    print("fp64 on fp32-rounded poses", None if r is None else (r[0], float(r[1]), np.round(r[2], 5)), tr)


if __name__ == "__main__":
    main()

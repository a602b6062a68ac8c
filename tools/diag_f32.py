"""Which mechanism moves a well-conditioned candidate?  (diagnostic)

CPU mode (default, no GPU): the fp32 build of the oracle (oracle/oracle_f32.c)
stands in for the kernel's own rounding.  GPU mode (--gpu): the kernel
itself -- the batch of the GPU parity tests (projected on the GPU), costs
from the rollout kernel, per-step evaluations from the plant
(mpcr_plant_step_debug, the same kernel with n = 1, H = 1).

Lists the candidates that probe A calls well-conditioned
(tests/parity_util.py) but whose fp32 / GPU cost misses 1e-4, then replays
each in fp64 step by step and evaluates every step in both precisions from
the same fp64 state: the outlier step (fp32 qacc error far above its
per-step floor and far above what rounding the state moves) and the contacts
that differ there name the mechanism; a tally closes the run.

    python tools/diag_f32.py [--gpu] [model=dual_arm] [n=1024] [H=100] [seed=4] [max_cands=12]
Env ORACLE_MASK: the oracle's EXACT_* mask (default 4 = the kernel's stop rules).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import oracle  # noqa: E402
import parity_util as pu  # noqa: E402
from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.projection import ProjectionFilter  # noqa: E402

TYPES = {0: "plane", 2: "sphere", 3: "capsule", 5: "cylinder", 6: "box", 7: "mesh"}


def batch_xi(n, H, seed, device="cpu"):
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    f = ProjectionFilter(P, Pd, Pdd, 6, torch.device(device))
    rng = np.random.default_rng(20250629 + seed)
    xi = torch.tensor(rng.normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32), device=device)
    return f(xi, f.boundary(pu.Q0, np.zeros(6), np.zeros(6), n), 10).cpu().numpy(), Pd


def batch(m, n, H, seed, device="cpu"):
    xi, Pd = batch_xi(n, H, seed, device)
    return np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)


def pair_name(m, p):
    G = m.names["geom"]
    g1, g2 = int(m.pair_geom1[p]), int(m.pair_geom2[p])
    return (f"{G[g1]}:{TYPES.get(int(m.geom_type[g1]), m.geom_type[g1])}-"
            f"{G[g2]}:{TYPES.get(int(m.geom_type[g2]), m.geom_type[g2])}")


def pair_kind(m, p):
    t1, t2 = int(m.geom_type[m.pair_geom1[p]]), int(m.geom_type[m.pair_geom2[p]])
    return f"{TYPES.get(t1, t1)}-{TYPES.get(t2, t2)}"


def replay(m, td_row, H):
    """fp64 states before every step (qvel[:6] overridden, SBP/mjx_planner.py:254)."""
    qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
    qpos = np.array(m.qpos_init[:m.nq], dtype=np.float64)
    qpos[qa] = pu.Q0
    qvel = np.array(m.qvel_init[:m.nv], dtype=np.float64)
    ws = np.zeros(m.nv)
    v = td_row.reshape(6, H)
    out = []
    for t in range(H):
        qv = qvel.copy()
        qv[da] = v[:, t]
        out.append((qpos.copy(), qv.copy(), ws.copy()))
        st = oracle.step(m, qpos, qv, ws)
        qpos, qvel, ws = st["qpos"], st["qvel"], st["qacc_warmstart"]
    return out


def contact_diffs(m, d64, d32, quiet=False):
    """Pairs whose contacts differ between the two evaluations of one step."""
    p64, p32 = list(d64["con_pair"]), list(d32["con_pair"])
    culprits = set()
    for p in sorted(set(p64) | set(p32)):
        k64 = [k for k in range(len(p64)) if p64[k] == p]
        k32 = [k for k in range(len(p32)) if p32[k] == p]
        if len(k64) != len(k32):
            if not quiet:
                print(f"   pair {p} {pair_name(m, p)} func {m.pair_func[p]}: contacts 64 {len(k64)} 32 {len(k32)} "
                      f"d64 {[round(float(d64['con_dist'][k]), 6) for k in k64]} "
                      f"d32 {[round(float(d32['con_dist'][k]), 6) for k in k32]}")
            culprits.add(p)
            continue
        for k, j in zip(k64, k32):
            dn = np.abs(d64["con_normal"][k] - d32["con_normal"][j]).max()
            dp = np.abs(d64["con_pos"][k] - d32["con_pos"][j]).max()
            dd = abs(d64["con_dist"][k] - d32["con_dist"][j])
            if dn > 1e-4 or dp > 1e-5 or dd > 1e-6:
                if not quiet:
                    print(f"   pair {p} {pair_name(m, p)} func {m.pair_func[p]}: depth {d64['con_dist'][k]:.5f} "
                          f"n64 {np.round(d64['con_normal'][k], 4)} n32 {np.round(d32['con_normal'][j], 4)} "
                          f"dpos {dp:.1e} ddist {dd:.1e}")
                culprits.add(p)
    return culprits


def main():
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    gpu = "--gpu" in sys.argv
    name = a[0] if a else "dual_arm"
    n = int(a[1]) if len(a) > 1 else 1024
    H = int(a[2]) if len(a) > 2 else 100
    seed = int(a[3]) if len(a) > 3 else 4
    maxc = int(a[4]) if len(a) > 4 else 12
    mask = int(os.environ.get("ORACLE_MASK", 4))
    m = models.load(name, 0.05)
    if gpu:
        if os.environ.get("MPCR_LIB"):  # a build variant (tools/build_variant.py)
            from manipulator_mujoco_amd import _lib
            _lib.LIB_PATH = os.path.abspath(os.environ["MPCR_LIB"])
        from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine, Plant
        xi, Pd = batch_xi(n, H, seed, "cuda:0")
        # the GPU-projected batch, for CPU experiments on the very same inputs (--xi)
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.save(os.path.join(ROOT, "gpurun_out", f"xi_{name}_{n}x{H}_s{seed}.npy"), xi)
        td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
        e = Engine(m, H, n, Pd)
        g4 = e.trace(xi, MPCR_LAYOUT_XI, pu.Q0, pu.W, pu.PT, pu.QT)["cost4"].astype(np.float64)
        g = g4[:, 0]
        plant = Plant(m)
        label = "GPU"
    else:
        xs = [x for x in sys.argv if x.startswith("--xi=")]
        if xs:  # a batch saved by a --gpu run (the GPU-projected inputs)
            xi = np.load(xs[0][5:])
            _, _, Pd, _ = basis.planner_basis(H, 0.05)
            td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
        else:
            td = batch(m, n, H, seed)
        label = "fp32 oracle"
    t0 = time.time()
    with oracle.exact(mask):
        o, sens = pu.conditioning(m, td)
    print(f"{name} {n} x {H} seed {seed} mask {mask}: conditioning in {time.time() - t0:.0f} s")
    well = (sens < pu.TOL / 10) & ~pu.grazing(m, o)
    pf, pb = o["probe_f4"][:, 0], o["probe_b"]
    rel = np.abs(g - o["cost4"][:, 0]) / np.abs(o["cost4"][:, 0]) if gpu else pf
    miss = np.where(well & (rel >= pu.TOL))[0]
    print(f"well {int(well.sum())}; probe B well-misses {int((well & (pb >= pu.TOL)).sum())}; "
          f"probe F (fp32 oracle) well-misses {int((well & (pf >= pu.TOL)).sum())}; {label} well-misses {len(miss)}, "
          f"worst {rel[well].max():.2e}")
    order = miss[np.argsort(-rel[miss])]
    cs_ = [x for x in sys.argv if x.startswith("--cand=")]
    if cs_:  # triage these candidates whatever their conditioning
        order = np.array([int(x) for x in cs_[0][7:].split(",")])
        print("chosen candidates:", " ".join(f"{i}: rel {rel[i]:.1e} probe-A {sens[i]:.1e}" for i in order))
    # the fp32 oracle's components on the same inputs (is the GPU nearer the
    # fp32 restatement than the fp64 one?)
    with oracle.exact(mask):
        run = oracle.Runner(m, pu.WORKERS, pu.Q0, pu.W, pu.PT, pu.QT, precision="fp32")
        f4 = run.rollout(td[order]).astype(np.float64) if len(order) else np.zeros((0, 4))
        run.close()
    for k, c in enumerate(order[:maxc]):
        print(f"  cand {c}: (cost, g, r, c) fp64 {np.round(o['cost4'][c], 4)} fp32 oracle {np.round(f4[k], 4)}"
              + (f" GPU {np.round(g4[c], 4)}" if gpu else ""))
    print(f"{label} well-misses (worst first):", " ".join(f"{i}:{rel[i]:.1e}" for i in order))
    tally = {}
    with oracle.exact(mask):
        for c in order[:maxc]:
            states = replay(m, td[c], H)
            v = td[c].reshape(6, H)
            evals = []
            for t, (qp, qv, ws) in enumerate(states):
                d64 = oracle.step_debug(m, qp, qv, ws)
                if gpu:
                    plant.set_state(qpos=qp, qvel=qv, qacc_warmstart=ws)
                    d32 = plant.step_debug(v[:, t])
                else:
                    d32 = oracle.step_debug(m, qp, qv, ws, precision="fp32")
                r32 = [np.asarray(x, dtype=np.float32).astype(np.float64) for x in (qp, qv, ws)]
                dr = oracle.step_debug(m, *r32)
                scale = max(1.0, np.abs(d64["qacc"]).max())
                e32 = np.abs(d32["qacc"] - d64["qacc"]).max() / scale
                er = np.abs(dr["qacc"] - d64["qacc"]).max() / scale
                evals.append((t, e32, er, d64, d32))
            # the outlier step: error far above its per-step floor (the stiff
            # implicit solve leaves ~1e-6 relative on every step) and far above
            # what rounding the state moves
            floor = float(np.median([e_[1] for e_ in evals]))
            cand = [e_ for e_ in evals if e_[1] > max(1e-5, 10 * floor) and e_[1] > 30 * max(e_[2], 1e-8)]
            if not cand:
                print(f"cand {c} ({label} {rel[c]:.1e}): no outlier step (per-step floor {floor:.1e}: accumulated)")
                tally["accumulated"] = tally.get("accumulated", 0) + 1
                continue
            first = cand[0]
            t, e32, er, d64, d32 = max(cand, key=lambda e_: e_[1])
            print(f"cand {c} ({label} {rel[c]:.1e}): worst step {t} qacc err {e32:.1e} (floor {floor:.1e}, state "
                  f"rounding {er:.1e}; {len(cand)} outlier steps, first {first[0]}), ncon 64 {d64['ncon']} "
                  f"32 {d32['ncon']}, nefc {d64['nefc']}/{d32['nefc']}, iters {d64['info'][0]:.0f}/{d32['info'][0]:.0f} "
                  f"ls {d64['info'][5]:.0f}/{d32['info'][5]:.0f}")
            culprits = contact_diffs(m, d64, d32)
            key = ", ".join(sorted({pair_kind(m, p) for p in culprits})) or "solver only"
            tally[key] = tally.get(key, 0) + 1
    print("mechanisms:", tally)


if __name__ == "__main__":
    main()

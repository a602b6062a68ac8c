"""The parity bar shared by the GPU parity tests (not a test module).

North star (BASELINE.json): selected trajectory costs within 1e-4 relative
of the reference on identical samples.  The checker is the fp64 oracle
(oracle/, test infrastructure).  Contact-rich rollouts are not well posed to
1e-4 in fp32: a one-iteration Newton warm-started next to a kink of its
piecewise-quadratic cost, or a masked slot distance next to zero, flips on
the last few bits of the state, and fp32 forward kinematics alone carries
~3e-7 m of position error.  So a fixed "x % of candidates within 1e-4"
would be an assertion about the inputs, not about the kernel.  Instead the
oracle measures every candidate's conditioning: its fp64 cost is recomputed
with the state perturbed after every step by relative noise of fp32 size
(probe A: 1e-7 and 1e-6, seeds 1 and 2; see oracle.rollout(noise=)), and an
independent probe B (1e-6, seed 3) shows how often a candidate that probe A
calls well-conditioned still moves by 1e-4 under fp32-sized noise.  State
noise does not model the rounding inside a step (a stiff contact solve
amplifies it 10-100x beyond the state's own rounding, tools/diag_parity.py),
so probe F runs the same restatement in fp32 (oracle/oracle_f32.c, scalar
and sequential: a different decomposition from the kernel's) and counts
how often fp32 arithmetic alone moves a well-conditioned candidate by 1e-4.
Round 4 traced the dual arm's excess of probe F over probe B to the line
search's fp32 bookkeeping and to MPR-seeded SAT candidates of deep pairs and
fixed both (84 -> 21 on the C4 shard), and compiled the dual-arm kernels
without fast math, which brought the GPU below probe F and inside probe B's
count (C4 shard 8 against probe B's 5 + 3 sigma = 11.7).
Probe F is reported (probe_f_well_miss, well_miss_allowed_with_probe_f),
not allowed.  Then

* well-conditioned candidates (probe A moves the cost < TOL / 10, no masked
  slot within 1e-5 m of zero): the GPU may miss 1e-4 on no more of them
  than probe B does, up to 3 binomial sigma;
* all candidates: no more misses than probe A has against the oracle, up to
  3 binomial sigma + 1 %;
* median error at fp32 level;
* the selection (SBP/mjx_planner.py:395 argmin): the GPU's pick has the
  oracle's minimum cost to within both candidates' conditioning (probes A
  and B), the GPU's
  cost of its pick is within its conditioning of the oracle's, and the
  indices agree unless the oracle's own best two are that close.
"""
import os

import numpy as np

import oracle

TOL = 1e-4  # north star: costs within 1e-4 relative fp32
Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
W = np.array([20.0, 3.0, 80.0])
PT = np.array([-0.3, -0.3, 0.5])
QT = np.array([0.0, 1.0, 0.0, 0.0])
WORKERS = min(16, os.cpu_count() or 1)  # the box's CPU share is 16 per GPU


def oracle_cost(m, td, want_slots=False):
    return oracle.rollout(m, td, Q0, W, PT, QT, want_theta=False, want_slots=want_slots, workers=WORKERS)


def _rel(a, b):
    return np.abs(a - b) / np.maximum(np.abs(a), 1e-12)


def conditioning(m, td, seed=0):
    """(oracle result, per-candidate sensitivity of the total cost under probe
    A).  The result also carries, per cost component (cost, g, r, c: the
    columns of cost4, SBP/mjx_planner.py:300-303), probe A's sensitivity
    ``sens4`` and probe B's relative change ``probe_b4``, and whether any
    probe changed the integer #{c < 0} count (``nneg_unstable``)."""
    o = oracle_cost(m, td, want_slots=m.nslot > 0)
    a = o["cost4"]
    nneg_unstable = np.zeros(len(a), bool)

    def probe(eps, sd):
        r = oracle.rollout(m, td, Q0, W, PT, QT, want_theta=False, workers=WORKERS, noise=eps,
                           seed=1000 * seed + sd)
        nneg_unstable[:] |= r["nneg"] != o["nneg"]
        return _rel(a, r["cost4"])

    s4 = np.maximum.reduce([probe(1e-7, 1), probe(1e-6, 1), probe(1e-6, 2)])
    o["sens4"] = s4
    o["probe_b4"] = probe(1e-6, 3)
    o["probe_b"] = o["probe_b4"][:, 0]
    o["nneg_unstable"] = nneg_unstable
    # probe F: the same restatement computed in fp32 (oracle_f32.c) -- how far
    # fp32 arithmetic alone moves each candidate.  State noise (probes A, B)
    # misses the rounding inside stiff contact solves
    run = oracle.Runner(m, WORKERS, Q0, W, PT, QT, precision="fp32", exact_mask=4)  # the kernel's stop rules
    try:
        o["probe_f4"] = _rel(a, run.rollout(td).astype(np.float64))
    finally:
        run.close()
    return o, s4[:, 0]


def grazing(m, o):
    if not m.nslot:
        return np.zeros(len(o["cost4"]), bool)
    return (np.abs(o["slots"]) < 1e-5).any(axis=(1, 2))


def _sigma3(p, n):
    return 3 * np.sqrt(max(p, 1.0 / max(n, 1)) * (1 - p) / max(n, 1))


def check(m, g_cost, o, sens, label="", strict_well=True):
    """Assert the bar above; returns a dict of the measured statistics (also
    appended to $MPCR_PARITY_LOG before anything is asserted).
    strict_well=False reports the well-conditioned misses instead of holding
    them to probe B's count; every other part of the bar still holds."""
    oc = o["cost4"][:, 0]
    g = np.asarray(g_cost, dtype=np.float64)
    rel = np.abs(g - oc) / np.maximum(np.abs(oc), 1e-12)
    graze = grazing(m, o)
    well = (sens < TOL / 10) & ~graze
    n, nw = len(oc), int(well.sum())
    pb = o["probe_b"]
    pf = o["probe_f4"][:, 0] if "probe_f4" in o else np.zeros(n)
    stats = dict(n=n, well=nw, graze=int(graze.sum()), miss=float((rel > TOL).mean()),
                 intrinsic_miss=float((sens > TOL).mean()), median_rel=float(np.median(rel)),
                 well_miss=int((well & (rel >= TOL)).sum()), probe_b_well_miss=int((well & (pb >= TOL)).sum()),
                 probe_f_well_miss=int((well & (pf >= TOL)).sum()),
                 max_rel_well=float(rel[well].max()) if well.any() else 0.0,
                 max_rel_well_probe_f=float(pf[well].max()) if well.any() else 0.0)
    # the allowance is probe B's count + 3 binomial sigma (round 4: probe F,
    # the fp32 restatement, is reported beside it, no longer allowed -- the
    # dual-arm kernels without fast math brought the C4 shard inside probe B)
    bw = stats["probe_b_well_miss"] / max(nw, 1)
    stats["well_miss_allowed"] = float((bw + _sigma3(bw, nw)) * max(nw, 1))
    stats["well_miss_allowed_probe_b_only"] = stats["well_miss_allowed"]
    bf = max(stats["probe_b_well_miss"], stats["probe_f_well_miss"]) / max(nw, 1)
    stats["well_miss_allowed_with_probe_f"] = float((bf + _sigma3(bf, nw)) * max(nw, 1))
    ig, io = int(np.argmin(g)), int(np.argmin(oc))
    ug, uo = max(TOL, sens[ig], pb[ig]), max(TOL, sens[io], pb[io])
    stats.update(sel_gpu=ig, sel_oracle=io, sel_rel=float(rel[ig]), sel_gap=float((oc[ig] - oc[io]) / abs(oc[io])),
                 sel_cond=float(ug), sel_probe_f=float(pf[ig]))
    _log(label, stats)
    assert not strict_well or stats["well_miss"] <= stats["well_miss_allowed"], (
        label, "well-conditioned misses beyond probe B's",
        [(int(i), float(rel[i]), float(sens[i])) for i in np.where(well & (rel >= TOL))[0][:6]], stats)
    im = stats["intrinsic_miss"]
    assert stats["miss"] <= im + _sigma3(im, n) + 0.01, (label, stats)
    assert stats["median_rel"] < 1e-5, (label, stats)
    # the selection (SBP/mjx_planner.py:395)
    assert rel[ig] < ug, (label, "selected cost", stats)
    assert oc[ig] <= oc[io] + (ug + uo) * abs(oc[io]), (label, "selected is not the oracle's best", stats)
    if ig != io:
        second = np.partition(oc, 1)[1]
        assert (second - oc[io]) <= (ug + uo) * abs(oc[io]), (label, "indices differ without a near-tie", stats)
    return stats


def _log(label, stats):
    """Append the statistics to $MPCR_PARITY_LOG (one JSON line per check)."""
    path = os.environ.get("MPCR_PARITY_LOG")
    if path:
        import json
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(dict(label=label, **stats)) + "\n")


COMPONENTS = ("cost", "cost_g", "cost_r", "cost_c")


def cost_c_parts(slots, y=0.005):
    """(relu sum, integer count) of cost_c from per-step masked slot
    distances (n, H, S) -- compute_cost_single, SBP/mjx_planner.py:287-296."""
    sl = np.asarray(slots, dtype=np.float64)
    relu = np.maximum((1 - y) * sl[:, :-1] - sl[:, 1:], 0).sum(axis=(1, 2))
    return relu, (sl < 0).sum(axis=(1, 2))


def check_components(m, g_cost4, o, label="", g_slots=None, strict=True):
    """Component-level parity (1e-4 on cost, g and r; cost_c
    exact except when grazing; the reference returns best_cost_g/r/c,
    SBP/mjx_planner.py:400-402).  Each of g, r and c is held to the same
    conditioning bar as the total, with its own probe sensitivities: the GPU
    may miss 1e-4 on no more of the component-well-conditioned candidates than
    probe B does (+3 sigma), and on no more of all candidates than probe A
    (+3 sigma + 1 %).

    With ``g_slots`` (the kernel's traced masked-slot distances, n x H x S)
    the integer #{c < 0} term of cost_c (SBP/mjx_planner.py:296) is checked
    two ways, bit for bit:
      * inside the kernel: its cost_c minus the relu sum of its own traced
        distances is exactly the count of its negative traced distances;
      * against the oracle: the counts are equal on every candidate that
        grazes no contact (no |dist| < 1e-5 m), whose count no probe changes
        and whose slot distances track the oracle's to 1e-4 m at every step
        (a trajectory that drifted -- fp32 contact-solve noise, DESIGN.md
        §Parity -- is reported, not held to an integer equality).
    Returns per-component stats."""
    g4 = np.asarray(g_cost4, dtype=np.float64)
    o4 = o["cost4"]
    graze = grazing(m, o)
    out = {}
    for k in (1, 2, 3):
        name = COMPONENTS[k]
        oc, gc = o4[:, k], g4[:, k]
        zero = (oc == 0) & (gc == 0)
        rel = np.where(zero, 0.0, np.abs(gc - oc) / np.maximum(np.abs(oc), 1e-12))
        sens, pb = o["sens4"][:, k], o["probe_b4"][:, k]
        pf = o["probe_f4"][:, k] if "probe_f4" in o else np.zeros(len(oc))
        sens, pb, pf = (np.where(zero, 0.0, x) for x in (sens, pb, pf))
        well = (sens < TOL / 10) & ~graze
        n, nw = len(oc), int(well.sum())
        st = dict(n=n, well=nw, miss=float((rel > TOL).mean()), intrinsic_miss=float((sens > TOL).mean()),
                  median_rel=float(np.median(rel)), well_miss=int((well & (rel >= TOL)).sum()),
                  probe_b_well_miss=int((well & (pb >= TOL)).sum()), probe_f_well_miss=int((well & (pf >= TOL)).sum()),
                  max_rel_well=float(rel[well].max()) if well.any() else 0.0,
                  max_rel_well_probe_f=float(pf[well].max()) if well.any() else 0.0)
        bw = st["probe_b_well_miss"] / max(nw, 1)  # probe B only (probe F reported)
        st["well_miss_allowed"] = float((bw + _sigma3(bw, nw)) * max(nw, 1))
        out[name] = st
    bad = np.zeros(0, int)
    if g_slots is not None and m.nslot:
        gs = np.asarray(g_slots, dtype=np.float64)
        relu, gn = cost_c_parts(gs)
        kint = g4[:, 3] - relu  # the kernel's integer term, recovered from its own cost_c
        k_bad = np.where(np.abs(kint - gn) >= 0.5)[0]
        on = o["nneg"].astype(np.int64)
        track = (np.abs(gs - o["slots"]) <= 1e-4).all(axis=(1, 2))
        stable = ~graze & ~o["nneg_unstable"] & track
        bad = np.where(stable & (gn != on))[0]
        out["nneg"] = dict(kernel_internal_mismatch=int(k_bad.size), stable=int(stable.sum()),
                           exact=int((stable & (gn == on)).sum()), mismatched=int(bad.size),
                           drifted=int((~graze & ~track).sum()), drifted_mismatched=int((~stable & (gn != on)).sum()),
                           total_oracle=int(on.sum()), total_gpu=int(gn.sum()))
    _log(label + " components", out)
    for k in (1, 2, 3):
        name, st = COMPONENTS[k], out[COMPONENTS[k]]
        n = st["n"]
        if strict:
            assert st["well_miss"] <= st["well_miss_allowed"], (label, name, "well-conditioned misses beyond probe B's", st)
            im = st["intrinsic_miss"]
            assert st["miss"] <= im + _sigma3(im, n) + 0.01, (label, name, st)
            assert st["median_rel"] < 1e-5, (label, name, st)
    if "nneg" in out:
        assert out["nneg"]["kernel_internal_mismatch"] == 0, (label, "cost_c's integer term", out["nneg"])
        if strict:
            assert bad.size == 0, (label, "#{c<0} differs on a stable candidate", [int(i) for i in bad[:6]], out["nneg"])
    return out

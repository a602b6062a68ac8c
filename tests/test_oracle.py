"""Oracle pinning: the fp64 C restatement vs the reference's logged CPU
MuJoCo run (SBP/data/theta.csv, thetadot.csv -> tests/golden/replay.npz), the
numpy transliteration of compute_cost_single, and analytic invariants."""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from oracle import cem_np

R = np.load(os.path.join(GOLDEN, "replay.npz"))


def _replay(m, steps):
    th, td, dt = R["theta"], R["thetadot"], float(R["dt"])
    prev = R["q0"].copy()
    err, ref = [], []
    for k in steps:
        prev = th[k - 1] if k > 0 else R["q0"]
        qpos = m.qpos_init.copy()
        qpos[:6] = prev
        qvel = np.zeros(m.nv)
        qvel[:6] = td[k]
        r = oracle.step(m, qpos, qvel, np.zeros(m.nv))
        qref = (th[k] - prev - dt * td[k]) / dt ** 2
        err.append(r["qacc"][:6] - qref)
        ref.append(qref)
    return np.array(err), np.array(ref)


def test_replay_pins_mass_matrix_coriolis_gravcomp(planner_model):
    """Row k of thetadot.csv was applied as qvel[:6] before mj_step and row k of
    theta.csv logged after it (SBP/mpc_planner.py:179-180,226-227): the
    residual recovers CPU MuJoCo's arm qacc to ~1e-10."""
    err, ref = _replay(planner_model, range(0, 896, 2))
    rel = np.linalg.norm(err) / np.linalg.norm(ref)
    assert rel < 2e-3, rel
    assert np.median(np.abs(err)) < 2e-6
    # a 5% change of the hand's mass would move the residual > 5x: the pin is sharp
    import copy
    m2 = copy.deepcopy(planner_model)
    hande = m2.names["body"].index("hande")
    m2.body_mass[hande] *= 1.05
    m2.body_inertia[hande] *= 1.05
    err2, _ = _replay(m2, range(0, 896, 8))
    assert np.linalg.norm(err2) / np.linalg.norm(ref[::4]) > 3 * rel


def test_gravcomp_zero_velocity_is_static(planner_model):
    m = planner_model
    qpos = m.qpos_init.copy()
    qpos[:6] = [1.5, -1.8, 1.75, -1.25, -1.6, 0.0]
    r = oracle.step(m, qpos, np.zeros(m.nv), np.zeros(m.nv))
    np.testing.assert_allclose(r["qacc"][:6], 0, atol=1e-10)
    M = r["M"]
    np.testing.assert_allclose(M, M.T, atol=1e-14)
    assert np.linalg.eigvalsh(M).min() > 0
    # the free target box falls at g
    np.testing.assert_allclose(r["qacc"][6:9], [0, 0, -9.81], atol=1e-9)


def test_no_gravcomp_arm_sags(all_models):
    m = all_models["ur5e_hande_mjx"]
    qpos = m.qpos_init.copy()
    qpos[:6] = [1.5, -1.8, 1.75, -1.25, -1.6, 0.0]
    r = oracle.step(m, qpos, np.zeros(m.nv), np.zeros(m.nv))
    assert np.abs(r["qacc"][:6]).max() > 1.0


def test_rollout_cost_matches_transliteration(all_models):
    m = all_models["scene_mjx"]
    rng = np.random.default_rng(3)
    n, H = 6, 20
    t = np.arange(H) * 0.05
    td = (rng.uniform(-0.6, 0.6, (n, 6, 1)) * np.sin(rng.uniform(0.2, 2, (n, 6, 1)) * t)).reshape(n, 6 * H)
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    w = np.array([20.0, 3.0, 80.0])
    pt, qt = np.array([-0.3, -0.3, 0.5]), np.array([0.0, 1.0, 0.0, 0.0])
    out = oracle.rollout(m, td, q0, w, pt, qt, want_slots=True, want_eef=True)
    for b in range(n):
        ref = cem_np.cost_single(out["eef"][b, :, :3], out["eef"][b, :, 3:], out["slots"][b], pt, qt, w)
        np.testing.assert_allclose(out["cost4"][b], ref, rtol=1e-12)
    # post-step theta: first step = q0 + dt*thetadot_0 + dt^2*qacc_0
    assert np.abs(out["theta"][:, ::H] - (q0 + 0.05 * td[:, ::H])).max() < 0.05 ** 2 * 50


def test_contact_slots_far_field_and_collision(planner_model):
    m = planner_model
    qpos = m.qpos_init.copy()
    qpos[:6] = [1.5, -1.8, 1.75, -1.25, -1.6, 0.0]
    r = oracle.step(m, qpos, np.zeros(m.nv), np.zeros(m.nv))
    d = r["dist"]
    masked = np.concatenate([d[m.pair_conadr[p]:m.pair_conadr[p] + m.pair_ncon[p]]
                             for p in range(m.npair) if m.pair_slotadr[p] >= 0])
    assert masked.size == m.nslot and np.all(np.isfinite(masked)) and masked.min() > 0
    # drive the elbow into the table: some masked slot must go negative
    qpos[:6] = [1.5, 0.9, 1.0, -1.25, -1.6, 0.0]
    d2 = oracle.step(m, qpos, np.zeros(m.nv), np.zeros(m.nv))["dist"]
    masked2 = np.concatenate([d2[m.pair_conadr[p]:m.pair_conadr[p] + m.pair_ncon[p]]
                              for p in range(m.npair) if m.pair_slotadr[p] >= 0])
    assert masked2.min() < 0


def test_box_settles_on_table(all_models):
    """C3's object_0 starts 25 mm inside the table (URD/object.xml:2-5): the
    contact pushes it out and it comes to rest on the top face (z = 0.525)."""
    m = all_models["scene_mjx"]
    qpos = m.qpos_init.copy()
    qpos[:6] = [1.5, -1.8, 1.75, -1.25, -1.6, 0.0]
    qvel = np.zeros(m.nv)
    ws = np.zeros(m.nv)
    a = m.jnt_qposadr[m.names["joint"].index("free_joint_0")]
    for _ in range(60):
        qvel[:6] = 0
        r = oracle.step(m, qpos, qvel, ws)
        qpos, qvel, ws = r["qpos"], r["qvel"], r["qacc_warmstart"]
    assert abs(qpos[a + 2] - 0.525) < 0.01, qpos[a:a + 3]
    assert np.abs(qvel[8:14]).max() < 0.05


def _cost_batch(m, n=8, H=20, seed=3):
    rng = np.random.default_rng(seed)
    t = np.arange(H) * 0.05
    td = (rng.uniform(-0.6, 0.6, (n, 6, 1)) * np.sin(rng.uniform(0.2, 2, (n, 6, 1)) * t)).reshape(n, 6 * H)
    return td, np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0]), np.array([20.0, 3.0, 80.0]), \
        np.array([-0.3, -0.3, 0.5]), np.array([0.0, 1.0, 0.0, 0.0])


def test_integer_collision_count_is_the_slot_count(all_models):
    """info's #{c < 0} (SBP/mjx_planner.py:296) is the number of negative
    masked-slot distances over the horizon."""
    m = all_models["scene_mjx"]
    td, q0, w, pt, qt = _cost_batch(m)
    out = oracle.rollout(m, td, q0, w, pt, qt, want_slots=True)
    np.testing.assert_array_equal(out["nneg"], (out["slots"] < 0).sum(axis=(1, 2)))


def test_exact_mode_switches_and_restores(all_models):
    """The MuJoCo-exact mode (every rule MuJoCo's, the support-axis tie by
    mju_sign too, exact argmax picks) is a global switch that the context
    manager restores."""
    m = all_models["scene_mjx"]
    td, q0, w, pt, qt = _cost_batch(m, n=4)
    a = oracle.rollout(m, td, q0, w, pt, qt)["cost4"]
    with oracle.exact():
        assert oracle.lib().oracle_get_exact() == 31
        b = oracle.rollout(m, td, q0, w, pt, qt)["cost4"]
    assert oracle.lib().oracle_get_exact() == oracle.DEFAULT_EXACT
    assert np.all(np.isfinite(b))
    assert np.median(np.abs(a - b) / np.maximum(np.abs(a), 1e-12)) < 1e-3


def test_fp32_build_tracks_fp64(all_models):
    """oracle_f32.c (bench.py's cpu_baseline at the reference's fp32) computes
    the same costs as the fp64 checker to fp32 accuracy on a smooth batch."""
    m = all_models["ur5e_hande_mjx"]
    td, q0, w, pt, qt = _cost_batch(m, n=6, H=16, seed=5)
    r64 = oracle.Runner(m, 2, q0, w, pt, qt, precision="fp64")
    r32 = oracle.Runner(m, 2, q0, w, pt, qt, precision="fp32")
    try:
        c64, c32 = r64.rollout(td), r32.rollout(td)
    finally:
        r64.close()
        r32.close()
    assert c32.dtype == np.float32
    rel = np.abs(c32[:, 0] - c64[:, 0]) / np.abs(c64[:, 0])
    assert np.median(rel) < 1e-4, rel

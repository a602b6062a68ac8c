"""Closed-loop plant (mpcr_plant_*, engine.Plant): the reference's CPU
``data.qvel[:6] = thetadot; mj_step`` (SBP/mpc_planner.py:179-180) and
``mj_forward`` (:114) on the GPU.

* bit-identical to the rollout kernel: k plant steps with a velocity sequence
  give the rollout's theta row and per-step eef pose exactly (same kernel,
  state round-tripped through fp32 HBM);
* the fp64 oracle's ``oracle_step`` from the same state: qpos/qvel/qacc and
  the pre-integration eef pose within 1e-4 (abs) per step, over a 20-step
  contact-free closed loop;
* mj_forward does not advance the state and reports the step's qacc.
"""
import numpy as np
import pytest

import oracle
from manipulator_mujoco_amd import basis, models
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_THETADOT, Engine, Plant

pytestmark = pytest.mark.gpu

Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch


def _start(m):
    qpos = np.array(m.qpos_init[:m.nq], dtype=np.float64)
    qpos[np.asarray(m.ctrl_qposadr[:6])] = Q0
    return qpos


@pytest.mark.parametrize("name", models.PLANNER_SCENES)
def test_plant_steps_equal_rollout_bitwise(torch_cuda, name):
    H = 12
    m = models.load(name, 0.05)
    rng = np.random.default_rng(3)
    td = rng.uniform(-0.6, 0.6, (1, 6 * H)).astype(np.float32)
    _, _, Pd, _ = basis.planner_basis(H, 0.05)
    eng = Engine(m, H, 1, Pd)
    tr = eng.trace(td, MPCR_LAYOUT_THETADOT, Q0, (20, 3, 80), (-0.3, -0.3, 0.5), (0, 1, 0, 0))
    plant = Plant(m)
    plant.set_state(qpos=_start(m))
    v = td.reshape(6, H)
    for t in range(H):
        plant.step(v[:, t].astype(np.float64))
        qa = np.asarray(m.ctrl_qposadr[:6])
        np.testing.assert_array_equal(plant.qpos[qa].astype(np.float32), tr["theta"][0].reshape(6, H)[:, t])
        np.testing.assert_array_equal(plant.eef.astype(np.float32), tr["eef"][0, t])


@pytest.mark.parametrize("name", ["planner_scene", "ur5e_hande_mjx", "scene_mjx"])
def test_plant_matches_oracle_step(torch_cuda, name):
    """Per step from the same state (plant re-synced to the oracle's fp64
    state each step, so contact chaos does not accumulate)."""
    m = models.load(name, 0.05)
    plant = Plant(m)
    qpos, qvel, qws = _start(m), np.array(m.qvel_init[:m.nv], dtype=np.float64), np.zeros(m.nv)
    rng = np.random.default_rng(5)
    da = np.asarray(m.ctrl_dofadr[:6])
    for t in range(20):
        u = rng.uniform(-0.3, 0.3, 6)
        plant.set_state(qpos=qpos, qvel=qvel, qacc_warmstart=qws)
        qvel = qvel.copy()
        qvel[da] = u
        o = oracle.step(m, qpos, qvel, qws)
        plant.step(u)
        np.testing.assert_allclose(plant.eef[:3], o["eef"][:3], atol=1e-5)
        np.testing.assert_allclose(np.abs(plant.eef[3:] @ o["eef"][3:]), 1.0, atol=1e-5)
        np.testing.assert_allclose(plant.qacc, o["qacc"], atol=2e-3, rtol=1e-3)
        qpos, qvel, qws = o["qpos"], o["qvel"], o["qacc_warmstart"]
        np.testing.assert_allclose(plant.qpos, qpos, atol=1e-5)
        np.testing.assert_allclose(plant.qvel, qvel, atol=1e-4, rtol=1e-4)


def test_plant_free_running_arm_tracks_oracle(torch_cuda):
    """20 free-running steps, contact-free arm (C2 model): the arm joints and
    the eef stay within 1e-4 of the fp64 oracle."""
    m = models.load("ur5e_hande_mjx", 0.05)
    plant = Plant(m)
    qpos, qvel, qws = _start(m), np.array(m.qvel_init[:m.nv], dtype=np.float64), np.zeros(m.nv)
    plant.set_state(qpos=qpos, qvel=qvel, qacc_warmstart=qws)
    rng = np.random.default_rng(9)
    da, qa = np.asarray(m.ctrl_dofadr[:6]), np.asarray(m.ctrl_qposadr[:6])
    for t in range(20):
        u = rng.uniform(-0.3, 0.3, 6)
        qvel = qvel.copy()
        qvel[da] = u
        o = oracle.step(m, qpos, qvel, qws)
        plant.step(u)
        qpos, qvel, qws = o["qpos"], o["qvel"], o["qacc_warmstart"]
        np.testing.assert_allclose(plant.qpos[qa], qpos[qa], atol=1e-4)
        np.testing.assert_allclose(plant.eef[:3], o["eef"][:3], atol=1e-4)


def test_forward_does_not_advance(torch_cuda):
    m = models.load("planner_scene", 0.05)
    plant = Plant(m)
    plant.set_state(qpos=_start(m))
    q = plant.qpos.copy()
    plant.forward()
    np.testing.assert_array_equal(plant.qpos, q)
    acc_fwd, eef_fwd = plant.qacc.copy(), plant.eef.copy()
    v = plant.qvel[np.asarray(m.ctrl_dofadr[:6])].copy()
    plant.step(v)
    np.testing.assert_array_equal(plant.qacc, acc_fwd)
    np.testing.assert_array_equal(plant.eef, eef_fwd)
    assert not np.array_equal(plant.qpos, q)


SYNTHETIC = {
    "spheres": """
    <body name="a" pos="0 0 1"><freejoint/><geom name="a" type="sphere" size="0.1"/></body>
    <body name="b" pos="0.03 0.04 1.13"><freejoint/><geom name="b" type="sphere" size="0.1"/></body>""",
    "mesh_cubes": """
    <body name="c" pos="0 0 0.04"><freejoint/><geom name="c" type="mesh" mesh="cube"/></body>
    <body name="k" pos="0.3 0.01 0.03" euler="0.1 0.2 0.3"><freejoint/><geom name="k" type="mesh" mesh="cube"/></body>
    <body name="t" pos="0.3 0 -0.015"><geom name="t" type="box" size="0.2 0.2 0.01"/></body>""",
    "cylinder_capsule": """
    <body name="t" pos="0 0 -0.5"><geom name="t" type="box" size="1 1 0.5"/></body>
    <body name="y" pos="0 0 0.097" euler="0.05 0 0"><freejoint/><geom name="y" type="cylinder" size="0.05 0.1"/></body>
    <body name="p" pos="0.5 0 0.015" euler="0 1.5 0"><freejoint/><geom name="p" type="capsule" size="0.02 0.1"/></body>
    <body name="q" pos="0.05 0.3 0.05"><freejoint/><geom name="q" type="cylinder" size="0.03 0.06"/></body>""",
    # two geoms of one mesh (one face range), 8 mm deep: the all-face SAT's
    # winner is g2's face (oracle pinned in tests/test_dual_arm.py)
    "shared_mesh_deep": """
    <body name="a" pos="0 0 0.2" euler="0.3 0 0"><freejoint/><geom name="a" type="mesh" mesh="cube"/></body>
    <body name="b" pos="0.01 0 0.30454"><freejoint/><geom name="b" type="mesh" mesh="cube"/></body>""",
}


@pytest.mark.parametrize("scene", list(SYNTHETIC))
def test_wide_kernel_convex_contacts_match_oracle(torch_cuda, tmp_path, scene):
    """The wide variant's MPR / plane-convex contacts on synthetic scenes with
    known penetrations (tests/test_dual_arm.py pins the oracle's depths
    analytically): the contact-driven accelerations of a forward pass and the
    state after 5 steps agree with the fp64 oracle."""
    from test_dual_arm import _scene
    m = _scene(tmp_path, SYNTHETIC[scene], option='<option timestep="0.01"/>')
    plant = Plant(m)
    plant.forward()
    qpos, qvel, qws = m.qpos_init[:m.nq].copy(), np.zeros(m.nv), np.zeros(m.nv)
    o = oracle.step(m, qpos, qvel, qws)
    assert o["nefc"] > 0
    np.testing.assert_allclose(plant.qacc, o["qacc"], rtol=2e-3, atol=2e-3 * np.abs(o["qacc"]).max())
    plant.step(None)  # o already holds the state after the first step
    for _ in range(4):
        plant.step(None)
        o = oracle.step(m, o["qpos"], o["qvel"], o["qacc_warmstart"])
    np.testing.assert_allclose(plant.qpos, o["qpos"], atol=1e-4)


# ---------------------------------------------------------------------------
# scene_robotiq_hande.xml: elliptic cones + impratio, fluid
# viscosity, a spatial-tendon length limit; wide kernel variant, no controls


def _hande_settled(m, steps=300):
    """The oracle's state after `steps` from qpos0: the gripper resting on
    the floor (elliptic contacts active), the box hanging on its tendon."""
    qpos, qvel, ws = m.qpos0[:m.nq].copy(), np.zeros(m.nv), np.zeros(m.nv)
    for _ in range(steps):
        o = oracle.step(m, qpos, qvel, ws)
        qpos, qvel, ws = o["qpos"], o["qvel"], o["qacc_warmstart"]
    return qpos, qvel, ws


def test_plant_hande_scene_matches_oracle_step(torch_cuda):
    """Per step from the oracle's fp64 state (re-synced every step): qacc,
    qpos, qvel of the wide kernel vs oracle_step, with the gripper's
    elliptic-cone floor contacts, the tendon limit row and viscosity live."""
    m = models.load("hande_scene")
    plant = Plant(m)
    qpos, qvel, ws = _hande_settled(m)
    for t in range(30):
        plant.set_state(qpos=qpos, qvel=qvel, qacc_warmstart=ws)
        o = oracle.step(m, qpos, qvel, ws)
        plant.step()
        # the rows the oracle built: the finger equality, the tendon limit (the
        # box hangs at 2 cm + stretch), and >= 2 elliptic contacts (3 rows
        # each) from the plane-mesh manifold under the resting gripper
        ncon = int((o["dist"] < 0).sum())
        assert ncon >= 2 and o["nefc"] >= 1 + 1 + 3 * ncon, (ncon, o["nefc"])
        scale = max(1.0, np.abs(o["qacc"]).max())
        np.testing.assert_allclose(plant.qacc, o["qacc"], atol=2e-3 * scale, rtol=2e-3)
        qpos, qvel, ws = o["qpos"], o["qvel"], o["qacc_warmstart"]
        np.testing.assert_allclose(plant.qpos, qpos, atol=1e-5)
        np.testing.assert_allclose(plant.qvel, qvel, atol=1e-4, rtol=1e-3)


def test_plant_hande_scene_transient_matches_oracle(torch_cuda):
    """The first 60 steps from qpos0 with the box thrown sideways (re-synced
    to the oracle every step): the tendon pulls the box in from 4.1 cm, the
    viscous drag acts on a fast box, the gripper lands.  qacc must agree, and
    so must the viscosity's own contribution (qacc with viscosity minus qacc
    without, a difference of two wide-kernel runs vs the oracle's)."""
    m = models.load("hande_scene")
    m0 = models.load("hande_scene")
    m0.viscosity = 0.0
    plant, plant0 = Plant(m), Plant(m0)
    ob = m.names["body"].index("object")
    d0 = int(m.body_dofadr[ob])
    qpos, qvel, ws = m.qpos0[:m.nq].copy(), np.zeros(m.nv), np.zeros(m.nv)
    qvel[d0:d0 + 3] = [0.8, -0.5, 0.3]
    qvel[d0 + 3:d0 + 6] = [3.0, -2.0, 1.0]
    tendon_seen = 0
    for t in range(60):
        for p in (plant, plant0):
            p.set_state(qpos=qpos, qvel=qvel, qacc_warmstart=ws)
            p.step()
        o = oracle.step(m, qpos, qvel, ws)
        o0 = oracle.step(m0, qpos, qvel, ws)
        scale = max(1.0, np.abs(o["qacc"]).max())
        np.testing.assert_allclose(plant.qacc, o["qacc"], atol=2e-3 * scale, rtol=2e-3)
        dv, dv_o = (plant.qacc - plant0.qacc)[d0:d0 + 6], (o["qacc"] - o0["qacc"])[d0:d0 + 6]
        # dv is a difference of two fp32 solves: each qacc carries ~1e-6 x scale
        # of rounding (a summation-order change alone moved dv by 1.7e-3 here)
        np.testing.assert_allclose(dv, dv_o, atol=1e-3 * max(1.0, np.abs(dv_o).max()) + 1e-5 * scale)
        from manipulator_mujoco_amd import mjcf
        tendon_seen += mjcf.tendon_jac(m, mjcf.kinematics0(m, qpos), 0)[0] > 0.02
        qpos, qvel, ws = o["qpos"], o["qvel"], o["qacc_warmstart"]
        np.testing.assert_allclose(plant.qpos, qpos, atol=1e-5)
    assert tendon_seen > 30  # the limit row was live for most of the window


def test_plant_hande_scene_free_running(torch_cuda):
    """600 free-running GPU steps from qpos0 (1.2 s): the same physical
    end state as the oracle's (tests/test_hande_scene.py): the box held at
    the tendon's 2 cm limit, the gripper resting on the floor."""
    from manipulator_mujoco_amd import mjcf
    m = models.load("hande_scene")
    plant = Plant(m)
    plant.set_state(qpos=m.qpos0[:m.nq], qvel=np.zeros(m.nv), qacc_warmstart=np.zeros(m.nv))
    for _ in range(600):
        plant.step()
    assert np.isfinite(plant.qpos).all()
    L = mjcf.tendon_jac(m, mjcf.kinematics0(m, plant.qpos), 0)[0]
    assert 0.02 <= L < 0.0215
    ob = m.names["body"].index("object")
    d0 = int(m.body_dofadr[ob])
    assert np.abs(plant.qvel[d0:d0 + 3]).max() < 0.05
    assert np.abs(plant.qvel[0:3]).max() < 0.05 and plant.qpos[2] < 0.05



def test_dual_arm_large_hull_plane_manifold_matches_oracle(torch_cuda):
    """The wave-cooperative plane-mesh manifold (csrc/rollout.hip
    plane_mesh_manifold_wave) on the hulls of >= 600 vertices: a C4 candidate
    whose gripper and wrist meshes land on the table (tools/diag_manifold.py,
    candidate 2989 of the seed-20250632 batch: 36 steps with 4-point mesh
    manifolds; 2986 until round 4's capsule-box far-end rule changed its
    trajectory so that the meshes no longer reach the table), stepped from the oracle's fp64
    state every step.  Bars: the same contacts of those pairs as the oracle
    (pair and vertex, position within 0.2 mm -- a different vertex is cm away)
    at every step; qacc within 5e-3 of the step's largest |qacc| (the stiff
    arm-1 servos; measured 2.3e-3 max, 8.8e-4 median), each against the fp64
    oracle or its fp32 build (probe F)."""
    import os
    import sys

    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import diag_manifold
    rows, big, pairs = diag_manifold.run(2989)
    act = [r for r in rows if r["n_mesh"] > 0]
    assert len(big) >= 2 and len(act) >= 20 and max(r["n_mesh"] for r in act) == 4
    assert all(r["same"] or r["same_f32"] for r in act), [r for r in act if not r["same"]][:3]
    # contacts and qacc: against the fp64 oracle, or -- where the step holds a flush
    # mesh-mesh contact whose MPR portal flips under fp32 rounding (gripper
    # linkage pair; tools/diag_parity.py) -- against the fp32 oracle build,
    # which then takes the kernel's portal; the bar holds against one of them
    bad = [r for r in rows if min(r["qacc_err"], r["qacc_err_f32"]) >= 5e-3]
    assert not bad, bad[:3]
    assert np.median([r["qacc_err"] for r in rows]) < 5e-3


def test_dual_arm_finger_hulls_match_oracle_at_traced_steps(torch_cuda):
    """C4's selected candidate (558 of the seed-4 shard):
    the Hand-E finger hulls interpenetrate ~2 cm, where the polyhedron
    manifold's clip can keep no point and the SAT axis then carries one
    contact at the incident support vertex.  The plant, set to the fp64
    oracle's state at each traced step, finds that pair's contacts with the
    oracle's normal and depth, and the step's qacc within 5e-3 of its scale
    (the GPU left the oracle there by 0.14 of 235-822 before the rule)."""
    import torch

    from manipulator_mujoco_amd.projection import ProjectionFilter
    m, H = models.load("dual_arm", 0.05), 100
    B, G = m.names["body"], m.geom_bodyid
    pair = next(p for p in range(m.npair)
                if {B[G[m.pair_geom1[p]]], B[G[m.pair_geom2[p]]]} == {"hande_left_finger", "hande_right_finger"})
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    f = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
    rng = np.random.default_rng(20250629 + 4)
    xi = torch.tensor(rng.normal(0, np.sqrt(10.003), (4096, 66)).astype(np.float32))[[558]]
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    xi = f(xi, f.boundary(q0, np.zeros(6), np.zeros(6), 1), 10).numpy()
    td = np.einsum("tk,njk->njt", Pd, xi.reshape(1, 6, 11).astype(np.float64)).reshape(6, H)
    qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
    qpos = np.array(m.qpos_init[:m.nq], dtype=np.float64)
    qpos[qa] = q0
    qvel, ws = np.array(m.qvel_init[:m.nv], dtype=np.float64), np.zeros(m.nv)
    plant = Plant(m)
    checked = 0
    for t in range(66):
        qv = qvel.copy()
        qv[da] = td[:, t]
        if t in (30, 54, 65):
            od = oracle.step_debug(m, qpos, qv, ws)
            plant.set_state(qpos=qpos, qvel=qv, qacc_warmstart=ws)
            gd = plant.step_debug(td[:, t])
            ko = [k for k in range(od["ncon"]) if od["con_pair"][k] == pair]
            kg = [k for k in range(gd["ncon"]) if gd["con_pair"][k] == pair]
            assert bool(ko) == bool(kg), (t, ko, kg)
            if ko:
                checked += 1
                assert np.abs(gd["con_normal"][kg[0]] - od["con_normal"][ko[0]]).max() < 1e-3, t
                assert abs(min(gd["con_dist"][k] for k in kg) - min(od["con_dist"][k] for k in ko)) < 1e-5, t
            scale = max(1.0, np.abs(od["qacc"]).max())
            assert np.abs(gd["qacc"] - od["qacc"]).max() < 5e-3 * scale, t
        st = oracle.step(m, qpos, qv, ws)
        qpos, qvel, ws = st["qpos"], st["qvel"], st["qacc_warmstart"]
    assert checked >= 2

"""Model front end: MJCF compiler (manipulator_mujoco_amd/mjcf.py) and the
bundled models the GPU box uses."""
import ctypes
import os

import numpy as np
import pytest

import oracle
from conftest import REFERENCE, has_reference
from manipulator_mujoco_amd import cmodel, mjcf, models

SCENES = {
    "planner_scene": "sampling_based_planner/ur5e_hande_mjx/scene.xml",
    "ur5e_hande_mjx": "universal_robots_ur5e/ur5e_1_robotiq_hande_mjx.xml",
    "scene_mjx": "universal_robots_ur5e/scene_mjx.xml",
}


def test_struct_layout_matches_c():
    assert ctypes.sizeof(cmodel.mpcr_model_t) == oracle.lib().oracle_model_size()


@pytest.mark.parametrize("name,expect", [
    # (nbody, nq, nv, npair, nslot, neq): SURVEY.md §8a-A5/A6, §8d C2/C3
    ("planner_scene", (18, 13, 12, 114, 187, 0)),
    ("ur5e_hande_mjx", (12, 8, 8, 37, 47, 1)),
    ("scene_mjx", (13, 15, 14, 59, 87, 1)),
])
def test_bundle_sizes(all_models, name, expect):
    m = all_models[name]
    assert (m.nbody, m.nq, m.nv, m.npair, m.nslot, m.neq) == expect


def test_planner_pair_inventory(planner_model):
    from collections import Counter
    c = Counter(planner_model.pair_func.tolist())
    # 10 capsule-plane, 1 box-plane, 27 capsule-capsule, 70 capsule-box, 6 box-box
    assert c == {0: 10, 1: 1, 2: 27, 3: 70, 4: 6}
    robot = planner_model.geom_robot.astype(bool)
    for p in range(planner_model.npair):
        masked = robot[planner_model.pair_geom1[p]] or robot[planner_model.pair_geom2[p]]
        assert (planner_model.pair_slotadr[p] >= 0) == masked


def test_planner_constants(planner_model):
    m = planner_model
    assert m.timestep == 0.05 and m.iterations == 1 and m.ls_iterations == 5
    assert m.disableflags & cmodel.DSBL_EULERDAMP
    np.testing.assert_allclose(m.dof_armature[:6], 0.1)
    np.testing.assert_allclose(m.body_gravcomp[3:12], 1.0)
    hande = m.names["body"].index("hande")
    # hande has no <inertial>: coupler + hande meshes (legacy mesh inertia) + capsule robot_0
    assert 1.55 < m.body_mass[hande] < 1.70
    np.testing.assert_allclose(m.qpos0[6:13], [-0.3, -0.3, 0.5, 0, 1, 0, 0], atol=1e-12)
    assert m.names["site"][m.tcp_site] == "tcp"


@pytest.mark.skipif(not has_reference(), reason="needs /root/reference MJCF")
@pytest.mark.parametrize("name", list(SCENES))
def test_bundle_is_current(name):
    m = mjcf.compile_mjcf(os.path.join(REFERENCE, SCENES[name]), 0.05)
    assert m.to_blob() == models.load(name, 0.05).to_blob()


def test_capacity_errors():
    m = models.load("planner_scene", 0.05)
    m2 = models.load_bundle(os.path.join(models.HERE, models.BUNDLES["planner_scene"]))
    m2.nbody = cmodel.MAX_BODY + 1
    with pytest.raises(ValueError):
        m2.to_blob()
    assert m.to_blob()[:4] == (cmodel.MAGIC).to_bytes(4, "little")

"""Precompiled model bundles (.npz) of the reference's MJCF scenes.

``/root/reference`` (MJCF + meshes) does not exist on the GPU box, so the
scenes the planner and BASELINE.json configs use are compiled here by
``tools/compile_models.py`` (manipulator_mujoco_amd.mjcf) and shipped as
plain numeric arrays:

* ``planner_scene``   SBP/ur5e_hande_mjx/scene.xml (what cem_planner loads,
                      SBP/mjx_planner.py:100) — UR5e + Hand-E (welded),
                      gravcomp, free target_0, static targets/obstacles
* ``ur5e_hande_mjx``  URD/ur5e_1_robotiq_hande_mjx.xml (config C2)
* ``scene_mjx``       URD/scene_mjx.xml = arm + object.xml box (config C3)
* ``dual_arm``        URD/dual_arm_gripper_scene.xml (configs C4/C5): UR5e +
                      Hand-E and UR5e + Robotiq 2F-85, implicitfast, 14
                      actuators, fixed tendons, connect/joint equalities,
                      convex-hull mesh collision
* ``hande_scene``     URD/scene_robotiq_hande.xml: free Hand-E
                      gripper + a box hung from a spatial tendon; elliptic
                      cones with impratio 10, fluid viscosity 0.1, own
                      timestep 0.002
"""

from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

BUNDLES = {
    "planner_scene": "planner_scene.npz",
    "ur5e_hande_mjx": "ur5e_hande_mjx.npz",
    "scene_mjx": "scene_mjx.npz",
    "dual_arm": "dual_arm.npz",
    "hande_scene": "hande_scene.npz",
}
# the scenes with a planner-controlled arm (num_dof = 6); hande_scene has none
PLANNER_SCENES = ("planner_scene", "ur5e_hande_mjx", "scene_mjx", "dual_arm")

_SCALARS = ("nbody", "njnt", "nq", "nv", "ngeom", "nsite", "npair", "neq", "ncon", "nslot", "nctrl",
            "hande_body", "tcp_site", "iterations", "ls_iterations", "disableflags", "ntree", "timestep",
            "tolerance", "ls_tolerance", "impratio", "meaninertia", "nu", "nhullv", "nhulla", "integrator",
            "cone", "nten", "viscosity", "density", "nface", "nfacev", "nvface")


def save_bundle(m, path):
    arrays = {}
    for k, v in vars(m).items():
        if isinstance(v, np.ndarray):
            arrays[k] = v
    meta = {k: (getattr(m, k).item() if hasattr(getattr(m, k), "item") else getattr(m, k)) for k in _SCALARS}
    meta["names"] = m.names
    meta["source"] = os.path.relpath(m.source, "/root/reference") if getattr(m, "source", "") else ""
    meta["opt"] = {k: (list(v) if isinstance(v, tuple) else v) for k, v in m.opt.items()}
    np.savez_compressed(path, __meta__=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8), **arrays)


def load_bundle(path, timestep=None):
    from ..mjcf import Model
    z = np.load(path, allow_pickle=False)
    meta = json.loads(bytes(z["__meta__"]).decode())
    m = Model()
    for k in z.files:
        if k != "__meta__":
            setattr(m, k, z[k])
    for k in _SCALARS:
        setattr(m, k, meta.get(k, 0))
    m.names = meta["names"]
    m.opt = meta["opt"]
    m.source = meta.get("source", "")
    if timestep is not None:
        m.timestep = float(timestep)
    return m


def load(name, timestep=None):
    """Load a bundled model by name (see BUNDLES)."""
    if name not in BUNDLES:
        raise KeyError(f"unknown bundled model {name!r}; have {sorted(BUNDLES)}")
    return load_bundle(os.path.join(HERE, BUNDLES[name]), timestep)

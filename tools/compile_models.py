"""Compile the reference's MJCF scenes into bundled .npz models.

Run in the build container (needs /root/reference for the MJCF + meshes):
    python tools/compile_models.py
The outputs are plain numeric arrays (no reference source text).
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from manipulator_mujoco_amd import mjcf, models  # noqa: E402

REF = os.environ.get("MPCR_REFERENCE", "/root/reference")
SCENES = {
    "planner_scene": "sampling_based_planner/ur5e_hande_mjx/scene.xml",
    "ur5e_hande_mjx": "universal_robots_ur5e/ur5e_1_robotiq_hande_mjx.xml",
    "scene_mjx": "universal_robots_ur5e/scene_mjx.xml",
    "dual_arm": "universal_robots_ur5e/dual_arm_gripper_scene.xml",
    "hande_scene": "universal_robots_ur5e/scene_robotiq_hande.xml",
}
# scenes simulated at their own timestep (not planner scenes)
NATIVE_DT = {"hande_scene"}


def main():
    for name, rel in SCENES.items():
        m = mjcf.compile_mjcf(os.path.join(REF, rel), timestep=None if name in NATIVE_DT else 0.05)
        out = os.path.join(models.HERE, models.BUNDLES[name])
        models.save_bundle(m, out)
        print(f"{name}: nbody={m.nbody} nq={m.nq} nv={m.nv} npair={m.npair} nslot={m.nslot} -> {out}")


if __name__ == "__main__":
    main()

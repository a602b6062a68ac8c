"""Generate tests/golden/ fixtures from the reference (run in the build container).

Imports ONLY the reference's numpy-only modules (the planner itself needs
jax/mujoco, which are absent):
  SBP/bernstein_coeff_ordern_arbitinterval.py  (called by the planner, :40)
  SBP/bernstein_coeff_order10_arbitinterval.py (closed-form equivalent)
  SBP/quat_math.py
and converts the reference's logged CPU-MuJoCo run (SBP/data/theta.csv,
thetadot.csv) to .npz.  Outputs are data only (inputs + expected outputs).
    PYTHONDONTWRITEBYTECODE=1 python tools/make_golden.py
"""

import os
import sys

import numpy as np

REF = os.environ.get("MPCR_REFERENCE", "/root/reference")
SBP = os.path.join(REF, "sampling_based_planner")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
sys.dont_write_bytecode = True
sys.path.insert(0, SBP)

import bernstein_coeff_order10_arbitinterval as b10  # noqa: E402
import bernstein_coeff_ordern_arbitinterval as bn  # noqa: E402
import quat_math  # noqa: E402


def main():
    os.makedirs(OUT, exist_ok=True)
    arrays = {}
    for H in (10, 16, 20, 50, 100):
        dt = 0.05
        t = np.linspace(0, H * dt, H).reshape(H, 1)  # SBP/mjx_planner.py:34-38
        P, Pd, Pdd = bn.bernstein_coeff_ordern_new(10, t[0], t[-1], t)
        P10, Pd10, Pdd10 = b10.bernstein_coeff_order10_new(10, t[0], t[-1], t)
        arrays[f"H{H}_t"] = t[:, 0]
        arrays[f"H{H}_P"] = P
        arrays[f"H{H}_Pdot"] = Pd
        arrays[f"H{H}_Pddot"] = Pdd
        arrays[f"H{H}_P10"] = P10
        arrays[f"H{H}_Pdot10"] = Pd10
        arrays[f"H{H}_Pddot10"] = Pdd10
    np.savez_compressed(os.path.join(OUT, "basis.npz"), **arrays)

    rng = np.random.default_rng(20250629)
    q1 = rng.normal(size=(64, 4))
    q1 /= np.linalg.norm(q1, axis=1, keepdims=True)
    q2 = rng.normal(size=(64, 4))
    q2 /= np.linalg.norm(q2, axis=1, keepdims=True)
    q2[:4] = q1[:4]          # identical -> 0
    q2[4:8] = -q1[4:8]       # antipodal -> 0 (abs)
    dist = np.array([quat_math.quaternion_distance(a, b) for a, b in zip(q1, q2)])
    mul = np.array([quat_math.quaternion_multiply(a, b) for a, b in zip(q1, q2)])
    ang = rng.uniform(-180, 180, 16)
    axes = rng.normal(size=(16, 3))
    rot = np.array([quat_math.rotation_quaternion(a, x) for a, x in zip(ang, axes)])
    np.savez_compressed(os.path.join(OUT, "quat.npz"), q1=q1, q2=q2, distance=dist, multiply=mul,
                        angle_deg=ang, axis=axes, rotation=rot)

    th = np.loadtxt(os.path.join(SBP, "data", "theta.csv"), delimiter=",")
    td = np.loadtxt(os.path.join(SBP, "data", "thetadot.csv"), delimiter=",")
    np.savez_compressed(os.path.join(OUT, "replay.npz"), theta=th, thetadot=td,
                        q0=np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0]), dt=np.array(0.05))
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()

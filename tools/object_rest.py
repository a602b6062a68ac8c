"""Does the C3 object (a free box on the table) stay bitwise at rest over a
rollout?  (diagnostic) Steps the plant (the rollout kernel with n = 1) along
a few candidates' joint velocities and counts the steps whose object qpos
equals the previous step's bit for bit -- where a cached box-box contact
set would be exact."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from diag_f32 import batch  # noqa: E402
from manipulator_mujoco_amd import models  # noqa: E402
from manipulator_mujoco_amd.engine import Plant  # noqa: E402

m = models.load("scene_mjx", 0.05)
H, n = 50, 8
td = batch(m, n, H, 3)
qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
obj = slice(m.nq - 7, m.nq)
tot = same = 0
for c in range(n):
    p = Plant(m)
    q = p.qpos.copy()
    q[qa] = [1.5, -1.8, 1.75, -1.25, -1.6, 0.0]
    p.set_state(qpos=q)
    prev = p.qpos[obj].copy()
    v = td[c].reshape(6, H)
    for t in range(H):
        p.step(v[:, t])
        cur = p.qpos[obj].copy()
        tot += 1
        same += bool(np.array_equal(cur, prev))
        prev = cur
    print(f"cand {c}: object qpos {np.round(cur, 6)} qvel {p.qvel[m.nv - 6:]}", flush=True)
print(f"steps with the object bitwise at rest: {same}/{tot}")

"""Distribution of per-candidate max constraint rows (status bits 2..7) on the bench workloads."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine  # noqa: E402
from manipulator_mujoco_amd.projection import ProjectionFilter  # noqa: E402

for name in ("scene_mjx", "planner_scene", "ur5e_hande_mjx", "dual_arm"):
    n, H = 4096, 50
    m = models.load(name, 0.05)
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    proj = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
    for seed in (3, 4):
        xi = proj(torch.tensor(np.random.default_rng(20250629 + seed).normal(0, np.sqrt(10.003), (n, 66))
                               .astype(np.float32)), proj.boundary(q0, np.zeros(6), np.zeros(6), n), 10).cuda()
        e = Engine(m, H, n, Pd)
        st = torch.zeros(n, dtype=torch.int32, device="cuda")
        e.rollout_cost(xi, MPCR_LAYOUT_XI, q0, (20., 3., 80.), (-0.3, -0.3, 0.5), (0., 1., 0., 0.), status=st)
        s = st.cpu().numpy()
        mx = (s >> 2) & 255
        print(f"{name} seed {seed}: mean rows {np.mean(s >> 11) / H:.1f}  max-rows pct50/99/99.9/max "
              f"{np.percentile(mx, 50):.0f}/{np.percentile(mx, 99):.0f}/{np.percentile(mx, 99.9):.0f}/{mx.max()}  "
              f"trunc {int((s & 1).sum())}")

"""Start independence of the kernel's hull supports for the library in
argv[1] (diagnostic; tests/test_gpu_parity.py::test_kernel_support_is_start_independent
at more shapes): the dual arm rolled out with the engine's start table and
with hashed starts (mpcr_set_hull_start_scramble, seeds 1..S), candidates
whose cost4 / theta / status differ, and the worst relative cost change.

    S=2 python tools/scramble_check.py build_variants/x.so
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from manipulator_mujoco_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
import torch  # noqa: E402

from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine  # noqa: E402
from test_gpu_parity import PT, Q0, QT, W, projected_xi  # noqa: E402

lib = _lib.load()
m = models.load("dual_arm", 0.05)
for n, H in ((1024, 50), (4096, 100)):
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 4, torch.device("cuda:0"))
    out = []
    for seed in range(int(os.environ.get("S", 2)) + 1):
        prev = lib.mpcr_set_hull_start_scramble(seed)
        try:
            e = Engine(m, H, n, Pd)
        finally:
            lib.mpcr_set_hull_start_scramble(prev)
        st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
        th = torch.empty((n, 6 * H), device="cuda:0")
        c = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, theta=th, status=st).clone()
        torch.cuda.synchronize()
        out.append((c.cpu().numpy(), th.cpu().numpy(), st.cpu().numpy()))
        del e
    ca, ta, sa = out[0]
    for seed, (cb, tb, sb) in enumerate(out[1:], 1):
        diff = (ca != cb).any(axis=1) | (ta != tb).any(axis=1) | (sa != sb)
        rel = np.abs(ca[:, 0].astype(np.float64) - cb[:, 0]) / np.abs(ca[:, 0])
        print(f"{os.path.basename(sys.argv[1])} {n}x{H} seed {seed}: {int(diff.sum())}/{n} candidates differ "
              f"(status {int((sa != sb).sum())}), worst cost rel {rel.max():.1e}, idx {np.where(diff)[0][:8].tolist()}",
              flush=True)

"""Time one libmpcr variant (path in argv[1]) on the C3 bench workload; prints
median kernel ms over R repetitions (HIP events on the launch stream)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from manipulator_mujoco_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
import torch  # noqa: E402

from manipulator_mujoco_amd import basis, models  # noqa: E402
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine  # noqa: E402
from manipulator_mujoco_amd.projection import ProjectionFilter  # noqa: E402

name = os.environ.get("MODEL", "scene_mjx")
n, H = int(os.environ.get("N", 4096)), int(os.environ.get("H", 50))
m = models.load(name, 0.05)
_, P, Pd, Pdd = basis.planner_basis(H, 0.05)
q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
proj = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
xi = proj(torch.tensor(np.random.default_rng(20250632).normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)),
          proj.boundary(q0, np.zeros(6), np.zeros(6), n), 10).cuda()
e = Engine(m, H, n, Pd)
st = torch.zeros(n, dtype=torch.int32, device="cuda")
c4 = torch.empty((n, 4), device="cuda")
th = torch.empty((n, 6 * H), device="cuda")
td = torch.empty((n, 6 * H), device="cuda")
if os.environ.get("THETA", "1") == "0":  # traffic attribution: no theta / thetadot outputs
    th = td = None
key = torch.empty(1, dtype=torch.int64, device="cuda")
args = (xi, MPCR_LAYOUT_XI, q0, (20., 3., 80.), (-0.3, -0.3, 0.5), (0., 1., 0., 0.))
for _ in range(2):
    e.rollout_cost(*args, cost4=c4, theta=th, thetadot=td, best_key=key)
torch.cuda.synchronize()
ts = []
for _ in range(int(os.environ.get("R", 10))):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    e.rollout_cost(*args, cost4=c4, theta=th, thetadot=td, best_key=key)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
occ = ""
lib = _lib.load()
if hasattr(lib, "mpcr_rollout_occupancy"):
    import ctypes
    info = (ctypes.c_int * 6)()
    lib.mpcr_rollout_occupancy.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    if lib.mpcr_rollout_occupancy(0, info) == 0:
        occ = (f" [narrow {info[0]} blocks/CU, {info[1]} B LDS, {info[2]} VGPR;"
               f" wide {info[3]} blocks/CU, {info[4]} B LDS, {info[5]} VGPR]")
e.rollout_cost(*args, cost4=c4, theta=th, thetadot=td, best_key=key, status=st)
sv = st.cpu().numpy()
rows = f" rows/step {float((sv >> 11).mean()) / H:.1f} max-rows p50/p90/p99 " + "/".join(
    str(int(np.percentile((sv >> 2) & 255, q))) for q in (50, 90, 99))
print(f"{os.path.basename(sys.argv[1])}{occ}{rows} {name} median {np.median(ts):.3f} ms min {np.min(ts):.3f} "
      f"-> {n / np.median(ts) * 1e3:.0f} rollouts/s  cost0 {float(c4[:, 0].sum()):.6e}")
if os.environ.get("SAVE"):  # outputs of the last launch, for bitwise comparisons between variants
    np.savez(os.environ["SAVE"], c4=c4.cpu().numpy(), th=None if th is None else th.cpu().numpy(), st=sv)

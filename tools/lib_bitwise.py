"""Are two libmpcr builds bitwise the same on a batch?  (diagnostic)

    python tools/lib_bitwise.py A.so B.so [model=scene_mjx] [n=4096] [H=50]

Each library runs in its own process (the bench's synthetic projected
inputs, cost4 / theta / status written to gpurun_out/); the parent compares
them bit for bit and prints how many candidates differ and by how much."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(so, model, n, H, out):
    sys.path.insert(0, ROOT)
    from manipulator_mujoco_amd import _lib
    _lib.LIB_PATH = os.path.abspath(so)
    import torch

    from manipulator_mujoco_amd import basis, models
    from manipulator_mujoco_amd.engine import MPCR_LAYOUT_XI, Engine
    from manipulator_mujoco_amd.projection import ProjectionFilter
    m = models.load(model, 0.05)
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    proj = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
    xi = proj(torch.tensor(np.random.default_rng(20250632).normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32)),
              proj.boundary(q0, np.zeros(6), np.zeros(6), n), 10).cuda()
    e = Engine(m, H, n, Pd)
    c4 = torch.empty((n, 4), device="cuda")
    th = torch.empty((n, 6 * H), device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    e.rollout_cost(xi, MPCR_LAYOUT_XI, q0, (20., 3., 80.), (-0.3, -0.3, 0.5), (0., 1., 0., 0.), cost4=c4, theta=th,
                   status=st)
    torch.cuda.synchronize()
    np.savez(out, cost4=c4.cpu().numpy(), theta=th.cpu().numpy(), status=st.cpu().numpy())


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), sys.argv[6])
    a, b = sys.argv[1], sys.argv[2]
    kw = dict(x.split("=") for x in sys.argv[3:])
    model, n, H = kw.get("model", "scene_mjx"), int(kw.get("n", 4096)), int(kw.get("H", 50))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    outs = []
    for k, so in enumerate((a, b)):
        out = os.path.join(ROOT, "gpurun_out", f"bitwise_{k}.npz")
        subprocess.run([sys.executable, __file__, "--child", so, model, str(n), str(H), out], check=True)
        outs.append(np.load(out))
    ca, cb = outs[0]["cost4"].astype(np.float64), outs[1]["cost4"].astype(np.float64)
    diff = (ca != cb).any(axis=1) | (outs[0]["theta"] != outs[1]["theta"]).any(axis=1)
    rel = np.abs(ca[:, 0] - cb[:, 0]) / np.abs(ca[:, 0])
    print(f"{os.path.basename(a)} vs {os.path.basename(b)} on {model} {n} x {H}: {int(diff.sum())} candidates differ, "
          f"worst cost rel {rel.max():.2e}, status equal {bool((outs[0]['status'] == outs[1]['status']).all())}")


if __name__ == "__main__":
    main()

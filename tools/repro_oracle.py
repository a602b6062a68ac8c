"""Run the fp64 oracle's conditioning probes on saved GPU-projected inputs (CPU only, diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from manipulator_mujoco_amd import basis, models  # noqa: E402
import parity_util as pu  # noqa: E402
H, n, workers = 100, 256, int(sys.argv[2])
pu.WORKERS = workers
m = models.load("dual_arm", 0.05)
_, P, Pd, Pdd = basis.planner_basis(H, 0.05)
xi = np.load(sys.argv[1])
td = np.einsum("tk,njk->njt", Pd, xi.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
o, sens = pu.conditioning(m, td, seed=H)
print("ok", workers, o["cost4"][:3, 0])

"""Save the projected xi the GPU parity tests draw (tests/test_gpu_parity.py::projected_xi) for CPU repro."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import torch  # noqa: E402
from test_gpu_parity import projected_xi  # noqa: E402
n, H, seed = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
np.save(sys.argv[4], projected_xi(n, H, seed, torch.device("cuda:0")).cpu().numpy())

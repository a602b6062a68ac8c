"""Drop-in ``cem_planner`` (reference: SBP/mjx_planner.py:17-406).

Same constructor keywords and the same ``compute_cem`` 9-tuple, so
``run_mpc_planner.py`` / ``mpc_planner.run_cem_planner`` only swap the import.
Per CEM iteration (``cem_iter``, :337-362), every step a HIP kernel of
libmpcr on the current torch stream (no host round trip inside the loop):

  1. L = chol(cov + 0.003 I)                                (:312-316)  mpcr_cem_factor
  2. MVN samples xi = mean + z L^T fused with the ADMM
     projection filter                                      (:180-249)  mpcr_cem_sample_project
  3. thetadot = A_thetadot xi, H physics steps, cost        (:348-354)  mpcr_rollout_cost
  4. elites (stable argsort, NaN last)                      (:305-310)  mpcr_topk
  5. weighted mean/cov update                               (:318-335)  mpcr_cem_update
and finally the best candidate of the last iteration through the packed
argmin key the rollout kernel reduces with an atomic min (:395-402).

Reference behaviours kept on purpose, each behind a flag:
  * elites are gathered from the *unprojected* samples (``elite_from_filtered=False``)
  * the sampling key is not advanced across calls (fixed ``seed`` per call)
  * ``init_vel`` only enters the boundary vector (the rollout overwrites qvel[:6])
  * a NaN cost wins the final argmin, sorts last among elites.
The MVN draws use Philox4x32-10 keyed by (seed, iteration), not JAX's
threefry, so samples are statistically equivalent but not bit-identical to
the reference's.
"""

from __future__ import annotations

import os
import time

import numpy as np

from . import _lib, basis, models
from .cem import CemContext, topk
from .engine import MPCR_LAYOUT_XI, Engine
from .mjcf import load_model

DEFAULT_MODEL = "planner_scene"  # SBP/ur5e_hande_mjx/scene.xml (:100)


def _resolve_model(model_path, timestep):
    if model_path is None:
        return models.load(DEFAULT_MODEL, timestep)
    if model_path in models.BUNDLES:
        return models.load(model_path, timestep)
    return load_model(model_path, timestep)


class cem_planner:  # noqa: N801 (reference name)
    def __init__(self, num_dof=None, num_batch=None, num_steps=None, timestep=None, maxiter_cem=None,
                 num_elite=None, w_pos=None, w_rot=None, w_col=None, maxiter_projection=None, *,
                 model_path=None, device=None, seed=0, elite_from_filtered=False, verbose=True):
        import torch

        if not torch.cuda.is_available():
            raise _lib.MpcrError("cem_planner needs a gfx950 GPU (no CPU fallback)")
        self.num_dof = int(num_dof)
        self.num_batch = int(num_batch)
        self.num = int(num_steps)
        self.t = float(timestep)
        self.maxiter_cem = int(maxiter_cem)
        self.maxiter_projection = int(maxiter_projection) if maxiter_projection is not None else 0
        self.num_elite = float(num_elite)
        self.ellite_num = int(self.num_elite * self.num_batch)
        self.cost_weights = {"w_pos": w_pos, "w_rot": w_rot, "w_col": w_col}
        self.seed = int(seed)
        self.elite_from_filtered = bool(elite_from_filtered)
        # CEM constants (:84-97)
        self.v_max, self.a_max, self.p_max = 0.8, 1.8, np.pi
        self.alpha_mean, self.alpha_cov, self.lamda = 0.6, 0.6, 10.0

        self.t_fin = self.num * self.t
        self.tot_time, self.P, self.Pdot, self.Pddot = basis.planner_basis(self.num, self.t)
        self.nvar_single = self.P.shape[1]
        self.nvar = self.nvar_single * self.num_dof

        dev = int(device) if device is not None else int(os.environ.get("LOCAL_RANK", 0))
        self.device = torch.device("cuda", dev)
        self.model = _resolve_model(model_path, self.t)
        self.model_path = getattr(self.model, "source", model_path)
        if self.model.nctrl != self.num_dof:
            raise ValueError(f"model controls {self.model.nctrl} dofs, num_dof={self.num_dof}")
        self.data = None  # the closed-loop plant lives in mpc.py (Plant)
        self.hande_id = self.model.hande_body
        self.tcp_id = self.model.tcp_site
        self.engine = Engine(self.model, self.num, self.num_batch, self.Pdot, device=dev)
        self.cem = CemContext(self.P, self.Pdot, self.Pddot, self.num_dof, self.num_batch, device=dev)
        f32 = dict(dtype=torch.float32, device=self.device)
        N = self.num_batch
        self._key = torch.empty(1, dtype=torch.int64, device=self.device)
        self._eye = torch.eye(self.nvar, **f32)
        self._mean = torch.empty(self.nvar, **f32)
        self._cov = torch.empty((self.nvar, self.nvar), **f32)
        self._xs = torch.empty((N, self.nvar), **f32)  # xi_samples
        self._xf = torch.empty((N, self.nvar), **f32)  # xi_filtered
        self._idx = torch.empty(max(self.ellite_num, 1), dtype=torch.int32, device=self.device)
        self._beq = torch.empty(5 * self.num_dof, **f32)
        if verbose:
            self.print_info()

    def print_info(self):
        name = _lib.load()
        del name
        print(f"\n Default backend: gfx950 (libmpcr)\n Model path: {self.model_path}"
              f"\n Timestep: {self.t}\n CEM Iter: {self.maxiter_cem}\n Number of batches: {self.num_batch}"
              f"\n Number of steps per trajectory: {self.num}\n Time per trajectory: {self.t_fin}")

    # ------------------------------------------------------------------
    def compute_cem(self, xi_mean, init_pos=(1.5, -1.8, 1.75, -1.25, -1.6, 0.0), init_vel=None, init_acc=None,
                    target_pos=None, target_rot=None):
        """One MPC tick of CEM (SBP/mjx_planner.py:364-406). Returns the reference 9-tuple (numpy)."""
        import torch

        d = self.num_dof
        N, H, it_n = self.num_batch, self.num, self.maxiter_cem
        init_pos = np.asarray(init_pos, np.float64)[:d]
        init_vel = np.zeros(d) if init_vel is None else np.asarray(init_vel, np.float64)[:d]
        init_acc = np.zeros(d) if init_acc is None else np.asarray(init_acc, np.float64)[:d]
        target_pos = np.zeros(3) if target_pos is None else np.asarray(target_pos, np.float64)
        target_rot = np.zeros(4) if target_rot is None else np.asarray(target_rot, np.float64)
        w = (self.cost_weights["w_pos"], self.cost_weights["w_rot"], self.cost_weights["w_col"])
        f32 = dict(dtype=torch.float32, device=self.device)

        if self.ellite_num < 1:
            raise ValueError("num_elite * num_batch must select at least one elite")
        self._mean.copy_(torch.as_tensor(np.asarray(xi_mean, np.float32).reshape(self.nvar)))
        self._cov.copy_(10.0 * self._eye)  # xi_cov (:386)
        st = np.stack([init_pos, init_vel, init_acc, np.zeros(d), np.zeros(d)], axis=1)  # state_term (:374-384)
        self._beq.copy_(torch.as_tensor(st.reshape(5 * d).astype(np.float32)))  # compute_boundary_vec (:174-178)
        bounds = (self.v_max, self.a_max, self.p_max)
        thetadot = torch.empty((it_n, N, d * H), **f32)
        theta = torch.empty((it_n, N, d * H), **f32)
        costs = torch.empty((it_n, N, 4), **f32)
        src = self._xf if self.elite_from_filtered else self._xs
        for it in range(it_n):
            self.cem.factor(self._cov, 0.003)
            self.cem.sample_project(N, self._mean, self.seed, it, self._beq, self.maxiter_projection, bounds,
                                    rho=1.0, xi_samples=self._xs, out=self._xf)
            self.engine.rollout_cost(self._xf, MPCR_LAYOUT_XI, init_pos, w, target_pos, target_rot,
                                     cost4=costs[it], theta=theta[it], thetadot=thetadot[it],
                                     best_key=self._key if it == it_n - 1 else None)
            topk(self.engine, costs[it], self.ellite_num, stride=4, out=self._idx)
            self.cem.update(src, costs[it], 4, self._idx, self.lamda, self.alpha_mean, self.alpha_cov,
                            self._mean, self._cov, reg=1e-4)
        mean = self._mean
        key = int(self._key.item())
        idx, _ = _lib.decode_key(key & 0xFFFFFFFFFFFFFFFF)
        cost_min = torch.amin(costs[:, :, 0], dim=1)
        best = costs[-1, idx]
        best_vels = thetadot[-1, idx].reshape(d, H).T
        best_traj = theta[-1, idx].reshape(d, H).T
        out = (cost_min, best[1], best[2], best[3], best_vels, best_traj, mean, thetadot, theta)
        return tuple(o.cpu().numpy() for o in out)


def main():  # SBP/mjx_planner.py:408-428 (with its unpacking bug fixed)
    t0 = time.time()
    opt = cem_planner(num_dof=6, num_batch=2000, num_steps=50, maxiter_cem=30, w_pos=1, w_rot=0.5, w_col=10,
                      num_elite=0.05, timestep=0.05, maxiter_projection=10)
    t1 = time.time()
    out = opt.compute_cem(np.zeros(opt.nvar))
    print(f"Total time: {round(time.time() - t0, 2)}s")
    print(f"Compute CEM time: {round(time.time() - t1, 2)}s")
    return out


if __name__ == "__main__":
    main()

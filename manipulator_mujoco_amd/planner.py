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

With ranks > 1 (``group``), each rank owns num_batch/ranks candidates
(Philox draws keyed by the global candidate index, so the samples are the
single-GPU ones), and steps 4-5 become local top-E -> all-gather of the elite
rows -> the same global top-E and update on every rank (dist.gather_elites);
the best candidate is one 8-byte MIN all-reduce.  With
``graph=True`` the per-iteration kernel sequences are captured in HIP graphs
on the first call (per-tick inputs live in static device buffers).

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
    """Reference constructor keywords plus, keyword-only:

    model_path          MJCF path or bundled model name (default: the
                        planner scene the reference hard-wires, :100)
    device              GPU ordinal (default LOCAL_RANK)
    seed                Philox key of the MVN draws (fixed per call, §0.6)
    elite_from_filtered gather elites from the projected samples instead
    graph               capture each CEM iteration's kernels in HIP graphs on
                        the first call and replay them on later calls
    group               torch.distributed process group: ``num_batch`` is
                        the GLOBAL batch, sharded evenly over the ranks
                        (SURVEY.md §8e); None = single GPU unless an
                        initialised default group has more than one rank
    gather_rollouts     with ranks > 1, all-gather the full thetadot/theta
                        arrays of the 9-tuple (default: this rank's shard)
    return_rollouts     False: the 9-tuple's thetadot/theta (iters x N x 6H,
                        what the closed loop discards) are returned as None
                        instead of being copied to the host every tick
    capture_exchange    with graph=True and an RCCL group, capture the elite
                        all-gathers in the tick's graph (default); False
                        captures each iteration's device segment and runs the
                        exchange eagerly between the replays (as with gloo)
    """

    def __init__(self, num_dof=None, num_batch=None, num_steps=None, timestep=None, maxiter_cem=None,
                 num_elite=None, w_pos=None, w_rot=None, w_col=None, maxiter_projection=None, *,
                 model_path=None, device=None, seed=0, elite_from_filtered=False, graph=False, group=None,
                 gather_rollouts=False, return_rollouts=True, capture_exchange=True, verbose=True):
        import torch
        import torch.distributed as tdist

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
        self.graph = bool(graph)
        self.gather_rollouts = bool(gather_rollouts)
        self.return_rollouts = bool(return_rollouts)
        self.capture_exchange = bool(capture_exchange)
        # CEM constants (:84-97)
        self.v_max, self.a_max, self.p_max = 0.8, 1.8, np.pi
        self.alpha_mean, self.alpha_cov, self.lamda = 0.6, 0.6, 10.0

        # candidate shards
        self.group = group
        if group is None and tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1:
            self.group = tdist.group.WORLD
        self.world = tdist.get_world_size(self.group) if self.group is not None else 1
        self.rank = tdist.get_rank(self.group) if self.group is not None else 0
        if self.num_batch % self.world:
            raise ValueError(f"num_batch={self.num_batch} must split evenly over {self.world} ranks")
        self.n_local = self.num_batch // self.world
        self.exchange = self.world > 1  # elites through gather_elites (forced on one rank in tests)
        self.index_base = self.rank * self.n_local

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
        self.data = None  # the closed-loop plant: mpc_planner.run_cem_planner (engine.Plant)
        self.hande_id = self.model.hande_body
        self.tcp_id = self.model.tcp_site
        n = self.n_local
        self.engine = Engine(self.model, self.num, n, self.Pdot, device=dev)
        self.cem = CemContext(self.P, self.Pdot, self.Pddot, self.num_dof, n, device=dev)
        f32 = dict(dtype=torch.float32, device=self.device)
        H, it_n = self.num, self.maxiter_cem
        self._key = torch.empty(1, dtype=torch.int64, device=self.device)
        self._eye10 = 10.0 * torch.eye(self.nvar, **f32)  # xi_cov (:386)
        self._mean = torch.empty(self.nvar, **f32)
        self._cov = torch.empty((self.nvar, self.nvar), **f32)
        self._xs = torch.empty((n, self.nvar), **f32)  # xi_samples
        self._xf = torch.empty((n, self.nvar), **f32)  # xi_filtered
        self._idx = torch.empty(max(self.ellite_num, 1), dtype=torch.int32, device=self.device)
        self._beq = torch.empty(5 * self.num_dof, **f32)
        self._par = torch.zeros(20, **f32)  # init_pos | weights | target (Engine.params)
        self._thetadot = torch.empty((it_n, n, self.num_dof * H), **f32)
        self._theta = torch.empty((it_n, n, self.num_dof * H), **f32)
        self._costs = torch.empty((it_n, n, 4), **f32)
        self._mean_in = torch.empty(self.nvar, **f32)
        self._graphs = None
        if verbose and self.rank == 0:
            self.print_info()

    def print_info(self):
        _lib.load()
        print(f"\n Default backend: gfx950 (libmpcr)\n Model path: {self.model_path}"
              f"\n Timestep: {self.t}\n CEM Iter: {self.maxiter_cem}\n Number of batches: {self.num_batch}"
              f"\n Number of steps per trajectory: {self.num}\n Time per trajectory: {self.t_fin}"
              + (f"\n Ranks: {self.world} x {self.n_local} candidates" if self.world > 1 else ""))

    # ------------------------------------------------------------------
    # one CEM iteration = two device segments around the (multi-rank) elite
    # exchange; each segment is a fixed kernel sequence on the current
    # stream, so it can be captured in a HIP graph and replayed
    def _seg_sample_rollout(self, it):
        """compute_xi_samples + projection + rollout + cost (:345-354)."""
        bounds = (self.v_max, self.a_max, self.p_max)
        if it == 0:
            self._mean.copy_(self._mean_in)
            self._cov.copy_(self._eye10)
        self.cem.factor(self._cov, 0.003)
        self.cem.sample_project(self.n_local, self._mean, self.seed, it, self._beq, self.maxiter_projection, bounds,
                                rho=1.0, xi_samples=self._xs, out=self._xf, index_base=self.index_base)
        last = it == self.maxiter_cem - 1
        self.engine.rollout_cost_dp(self._xf, MPCR_LAYOUT_XI, self._par, self._costs[it], theta=self._theta[it],
                                    thetadot=self._thetadot[it], best_key=self._key if last else None,
                                    index_base=self.index_base)

    def _seg_local_update(self, it):
        """compute_ellite_samples + compute_mean_cov on one rank (:355-360)."""
        src = self._xf if self.elite_from_filtered else self._xs
        topk(self.engine, self._costs[it], self.ellite_num, stride=4, out=self._idx)
        self.cem.update(src, self._costs[it], 4, self._idx, self.lamda, self.alpha_mean, self.alpha_cov,
                        self._mean, self._cov, reg=1e-4)

    def _topk_fn(self, cost, k):
        return topk(self.engine, cost, k, stride=1)

    def _exchange_update(self, it):
        """Sharded elites: all-gather local top-E rows, select, replicated update."""
        from .dist import gather_elites
        src = self._xf if self.elite_from_filtered else self._xs
        g_cost, g_xi, sel = gather_elites(self._costs[it, :, 0].contiguous(), src, self.ellite_num, self._topk_fn,
                                          group=self.group)
        self.cem.update(g_xi, g_cost, 1, sel, self.lamda, self.alpha_mean, self.alpha_cov, self._mean, self._cov,
                        reg=1e-4)

    def _run_iterations(self):
        import torch
        it_n = self.maxiter_cem
        if not self.graph:
            for it in range(it_n):
                self._seg_sample_rollout(it)
                if not self.exchange:
                    self._seg_local_update(it)
                else:
                    self._exchange_update(it)
            return
        if self._graphs is None:
            # warm up on a side stream (allocator / library state), then capture
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._run_eager_once()
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            graphs = []
            if not self.exchange or (self.capture_exchange and self._exchange_capturable()):
                # the whole tick in one graph; with an RCCL group the elite
                # all-gathers are captured too (device buffers, stream-ordered)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for it in range(it_n):
                        self._seg_sample_rollout(it)
                        if not self.exchange:
                            self._seg_local_update(it)
                        else:
                            self._exchange_update(it)
                graphs.append(g)
            else:  # gloo (host-staged) exchange: device segments in graphs, the exchange between them eager
                for it in range(it_n):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        self._seg_sample_rollout(it)
                    graphs.append(g)
            self._graphs = graphs
        if len(self._graphs) == 1:
            self._graphs[0].replay()
        else:
            for it in range(it_n):
                self._graphs[it].replay()
                self._exchange_update(it)

    def _exchange_capturable(self):
        """RCCL collectives on device tensors can be captured into the tick's
        graph; host-staged (gloo) ones cannot."""
        import torch.distributed as dist
        return dist.get_backend(self.group) == "nccl"

    def _run_eager_once(self):
        graph, self.graph = self.graph, False
        try:
            self._run_iterations()
        finally:
            self.graph = graph

    def compute_cem(self, xi_mean, init_pos=(1.5, -1.8, 1.75, -1.25, -1.6, 0.0), init_vel=None, init_acc=None,
                    target_pos=None, target_rot=None):
        """One MPC tick of CEM (SBP/mjx_planner.py:364-406). Returns the reference 9-tuple (numpy)."""
        import torch

        from . import dist as mdist

        d = self.num_dof
        H = self.num
        init_pos = np.asarray(init_pos, np.float64)[:d]
        init_vel = np.zeros(d) if init_vel is None else np.asarray(init_vel, np.float64)[:d]
        init_acc = np.zeros(d) if init_acc is None else np.asarray(init_acc, np.float64)[:d]
        target_pos = np.zeros(3) if target_pos is None else np.asarray(target_pos, np.float64)
        target_rot = np.zeros(4) if target_rot is None else np.asarray(target_rot, np.float64)
        w = (self.cost_weights["w_pos"], self.cost_weights["w_rot"], self.cost_weights["w_col"])

        if self.ellite_num < 1:
            raise ValueError("num_elite * num_batch must select at least one elite")
        # per-tick inputs into the static device buffers the (captured) kernels read
        self._mean_in.copy_(torch.as_tensor(np.asarray(xi_mean, np.float32).reshape(self.nvar)))
        st = np.stack([init_pos, init_vel, init_acc, np.zeros(d), np.zeros(d)], axis=1)  # state_term (:374-384)
        self._beq.copy_(torch.as_tensor(st.reshape(5 * d).astype(np.float32)))  # compute_boundary_vec (:174-178)
        self._par.copy_(torch.as_tensor(Engine.params(init_pos, w, target_pos, target_rot)))
        self._run_iterations()

        costs, theta, thetadot = self._costs, self._theta, self._thetadot
        cost_min = torch.amin(costs[:, :, 0], dim=1)
        if self.world > 1:
            mdist.allreduce_min_key(self._key, group=self.group)
            cost_min = torch.as_tensor(mdist.allgather_min(cost_min, group=self.group))
        idx, _ = _lib.decode_key(int(self._key.item()) & 0xFFFFFFFFFFFFFFFF)
        owner, li = divmod(idx, self.n_local)
        best = torch.empty(4 + 2 * d * H, dtype=torch.float32, device=self.device)
        if owner == self.rank:
            best[:4] = costs[-1, li]
            best[4:4 + d * H] = thetadot[-1, li]
            best[4 + d * H:] = theta[-1, li]
        if self.world > 1:
            mdist.broadcast(best, owner, group=self.group)
            if self.gather_rollouts and self.return_rollouts:
                theta, thetadot = (self._gather_all(x) for x in (theta, thetadot))
        if not self.return_rollouts:
            theta = thetadot = None
        best_vels = best[4:4 + d * H].reshape(d, H).T
        best_traj = best[4 + d * H:].reshape(d, H).T
        out = (cost_min, best[1], best[2], best[3], best_vels, best_traj, self._mean, thetadot, theta)
        return tuple(o.cpu().numpy() if isinstance(o, torch.Tensor) else o for o in out)

    def _gather_all(self, x):
        from .dist import all_gather
        it_n, n, c = x.shape
        return all_gather(x, self.group).permute(1, 0, 2, 3).reshape(it_n, self.world * n, c)


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

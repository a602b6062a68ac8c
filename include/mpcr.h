/*
 * mpcr.h — C ABI of libmpcr, the MI355X rollout engine behind the drop-in
 * cem_planner (manipulator_mujoco_amd/planner.py).
 *
 * Plain C: pointers + sizes, no torch/HIP types in the signatures.  Every
 * function returns 0 on success or a negative MPCR_E* code; the message of
 * the last failure on the calling thread is available from
 * mpcr_last_error().  Engines are independent (one per host thread / stream);
 * there is no global mutable state besides the thread-local error string and
 * the process-wide two-wave batch threshold (mpcr_set_two_wave_max_n).
 *
 * Reference interface each entry point replaces (file:line in
 * /root/reference/sampling_based_planner/):
 *   mpcr_model_*          MjModel.from_xml_path + mjx.put_model/put_data +
 *                         jit(mjx.forward) template          mjx_planner.py:100-108
 *   mpcr_engine_create    cem_planner.__init__ (basis P/Pdot, mask, ids)
 *                                                             mjx_planner.py:19-126
 *   mpcr_rollout_cost     A_thetadot @ xi + compute_rollout_batch (vmap of
 *                         compute_rollout_single / lax.scan of mjx_step) +
 *                         compute_cost_batch                  mjx_planner.py:348-354,
 *                                                             251-303
 *   best_key / mpcr_argmin / mpcr_best_key_decode
 *                         idx_min = argmin(cost_batch[-1])    mjx_planner.py:395
 *   mpcr_topk             compute_ellite_samples argsort     mjx_planner.py:305-310
 *   mpcr_cem_create       cem_planner.__init__ basis + get_Q_inv mjx_planner.py:40-46,
 *                                                             140-172
 *   mpcr_cem_factor       the Cholesky inside jax.random.multivariate_normal
 *                                                             mjx_planner.py:312-316
 *   mpcr_cem_sample_project / mpcr_project
 *                         compute_xi_samples + compute_projection_filter
 *                         (+ compute_projection)              mjx_planner.py:312-316,
 *                                                             180-249
 *   mpcr_cem_update       compute_mean_cov + comp_prod       mjx_planner.py:318-335
 *   mpcr_rollout_cost_dp  mpcr_rollout_cost with the per-tick arguments
 *                         (init_pos, weights, target pose) read from device
 *                         memory, so a whole cem_iter can be graph-captured
 *                         once and replayed every tick       mjx_planner.py:364-406
 *   mpcr_plant_*          the closed-loop plant: data.qvel[:num_dof] = thetadot;
 *                         mujoco.mj_step / mj_forward on the planner's model
 *                         (CPU MjData in the reference)      mpc_planner.py:109-114,
 *                                                             120-121,173-184
 */
#ifndef MPCR_H_
#define MPCR_H_

#include <stddef.h>
#include <stdint.h>

#include "mpcr_model.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version.  4 (round 6): model format v9 without the support start
   table, which the engine builds (mpcr_model_hull_starts).  3: bit 10 reports a lost two-wave handshake
   (MPCR_STATUS_SYNC), so rows-summed moved to bit 11.  2 (round 4): the
   max-rows field widened to 8 bits (version 1: 6 bits << 2, sum << 8).
   Decode with the accessors below, not raw shifts. */
#define MPCR_ABI_VERSION 4

/* the per-candidate status word of mpcr_rollout_cost / _dp */
#define MPCR_STATUS_TRUNCATED(s) ((s) & 1)                  /* constraint rows truncated  */
#define MPCR_STATUS_NONFINITE(s) (((s) >> 1) & 1)           /* non-finite state           */
#define MPCR_STATUS_MAX_ROWS(s) (((s) >> 2) & 255)          /* busiest step's rows (<= 255) */
#define MPCR_STATUS_SYNC(s) (((s) >> 10) & 1)               /* two-wave handshake timed out:
                                                                the candidate's outputs are void
                                                                and its cost is +inf */
#define MPCR_STATUS_ROWS_SUM(s) ((unsigned)(s) >> 11)       /* rows summed over the horizon */
#define MPCR_STATUS_FAILED(s) (((s) & 2) | ((s) & (1 << 10)))  /* no usable result */

enum {
  MPCR_OK = 0,
  MPCR_EINVAL = -1,   /* bad argument / shape                      */
  MPCR_EMODEL = -2,   /* model blob invalid or over capacity        */
  MPCR_EHIP = -3,     /* HIP runtime error                          */
  MPCR_ENOMEM = -4,
  MPCR_ENODEV = -5    /* no gfx950 device                           */
};

/* input layouts for mpcr_rollout_cost */
enum {
  MPCR_LAYOUT_XI = 0,       /* n x (nctrl*nbasis) Bernstein coefficients,
                               joint-major (xi_filtered, mjx_planner.py:348) */
  MPCR_LAYOUT_THETADOT = 1  /* n x (nctrl*H) joint velocities, joint-major */
};

/* flags */
enum {
  MPCR_F_DEVICE_PTRS = 1 << 0, /* every array argument is a device pointer  */
  MPCR_F_RESET_BEST  = 1 << 1, /* set *best_key to UINT64_MAX before launch */
  MPCR_F_SYNC        = 1 << 2  /* block until the stream is idle           */
};

typedef struct mpcr_model mpcr_model;   /* opaque host model handle */
typedef struct mpcr_engine mpcr_engine; /* opaque device engine      */
typedef struct mpcr_cem mpcr_cem;       /* opaque CEM context (projection tables, Cholesky factor) */

const char* mpcr_last_error(void);
int mpcr_abi_version(void);
/* gfx target name of `device` (e.g. "gfx950") into buf */
int mpcr_device_arch(int device, char* buf, int buflen);

/* models: a serialised mpcr_model_t (see mpcr_model.h) */
int mpcr_model_from_blob(const void* blob, size_t nbytes, mpcr_model** out);
/* path: an MJCF scene (.xml, or any file starting with '<') -- compiled by
   the MJCF compiler of libmpcr_mjcf.so (include/mpcr_mjcf.h), dlopened from
   this library's directory on first use: MjModel.from_xml_path,
   SBP/mjx_planner.py:100-103 -- or a serialised mpcr_model_t blob.
   timestep > 0 overrides the model's (opt.timestep = dt, :102). */
int mpcr_model_load(const char* path, double timestep, mpcr_model** out);
int mpcr_model_set_timestep(mpcr_model* m, double timestep);
int mpcr_model_info(const mpcr_model* m, int* nq, int* nv, int* nslot, int* nctrl, int* npair);
void mpcr_model_free(mpcr_model* m);
/* The support start table an engine builds for m's convex hulls (model
   format v9 dropped it from the blob; engine.hip hull_start_table): R x R
   cells on each of the 6 cube faces (R = 0: the library's MPCR_LUT_R), cell
   (2 axis + negative) R^2 + iu R + iv (rollout.hip lut_cell), each naming
   the global hull vertex extreme along the cell centre (fp64; the lowest
   index among exact ties).  geom_adr[ngeom] (nullable) receives each geom's
   first cell (-1: no hull), cells and exact (nullable) every cell when cap
   holds the count -- exact[c] = 1 where the engine skips the climb (the
   start vertex beats each neighbour along every direction of the cell by the
   fp32 margin).  Returns the cell count (< 0: error).  Host only, no device
   (tests/test_hull_lut.py). */
int64_t mpcr_model_hull_starts(const mpcr_model* m, int R, int32_t* geom_adr, int32_t* cells, uint8_t* exact,
                               int64_t cap);
/* Test knob (the start-independence tests): engines created while seed != 0
   start every hull climb at a vertex of its hull hashed from (seed, geom,
   cell) instead of the extreme one.  Process-wide; returns the previous seed. */
uint64_t mpcr_set_hull_start_scramble(uint64_t seed);

/* engines: device copy of the model + the Pdot basis (horizon x nbasis,
   row-major fp32, bernstein_coeff_ordern_new(..)[1]) + scratch for max_n. */
int mpcr_engine_create(const mpcr_model* m, int device, int max_n, int horizon, const float* pdot,
                       int nbasis, mpcr_engine** out);
void mpcr_engine_free(mpcr_engine* e);

/* Fused basis -> H MuJoCo-semantics steps -> cost for n candidates.
   q0[nctrl]            initial joint positions (init_pos)
   w[3]                 (w_pos, w_rot, w_col)
   ptgt[3], qtgt[4]     target position / orientation (wxyz)
   cost4 [n x 4]        (cost, cost_g, cost_r, cost_c)          (required)
   theta [n x nctrl*H]  post-step joint positions, joint-major    (nullable)
   thetadot [n x nctrl*H] the applied joint velocities           (nullable)
   best_key             device uint64: atomic-min of
                        (ordered(cost) << 32 | (index_base + i)), NaN first (nullable)
   status [n]           per-candidate flags (bit0: constraint rows truncated,
                        bit1: non-finite state, bit10: two-wave handshake
                        lost) | (max constraint rows in one step, 8 bits
                        capped at 255, << 2) | (constraint rows summed over
                        the horizon << 11)                       (nullable)
   stream               hipStream_t or NULL (default stream)
   n = 0 is a no-op returning MPCR_OK (input and cost4 may then be NULL). */
int mpcr_rollout_cost(mpcr_engine* e, const float* input, int layout, int n, const double* q0,
                      const float* w, const float* ptgt, const float* qtgt, float* cost4, float* theta,
                      float* thetadot, uint64_t* best_key, int index_base, int* status, int flags,
                      void* stream);

/* Diagnostic: resident workgroups (= candidates) per CU, static LDS bytes and
   VGPRs of the two rollout kernel variants on `device`:
   info[6] = narrow (blocks, lds, vgprs), dual-arm class (blocks, lds, vgprs). */
int mpcr_rollout_occupancy(int device, int* info);
/* Narrow-variant batches of at most n candidates run two waves per candidate
   (the collision phase beside the dynamics; bitwise the one-wave results);
   dual-arm batches of at most min(n, 1024) too (MPCR_WPC2W_MAX_N overrides
   the 1024: four two-wave blocks per CU).  0 disables both.
   n < 0 only queries.  Returns the previous threshold (default: the build's
   MPCR_WPC2_MAX_N_DEFAULT, or the MPCR_WPC2_MAX_N environment variable).
   Process-wide (an atomic read by every engine's next launch; the
   environment is read once, when the library loads). */
int mpcr_set_two_wave_max_n(int n);
/* Kernel dispatches one mpcr_rollout_cost call over n candidates issues on
   this engine (1, or -- dual-arm batches above the resident-block count --
   one per horizon segment and candidate group, MPCR_SEG_STEPS /
   MPCR_SEG_GROUPS): a profiler's per-dispatch counters times *out are per
   call.  No GPU work. */
int mpcr_engine_dispatches(const mpcr_engine* e, int n, int* out);

/* Same as mpcr_rollout_cost with MPCR_F_DEVICE_PTRS, except that the
   per-call arguments are a device block read when the kernel runs:
   params[20] = init_pos[8] | (w_pos, w_rot, w_col, 0) | ptgt[3], 0 | qtgt[4]
   (wxyz, normalised by the kernel).  Graph-capturable. */
int mpcr_rollout_cost_dp(mpcr_engine* e, const float* input, int layout, int n, const float* params,
                         float* cost4, float* theta, float* thetadot, uint64_t* best_key, int index_base,
                         int* status, int flags, void* stream);

/* Closed-loop plant: one environment of the model, stepped by the rollout
   kernel (fp32 state resident on the device).  Created at the template
   state (qpos_init, qvel_init, zero warm start). */
typedef struct mpcr_plant mpcr_plant;
int mpcr_plant_create(const mpcr_model* m, int device, mpcr_plant** out);
void mpcr_plant_free(mpcr_plant* p);
/* Overwrite the state (NULL leaves a part unchanged): qpos[nq], qvel[nv],
   qacc_warmstart[nv]. */
int mpcr_plant_set_state(mpcr_plant* p, const double* qpos, const double* qvel, const double* qacc_warmstart);
/* Read qpos[nq], qvel[nv], qacc[nv] (of the last step / forward) and eef[7] =
   tcp site position | hande body quaternion (wxyz) evaluated at the state the
   last step / forward started from (mj_step's kinematics run before the
   integration).  NULL skips a part. */
int mpcr_plant_get_state(mpcr_plant* p, double* qpos, double* qvel, double* qacc, double* eef);
/* commit = 1: mj_step with qvel[:nctrl] = qvel_ctrl first (NULL keeps the
   current velocities).  commit = 0: mj_forward, the state is not advanced.
   Blocks until done. */
int mpcr_plant_step(mpcr_plant* p, const double* qvel_ctrl, int commit, void* stream);

/* argmin over cost[i*stride] with NaN-first / first-index semantics
   (jnp.argmin).  key_out (device, nullable) receives the packed key. */
int mpcr_argmin(mpcr_engine* e, const float* cost, int stride, int n, int index_base, uint64_t* key_out,
                int* idx_out, float* val_out, int flags, void* stream);

/* decode a packed best key */
void mpcr_best_key_decode(uint64_t key, int* idx, float* cost);

/* indices of the k smallest of cost[i*stride], ascending, NaN last, ties by
   index, -0 == +0 (jnp.argsort is stable): compute_ellite_samples.
   k <= min(n, 4096).  Host pointers: n <= max_n and stride <= 4. */
int mpcr_topk(mpcr_engine* e, const float* cost, int stride, int n, int k, int* idx_out, int flags,
              void* stream);

/* ---- the CEM distribution step (device pointers only: MPCR_F_DEVICE_PTRS) ----
   num_dof <= 8 joints, nbasis = 11 (order-10 Bernstein), P/Pdot/Pddot
   horizon x nbasis row-major fp64 (bernstein_coeff_ordern_new).  qinv
   (nullable): the (nv+5nd)^2 fp64 KKT inverse; NULL computes get_Q_inv's
   matrix (fp32 Gram blocks, fp64 inverse, rho_ineq = 1). */
int mpcr_cem_create(int device, int num_dof, int horizon, int nbasis, const double* P, const double* Pdot,
                    const double* Pddot, const double* qinv, int max_n, mpcr_cem** out);
void mpcr_cem_free(mpcr_cem* c);

/* L = chol(cov + reg I) (nv x nv fp32, reg = 0.003 in the reference) into the
   context, for the next sampling call.  Non-PD input yields NaN samples. */
int mpcr_cem_factor(mpcr_cem* c, const float* cov, float reg, int flags, void* stream);

/* Fused sampling + projection for n candidates.
   mean != NULL: xi_samples = mean + z L^T with z ~ N(0, I) from Philox4x32-10
     keyed by seed, counter = (call counter), element (candidate, joint, block)
     -- independent of the launch shape; written to xi_samples if non-NULL.
   mean == NULL: the samples are read from xi_in (n x nv).
   Then maxiter ADMM iterations onto |Pdot xi| <= bounds[0], |Pddot xi| <=
   bounds[1], |P xi| <= bounds[2] with the boundary equalities b_eq
   (n x 5nd, per joint (theta0, thetadot0, thetaddot0, 0, 0); beq_stride 0 =
   one row shared by all candidates) and multiplier step rho; maxiter = 0
   returns the samples.  xi_out n x nv. */
int mpcr_cem_sample_project(mpcr_cem* c, int n, const float* mean, uint64_t seed, uint64_t counter,
                            int index_base, const float* xi_in, float* xi_samples, const float* b_eq, int beq_stride, int maxiter,
                            const float* bounds, float rho, float* xi_out, int flags, void* stream);
/* projection only (compute_projection_filter) */
int mpcr_project(mpcr_cem* c, const float* xi, const float* b_eq, int beq_stride, int n, int maxiter,
                 const float* bounds, float rho, float* xi_out, int flags, void* stream);

/* Elite moments, in place: w = exp(-(c - min c)/lamda) over the k elites
   xi[elite_idx[i]] (n x nv rows), cost[elite_idx[i]*stride];
   mean <- (1-alpha_mean) mean + alpha_mean sum(w xi)/sum(w);
   cov  <- (1-alpha_cov) cov + alpha_cov sum(w d d^T)/sum(w) + reg I, d = xi - mean_new.
   k <= 4096. */
int mpcr_cem_update(mpcr_cem* c, const float* xi, int n, const float* cost, int stride, const int* elite_idx, int k,
                    float lamda, float alpha_mean, float alpha_cov, float reg, float* mean, float* cov, int flags,
                    void* stream);

/* ---- multi-GPU exchange over RCCL / xGMI (SURVEY.md §8b "later":
   mpcr_comm_init; §8e).  One process (or host thread) per GPU, candidates
   sharded by rank (rank r rolls out [r n, (r+1) n) with index_base = r n).
   Replaces the torch.distributed path of manipulator_mujoco_amd/dist.py for
   hosts without Python; the reference itself is single-device
   (SBP/mjx_planner.py:395 argmin, :305-310 elites).  RCCL is dlopen'ed at the
   first call (librccl.so.1).  A communicator is single-stream, like an RCCL
   communicator: mpcr_comm_gather_elites stages the local elites in scratch
   owned by the comm, so calls on one comm must be ordered on one stream (or
   use one comm per stream). */
#define MPCR_COMM_ID_BYTES 128
typedef struct mpcr_comm mpcr_comm;
/* rank 0 creates the id and hands it to the other ranks out of band */
int mpcr_comm_unique_id(unsigned char* id_out /* MPCR_COMM_ID_BYTES */);
int mpcr_comm_init(int rank, int nranks, const unsigned char* id, int device, mpcr_comm** out);
void mpcr_comm_free(mpcr_comm* c);
/* in place, device pointer: global MIN of count packed best keys (the
   rollout's fused key is unsigned-ordered, so this is the global jnp.argmin:
   NaN first, ties to the lowest global index) */
int mpcr_comm_allreduce_key(mpcr_comm* c, uint64_t* d_key, int count, void* stream);
/* rank-major all-gather of count floats per rank (device pointers) */
int mpcr_comm_allgather(mpcr_comm* c, const float* d_send, float* d_recv, size_t count, void* stream);
/* sharded elites: local top-kl (kl = min(k, n)) of d_cost[n], their rows
   (d_xi row | cost) all-gathered into d_rows (nranks x kl x (nv+1)), and
   d_sel[k] = the global top-k positions in d_rows, in the single-GPU
   argsort(kind="stable")[:k] order.  Every rank passes the same n, nv, k. */
int mpcr_comm_gather_elites(mpcr_comm* c, const float* d_cost, const float* d_xi, int n, int nv, int k, float* d_rows,
                            int* d_sel, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MPCR_H_ */

// rollout.h -- what the host side (engine.hip) shares with the rollout
// kernel's translation unit (rollout.hip): the launch arguments, the plant
// state layout, the per-block LDS images (sizes for the HBM slabs), and the
// launchers.  rollout.hip is compiled on its own, with its own flags (see
// manipulator_mujoco_amd/build.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <type_traits>

#include "mpcr_device.h"
#include "../../include/mpcr_model.h"  // MPCR_FACE_MAXV (the face polygon cap)

namespace mpcr {

constexpr float kMinVal = 1e-15f;
constexpr float kMinImp = 0.0001f;
constexpr float kMaxImp = 0.9999f;

// per-call parameter block (RolloutArgs::par / dpar) and plant state layout
enum { PAR_Q0 = 0, PAR_W = 8, PAR_PT = 12, PAR_QT = 16, PAR_N = 20 };
// debug dump of candidate 0's last step (the same layout as the oracle's
// oracle_step_debug): active contacts (pos xyz, dist, pair, normal xyz),
// constraint rows (D, aref, vel), qacc_smooth, the final qacc
enum { DBG_NCON = 0, DBG_NEFC = 1, DBG_CON = 2, DBG_MAXCON = 48, DBG_ROW = DBG_CON + 8 * DBG_MAXCON, DBG_MAXROW = 200,
       DBG_QAS = DBG_ROW + 3 * DBG_MAXROW, DBG_QACC = DBG_QAS + DX_NV, DBG_INFO = DBG_QACC + DX_NV,
       DBG_GRAD = DBG_INFO + 8, DBG_SRCH = DBG_GRAD + DX_NV, DBG_MPR = DBG_SRCH + DX_NV, DBG_N = DBG_MPR + 112 };
// DBG_MPR: the host puts a pair index in [0]; the kernel's MPR on that pair writes [1] hit, [2] depth,
// [3..5] dir, [6..8] pos, [9..11] phase counts (discovery, refinement, penetration), [12..47] the final
// portal's v / a / b of vertices 0..3 (4 x 9), [48..111] the hull vertices (side 0, side 1) after each of
// the first 32 support queries
// DBG_INFO: warm start taken, its cost, qacc_smooth's cost, first iteration's p0 cost, alpha, line-search
// passes, the final bracket's best cost, Newton iterations run
enum { ST_QPOS = 0, ST_QVEL = DX_NQ, ST_QWS = ST_QVEL + DX_NV, ST_QACC = ST_QWS + DX_NV, ST_EEF = ST_QACC + DX_NV,
       ST_N = ST_EEF + 8 };

// horizon-segment state per candidate (RolloutArgs::seg_state): qpos (DX_NQ),
// qvel and the warm start (32 each), every lane's cost_c (the outputs sum it
// over lanes), then lane 0's cost_g, cost_r, status, rows summed, rows max
// (the outputs read them from lane 0 only; the other lanes' copies are never
// read): 672 B per candidate
constexpr int SEG_QPOS = 0, SEG_QVEL = DX_NQ, SEG_QWS = DX_NQ + 32, SEG_COSTC = DX_NQ + 64, SEG_SCAL = DX_NQ + 128,
              SEG_STRIDE = SEG_SCAL + 8;

// pacing table: (XCC 8 x SE 8 x SH 2 x CU 16 x SIMD 4) groups of 16 wave slots
constexpr unsigned MPCR_PACE_SLOTS = 8u * 8u * 2u * 16u * 4u * 16u;

struct RolloutArgs {
  const DevModel* m;
  const float* input;
  const float* pdot;  // H x nbasis
  float* cost4;
  float* theta;
  float* thetadot;
  unsigned long long* best_key;
  int* status;
  float* trace_eef;    // n x H x 7 (debug)
  float* trace_slots;  // n x H x nslot (debug)
  float* slot_prev;    // n x nslot previous slot distances (variants keeping them in HBM)
  float* jx;           // n x (MAXEFC - JL) x LDJ: J rows past the LDS ones
  short* hints;        // n x NHINT x 2: hull-climb start per convex pair and side (dual-arm class)
  unsigned long long* prof;  // per-phase cycles (MPCR_PROFILE builds only)
  float* tdscratch;  // (n + 1) x nctrl x H: the joint-velocity table when thetadot is not requested
  // per hardware wave slot: the step a resident wave is on (~0u when none),
  // MPCR_PACE_SLOTS words; the kernel's pacing reads its SIMD's 16 slots
  unsigned* pace;
  float* mslab;  // (n + 1) x NVW x LD: the mass matrix of the dual-arm class (SmemT::M_SLAB)
  // horizon segments (dual-arm class, one wave per candidate): this launch
  // runs steps [t0, t1) of every candidate; a segment that does not start at
  // 0 resumes from seg_state, one that does not end at H saves to it and
  // writes no outputs (the engine launches the segments in stream order:
  // kernel boundaries order them, rollout_launch)
  float* seg_state;  // n x SEG_STRIDE: qpos | qvel | qws | cost_c per lane | lane 0 scalars
  int t0, t1, seg;   // segment [t0, t1); seg = steps per segment for rollout_launch (0: one launch)
  int nctrl, nslot;  // the model's (host side: per-candidate strides of grouped launches)
  int seg_min_n;     // segments only for batches above this (the one-wave variant's resident blocks)
  float* dbg;  // parity debugging (mpcr_plant_step_debug): candidate 0's last step, DBG_* layout
  // per-call parameters: by value (par) or, for graph-captured ticks, read
  // from device memory (dpar, same layout) when the launch runs
  const float* dpar;
  // plant mode (single environment, mpcr_plant_*): plant & 1 starts from
  // state (qpos | qvel | qacc_warmstart) instead of the template,
  // plant & 2 writes the final state back; qacc and the pre-integration eef
  // pose of the last step always go to state when plant != 0
  float* state;
  int layout, n, H, nbasis, index_base, plant;
  float par[PAR_N];  // q0[8] | w[4] | ptgt[4] | qtgt[4] (any norm)
};

// Per-block LDS image, sized by the kernel variant: NVW = dense-solve width
// (16 or 32 dofs), NBW = moving bodies, NGW = collision geoms.  Row stride
// LD = NVW + 4 floats: rows are 16-byte aligned for ds_read_b128 and 16 lanes
// reading 16 different rows hit distinct bank quads (LD*r mod 64 distinct
// multiples of 4 for LD = 20 and 36) -> conflict free, 4x fewer LDS
// instructions than b32.
// qpos entries of the narrow image (the engine sends larger models to the wide
// variant; the single-arm scenes have nq <= 15)
#ifndef MPCR_N_NQ
#define MPCR_N_NQ 20
#endif
// polyhedron manifold: a penetration deeper than POLY_DEEP m between hulls of
// at most POLY_ALLF faces together scans every face for the SAT axis instead
// of the cone about MPR's normal (the oracle's poly_manifold, same constants)
#ifndef MPCR_POLY_ALLF
#define MPCR_POLY_ALLF 512  // 0: the cone always (timing experiments only)
#endif
// compact mass-matrix rows in the dual-arm image (SmemT::Mc; the dual arm has 22 dofs)
#ifndef MPCR_W_MC_ROWS
#define MPCR_W_MC_ROWS 24
#endif
// faces per lane per pass of that scan (their loads in flight together)
#ifndef MPCR_ALLF_U
#define MPCR_ALLF_U 2
#endif
constexpr float POLY_DEEP = 5e-3f;
constexpr int POLY_ALLF = MPCR_POLY_ALLF > 0 ? MPCR_POLY_ALLF : 1;
constexpr bool POLY_ALLF_ON = MPCR_POLY_ALLF > 0;

template <int NVW_, int NBW_, int NGW_, int MAXEFC_ = DX_MAXEFC, int LDJ_ = NVW_ + 4, bool CPREV_GLOBAL_ = false,
          int JL_ = MAXEFC_, int CPW_ = 1, int MAXACT_ = DX_MAXACT, bool SPLIT_ = false>
struct __align__(16) SmemT {
  // SPLIT: the dynamics scratch and the contact / constraint arrays do not
  // overlay (the two-wave variant runs the dynamics and the collision phase
  // at the same time)
  static constexpr bool SPLIT = SPLIT_;
  static constexpr int DYN_FLOATS = NBW_ * 64 + NVW_ * 16;  // xpos .. fvec below
  static constexpr int NVW = NVW_, NBW = NBW_, NGW = NGW_, LD = NVW_ + 4;
  // candidates per wave: CPW images per workgroup, HL = 64 / CPW lanes each
  static constexpr int CPW = CPW_, HL = WAVE / CPW_;
  static constexpr int MAXEFC = MAXEFC_, LDJ = LDJ_;      // constraint rows kept, J row stride
  static constexpr int MAXACT = MAXACT_;                  // active contacts kept
  static constexpr int JL = JL_;  // J rows held in LDS; rows JL.. live in the block's HBM slab (RolloutArgs::jx)
  static_assert(JL <= MAXEFC && JL % 4 == 0, "J rows in LDS");
  static constexpr bool CPREV_GLOBAL = CPREV_GLOBAL_;     // previous slot distances in HBM (L2) instead of LDS
  static constexpr int LOG_NVW = NVW_ == 32 ? 5 : 4;
  static constexpr bool WIDE = NVW_ == 32;  // dual-arm class: equalities, actuators, convex hulls
  static constexpr int NQW = WIDE ? DX_NQ : MPCR_N_NQ, NEQP = WIDE ? DX_NEQ : 1, NACT = WIDE ? DX_NU : 1;
  // compacted convex-pair list: room for every convex pair a model may have
  // (the engine allows 512), so the collision phase flushes it once, at its
  // end (round 5: the flush runs on both waves of a two-wave candidate)
  static constexpr int CVXN = WIDE ? 512 : 1;
  static constexpr int NHINT = WIDE ? 512 : 1;  // hull-climb start per convex pair and side
  static constexpr int PMAXW = 2 * MPCR_FACE_MAXV + 2;  // clipped incident face: <= its vertices + one per side plane
  static constexpr int FRAMEW = WIDE ? 3 : 9;  // contact frame entries kept (the wide image recomputes the tangents)
  // ---- persistent across the step ----
  float qpos[NQW];
  alignas(16) float qvel[NVW];
  alignas(16) float qacc[NVW];
  alignas(16) float qws[NVW];
  alignas(16) float qfs[NVW];   // qfrc_smooth
  alignas(16) float qas[NVW];   // qacc_smooth
  alignas(16) float srch[NVW];  // Newton search direction
  float com[DX_NTREE][4];
  float cdof[NVW][WIDE ? 6 : 8];
  // the dual-arm class keeps M compact in LDS (Mc: row i is the MCW = 16
  // columns from DevModel::mc_c0[i] on, which hold its tree's; 1.4 KB for the
  // dual arm's 22 dofs where the dense image was 4.6 KB), or -- a model whose
  // trees do not fit that, DevModel::mc_n == 0 -- in a per-candidate HBM slab
  // (RolloutArgs::mslab)
  static constexpr bool M_SLAB = NVW_ == 32;
  static constexpr int MCW = 16, MC = M_SLAB ? MPCR_W_MC_ROWS * MCW : 4;
  union {
    alignas(16) float M[M_SLAB ? 1 : NVW][M_SLAB ? 4 : LD];  // the dense image (single-arm variants)
    alignas(16) float Mc[MC];
  };
  alignas(16) float gxpos[NGW][4];   // gxpos+gxmat (dead during Newton) double as the
  float gxmat[NGW][12];  // Hessian solve's LDS scratch (NGW*16 >= NVW*LD)
  float cprev[CPREV_GLOBAL ? 1 : DX_NSLOT];  // previous-step masked slot distances (cost_c)
  float par[PAR_N];       // q0 | w | ptgt | qtgt (normalised)
  float eqp[NEQP][2][4];  // connect anchors in world (body1, body2)
  float tenp[WIDE ? DX_NTEN : 1][2][4];  // spatial-tendon sites in world
  float actf[NACT];       // actuator forces
  int ncon, nefc, ncvx, pad_;
  int ctok_[SPLIT_ ? 4 : 0];  // two-wave images: [0] the step whose pair cull is done (rollout.hip, swap mode)
  // ---- phase-local: dynamics (kinematics .. mass matrix) overlays the
  //      contact / constraint arrays (collision .. Newton) ----
  union {
    struct {
      alignas(16) float xpos[NBW][4];
      float xquat[NBW][4];
      float xmat[NBW][12];
      float xipos[NBW][4];
      float cinert[NBW][12];
      float crb[NBW][12];
      float cvel[NBW][8];
      float cfrc[NBW][8];
      float cdofdot[NVW][8];
      float fvec[NVW][8];
    };
    struct {
      float split_pad_[SPLIT_ ? DYN_FLOATS : 0];  // SPLIT: past the dynamics scratch
      union {
        alignas(16) float J[JL][LDJ];  // constraint rows .. Newton
        struct {                        // collision:
          int cvx[CVXN];                // the compacted convex-pair list
          alignas(16) float polyw[2][WIDE ? PMAXW : 1][4];  // polyhedron-manifold clip polygon (double buffered)
          float satsep[WIDE ? POLY_ALLF : 1];  // a deep polyhedron pair's SAT separation of every face
        };
      };
      float efc_D[MAXEFC];
      float efc_aref[MAXEFC];
      int efc_src[MAXEFC];  // (kind << 24) | (index << 4) | side
      union {
        struct {  // collision .. constraint rows
          float con_pos[MAXACT][4];
          float con_frame[MAXACT][FRAMEW == 3 ? 4 : 12];  // rows n, t1, t2 (the wide image: n only)
          float con_dist[MAXACT];
          int con_pair[MAXACT];
          int con_row[MAXACT];
          float poly[2][8][4];  // box-box clipping polygon (double buffered)
        };
        struct {  // Newton (the contacts are dead once the rows are built)
          float efc_jar[MAXEFC];
          float efc_jv[MAXEFC];
          float efc_f[MAXEFC];   // -D * jar on active rows, else 0
          float efc_Da[MAXEFC];  // D on active rows, else 0
        };
      };
    };
  };
};
// The polyhedron manifold's scratch (clip polygon, SAT separations) as its
// own type: the LDS image's (polyw, satsep: the same layout inside the J
// rows) or, for the dynamics wave of a two-wave candidate in the joint convex
// flush, one in the dynamics region (dead from the mass-matrix solve to the
// next step's kinematics), followed there by the flush's per-item contact
// counts (jcnt, 2 x 64 items per round)
template <int PMAXW_>
struct PolyScratchT {
  alignas(16) float polyw[2][PMAXW_][4];
  float satsep[POLY_ALLF];
};

// The two variants: single-arm scenes (nv <= 16) and the dual-arm class.
// Single-arm image: 96 constraint rows of which the first 40 keep their J row
// in LDS (stride 16) and the rest in a per-candidate HBM slab (RolloutArgs::jx;
// the per-step row count is ~23 on average, p50 of a candidate's busiest step
// 39, so the slab serves a minority of the rows), the contacts overlaid with
// the Newton-only row arrays, the cost history and the Bernstein
// coefficients in HBM: 9.3 KB of LDS -> 16 blocks per CU = 4 waves/SIMD at 128
// VGPRs (was 17.3 KB and 178 VGPRs: 2 waves/SIMD).  Measured on MI355X
// (round 4, extra dynamic LDS on C3): 16 blocks per CU up to 10240 B each
// (the CU's whole 160 KB), 15 at 10368 B; the image keeps 9520 B (the J rows
// in LDS 40 -> 44 / 48 gained nothing).
#ifndef MPCR_N_MAXEFC
#define MPCR_N_MAXEFC DX_MAXEFC
#endif
#ifndef MPCR_N_JL
#define MPCR_N_JL 40  // 36 -> 40 with the 20-entry qpos image: the budget exactly (C3 1.616 -> 1.610 ms)
#endif
#ifndef MPCR_N_LDJ
#define MPCR_N_LDJ 16
#endif
#ifndef MPCR_N_CPREV_GLOBAL
#define MPCR_N_CPREV_GLOBAL 1
#endif
#ifndef MPCR_N_CPW
#define MPCR_N_CPW 1
#endif
using SmemN = SmemT<16, 16, 24, MPCR_N_MAXEFC, MPCR_N_LDJ, MPCR_N_CPREV_GLOBAL, MPCR_N_JL, MPCR_N_CPW>;
#if !defined(MPCR_N_LDS_UNCHECKED)
static_assert(sizeof(SmemN) <= 9520, "narrow LDS image must fit 16 blocks per CU (see above)");
#endif
// The two-wave narrow image (small batches, rollout_kernel<..., 2>): dynamics
// scratch and contacts side by side, every J row in LDS (no HBM slab) -- at
// most 2048 candidates = 8 blocks per CU, so LDS is not the limit
using SmemN2 = SmemT<16, 16, 24, MPCR_N_MAXEFC, MPCR_N_LDJ, MPCR_N_CPREV_GLOBAL, MPCR_N_MAXEFC, 1, DX_MAXACT, true>;
static_assert(sizeof(SmemN2) <= 152448 / 8, "two-wave narrow image: 8 blocks per CU");
// Dual-arm image: J rows past 44 in the HBM slab, cost history and hull-climb
// hints in HBM (the class has no robot-masked slots), the convex-pair list
// inside the J rows, 6-float cdof rows, the mass matrix in an HBM slab:
// 17.2 KB -> 8 blocks per CU (21.7 KB / 7 before the M slab; 32.3 KB / 4
// before the J slab); the kernel is compiled for 2 waves/SIMD (<= 256 VGPRs),
// so 8 blocks per CU is also its register limit.
#ifndef MPCR_W_JL
#define MPCR_W_JL 44  // 40 -> 44 since the manifold doubled the rows (53.5 per step): C4 50.4 -> 49.7 ms
#endif
#ifndef MPCR_W_MAXACT
#define MPCR_W_MAXACT 48  // the polyhedron manifold's 4 contacts per face pair (40 truncated 0.5 % of a C4 shard)
#endif
using SmemW = SmemT<32, 32, 72, 8 + 4 * MPCR_W_MAXACT, 36, true, MPCR_W_JL, 1, MPCR_W_MAXACT>;
// The two-wave dual-arm image (MPCR_W_WPC2 builds, small batches): the
// dynamics scratch beside the contact / constraint arrays
// and, since it runs at most 4 blocks per CU (<= 1024 candidates on 256
// CUs: 40 960 B each of the CU's 160 KB), J rows 0..103 in LDS instead of
// 0..43 (round 5): the rows past 44 -- a dual-arm step has 51 on average,
// p50 of a candidate's busiest step 60 -- were dependent L2 / HBM-slab loads
// inside Newton's row loops.  Same values in the same order: bitwise.
#ifndef MPCR_W2_JL
#define MPCR_W2_JL 104
#endif
using SmemW2 = SmemT<32, 32, 72, 8 + 4 * MPCR_W_MAXACT, 36, true, MPCR_W2_JL, 1, MPCR_W_MAXACT, true>;
static_assert(sizeof(SmemW2) <= 163840 / 4, "two-wave dual-arm image: 4 blocks per CU");
static_assert(sizeof(PolyScratchT<SmemW2::PMAXW>) + 2 * WAVE * 4 <= SmemW2::DYN_FLOATS * 4,
              "the dynamics wave's manifold scratch and the flush counts inside the dynamics region");
// the two-wave lead flush (rollout.hip): at most W2_LEAD_MAX convex pairs in
// the step's list (else the dealt flush), a manifold-queue record of
// W2_JOB_REC ints per job inside the convex-pair list, and wave 0's results
// (4 distances, points, normals, the count) W2_JOB_OUT floats per job in the
// dynamics region after its manifold scratch
#ifndef MPCR_W2_LEAD
#define MPCR_W2_LEAD 1
#endif
// swap mode (rollout.hip): wave 0 runs the non-convex narrow phase
#ifndef MPCR_W2_SWAP
#define MPCR_W2_SWAP 1
#endif
constexpr int W2_LEAD_MAX = 56, W2_JOB_REC = 8, W2_JOB_OUT = 29;
static_assert(W2_LEAD_MAX <= WAVE && 2 + W2_JOB_REC * W2_LEAD_MAX <= SmemW2::CVXN, "manifold queue inside the list");
static_assert(sizeof(PolyScratchT<SmemW2::PMAXW>) + 4 * W2_JOB_OUT * W2_LEAD_MAX <= SmemW2::DYN_FLOATS * 4,
              "wave 0's manifold mailbox inside the dynamics region");
static_assert(offsetof(SmemW, satsep) - offsetof(SmemW, polyw) == offsetof(PolyScratchT<SmemW::PMAXW>, satsep),
              "the image's manifold scratch has PolyScratchT's layout");
static_assert(SmemN::NGW * 16 >= SmemN::NVW * SmemN::LD + SmemN::NVW, "Hessian + J^T f scratch");
static_assert(SmemW::NGW * 16 >= SmemW::NVW * SmemW::LD, "Hessian scratch");
static_assert(SmemW::JL * SmemW::LDJ * 4 >= SmemW::CVXN * 4 + 2 * SmemW::PMAXW * 16 + 16 + POLY_ALLF * 4,
              "convex-pair list, clip polygon and SAT separations inside the J rows");
#if !defined(MPCR_N_LDS_UNCHECKED)
// measured on MI355X (C4 shard, extra dynamic LDS per block): 8 blocks per CU
// up to 18912 + 1536 B, 7 at 18912 + 2048 B
static_assert(sizeof(SmemW) <= 20448, "dual-arm LDS image must fit 8 blocks per CU");
#endif


// launchers (defined in rollout.hip): the rollout kernel variant for the
// model class over `grid` blocks of one wave; dyn_lds extra bytes per block
// (occupancy experiments only)
// Dual-arm batches of the one-wave variant with a.seg > 0 and H > a.seg run as
// horizon segments of a.seg steps over `groups` candidate groups, group g on
// gstream[g] (forked from st by gev[0] and joined back by gev[1 + g]); every
// group's segments in stream order.  The launches of different groups overlap,
// so one segment's tail is filled by the other groups' work.
void rollout_launch(bool wide, const RolloutArgs& a, const DevModel* dm, unsigned grid, size_t dyn_lds,
                    hipStream_t st, int groups = 0, hipStream_t* gstream = nullptr, hipEvent_t* gev = nullptr);
// the dual-arm kernels' launches and occupancy (their own translation unit,
// rollout.hip built with MPCR_TU = 2): wpc 1 (one wave per candidate, block
// per candidate) or 2 (two waves); info[0..2] blocks per CU, LDS, VGPRs
void rollout_wide_launch(int wpc, unsigned grid, hipStream_t st, const RolloutArgs& a, const DevModel* dm);
hipError_t rollout_wide_occupancy(int* info);
// kernel dispatches rollout_launch issues for the same arguments (gstream /
// gev given: streams)
int rollout_dispatches(bool wide, const RolloutArgs& a, unsigned grid, int groups, bool streams);
// resident blocks per CU, static LDS bytes, VGPRs: narrow (0..2), wide (3..5)
hipError_t rollout_occupancy(int* info, size_t dyn_lds);
int rollout_set_wpc2_max_n(int n);  // two waves per candidate up to n (narrow variant); returns the previous

}  // namespace mpcr

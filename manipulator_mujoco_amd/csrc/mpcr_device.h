// mpcr_device.h — fp32 device mirror of mpcr_model_t with the derived tables
// the wave-per-rollout kernel needs (static-body poses folded in, subtree /
// dof-chain bitmasks, collision-geom remap).  Built once per engine on the
// host (engine.cpp: build_dev_model) and read by the kernel with uniform
// (scalar-cache) loads.
#pragma once
#include <stdint.h>

namespace mpcr {

constexpr int WAVE = 64;
// capacities of the device model (the kernel variants size their LDS by
// their own widths, rollout.hip SmemT)
constexpr int DX_NB = 32;    // moving bodies (32-bit subtree masks)
constexpr int DX_NV = 32;    // dofs (32-bit dof masks; widest dense solve)
constexpr int DX_NQ = 32;
constexpr int DX_NJ = 32;
constexpr int DX_NG = 72;    // collision geoms (remapped)
constexpr int DX_NP = 768;   // pairs
constexpr int DX_NEQ = 8;
constexpr int DX_NEQROW = 24;  // equality constraint rows (joint 1, connect 3)
constexpr int DX_NU = 16;    // actuators
constexpr int DX_NCTRL = 8;
constexpr int DX_NTREE = 4;
constexpr int DX_MAXACT = 20;  // active contacts kept per step
constexpr int DX_MAXEFC = 96;  // constraint rows kept per step
constexpr int DX_NSLOT = 192;  // robot-masked contact slots
constexpr int DX_NTEN = 2;     // spatial (two-site) tendons with length limits
// polyhedron manifold: the faces of a geom whose outward normal can lie within
// the Gauss-map cone (kPolyConeCos) of a direction in each cube-map cell of
// CONE_R x CONE_R per cube face (built on the host from the face planes)
constexpr int CONE_R = 8;
constexpr int CONE_CELLS = 6 * CONE_R * CONE_R;
constexpr double CONE_COS = 0.94;  // the kernel's and the oracle's cone (rollout.hip kPolyConeCos)

// The model's table pointers are global memory: typed so in the device pass
// (same 8-byte layout as the host's plain pointers), so the kernel's loads
// through them are global_load, not flat_load (a flat load counts against the
// LDS wait counter too, and waits for an LDS read then also wait for it)
#if defined(__HIP_DEVICE_COMPILE__)
#define MPCR_GMEM __attribute__((address_space(1)))
#else
#define MPCR_GMEM
#endif
// host side: a device allocation as the model's table pointer type
template <class T>
inline const MPCR_GMEM T* as_gmem(T* p) {
  return (const MPCR_GMEM T*)p;
}

// body kinds for the kinematics pass
enum { BK_STATIC = 0, BK_FREE = 1, BK_HINGE = 2, BK_SLIDE = 3, BK_WELD = 4 };

struct DevModel {
  int nbody, njnt, nq, nv, ngeom, npair, neq, nslot;
  int nctrl, ntree, hande_body, tcp_body;
  int iterations, ls_iterations, disableflags, jump_rounds;
  int nhdof;  // number of dofs, rounded to the solve width
  int nu, neqrow, integrator;  // actuators, equality rows, 0 Euler / 3 implicitfast
  int has_spring;
  int cvx_base;  // first general-convex pair (pairs are sorted by function)
  // two waves per candidate (narrow variant): the collision wave also builds
  // the constraint rows (models whose collision phase is light: one chunk of
  // pairs, no wave-cooperative box-box pair -- measured: C2 0.955 -> 0.850 ms,
  // scene_mjx at 1024 / 2048 candidates 1.081 / 1.189 -> 1.093 / 1.207 ms)
  int coll_rows;
  // dual-arm class, two waves per candidate: the convex flush deals its pairs
  // over both waves (no convex pair has a cost slot, so no per-lane cost_c
  // order is at stake; the contacts still go to the list in pair order)
  int cvx_joint;
  int w2_lead_max;  // the two-wave lead flush's pair limit (rollout.h W2_LEAD_MAX; MPCR_W2_LEAD_MAX lowers it: tests)
  float timestep, tolerance, ls_tolerance, meaninertia;
  float gravity[4];
  float tcp_pos[4];  // tcp site position in tcp_body frame

  // bodies -------------------------------------------------------------
  int body_kind[DX_NB];
  int body_anc[DX_NB];      // first ancestor for pointer jumping (-1: none)
  int body_jnt[DX_NB];      // hinge/slide/free joint of the body (-1: none)
  int body_tree[DX_NB];     // dynamic tree index (-1: static)
  uint32_t body_dofmask[DX_NB];  // dofs on the path body..root
  uint32_t body_submask[DX_NB];  // bodies in the subtree (incl. itself)
  float body_bpos[DX_NB][4];     // pre-joint local (or constant world) pose
  float body_bquat[DX_NB][4];
  float body_ipos[DX_NB][4];
  float body_Iloc[DX_NB][8];     // inertia about COM in body frame: xx,yy,zz,xy,xz,yz
  float body_mass[DX_NB];
  float body_gravcomp[DX_NB];
  float body_invw[DX_NB];        // translational invweight0
  float tree_mass[DX_NTREE];

  // joints ------------------------------------------------------------
  int jnt_type[DX_NJ], jnt_qposadr[DX_NJ], jnt_dofadr[DX_NJ], jnt_body[DX_NJ], jnt_limited[DX_NJ];
  float jnt_pos[DX_NJ][4], jnt_axis[DX_NJ][4], jnt_range[DX_NJ][2];
  float jnt_solref[DX_NJ][2], jnt_solimp[DX_NJ][5], jnt_margin[DX_NJ];
  float jnt_qpos0[DX_NJ];

  // dofs --------------------------------------------------------------
  int dof_body[DX_NV], dof_jnt[DX_NV], dof_kind[DX_NV];  // kind: 0 hinge 1 slide 2 free-trans 3 free-rot
  int dof_sub[DX_NV];            // free: axis index 0..2
  uint32_t dof_chainmask[DX_NV]; // dofs j with M[i][j] possibly nonzero (ancestors incl. self)
  uint32_t dof_velmask[DX_NV];   // dofs forming the velocity cdof_dot uses
  uint32_t dof_submask[DX_NV];   // bodies in the subtree of the dof's body (bias force sum)
  // blocked Cholesky (narrow kernel): every kinematic tree's dofs (<= 8 each,
  // <= 4 trees) in their own 16-lane DPP row, so M -- block diagonal by tree --
  // and an uncoupled Newton H factor as ntree simultaneous 8-column chains
  int blk_n;                     // 8 / 16: every tree has <= that many dofs; 0: dense paths only
  int eq_cross;                  // an equality / tendon row couples two trees (Newton stays dense)
  int impl_cross;                // implicitfast's D couples two trees (its solve stays dense)
  int blane_dof[64];             // lane 16 tree + k -> dof (-1: pad)
  // compact mass matrix (dual-arm class, in LDS): row i keeps the 16 columns
  // from mc_c0[i] (a multiple of 4) on, which cover its tree's dofs; mc_n:
  // rows kept (0: M in the per-candidate HBM slab instead -- a tree's dofs
  // not contiguous or wider than that window, or more rows than the image has)
  int mc_n;
  int mc_c0[DX_NV];
  float dof_armature[DX_NV], dof_damping[DX_NV], dof_invweight0[DX_NV];

  float qpos_init[DX_NQ];
  float qvel_init[DX_NV];

  // collision geoms (remapped to the ones any pair uses) ----------------
  int geom_body[DX_NG], geom_type[DX_NG];
  float geom_pos[DX_NG][4], geom_quat[DX_NG][4], geom_size[DX_NG][4];
  float geom_rbound[DX_NG];

  // pairs ---------------------------------------------------------------
  int pair_g1[DX_NP], pair_g2[DX_NP], pair_func[DX_NP], pair_ncon[DX_NP];
  int4 pair_jinfo[DX_NP];  // contact Jacobian per pair: (dof mask of body 1, of body 2, tree 1, tree 2); world: mask 0
  int pair_slotadr[DX_NP], pair_condim[DX_NP];
  float pair_friction[DX_NP], pair_margin[DX_NP];  // margin = includemargin (margin - gap)
  float pair_solref[DX_NP][2], pair_solimp[DX_NP][5];
  float pair_diag[DX_NP];        // tran invweight of the two bodies

  // equalities: joint (eq_j1/j2, polycoef in eq_data) and connect (moving
  // bodies eq_b1/b2 or -1 for a static body, whose anchor eq_data[4*side..]
  // is then already in world coordinates) -----------------------------------
  int eq_type[DX_NEQ], eq_j1[DX_NEQ], eq_j2[DX_NEQ], eq_b1[DX_NEQ], eq_b2[DX_NEQ];
  float eq_data[DX_NEQ][8], eq_solref[DX_NEQ][2], eq_solimp[DX_NEQ][5], eq_diag[DX_NEQ];
  int eqrow_eq[DX_NEQROW], eqrow_k[DX_NEQROW];  // row -> (equality, component)

  // passive springs and actuation per dof --------------------------------------
  float dof_stiffness[DX_NV], dof_springref[DX_NV];
  int dof_qposadr[DX_NV];
  int dof_actn[DX_NV], dof_acta[DX_NV][2];  // actuators driving this dof
  float dof_actm[DX_NV][2];                  // their moments on it
  float dof_actfrc[DX_NV][2];                // joint-level actuator force range
  // actuators: force = gain * ctrl + bias, gain = g0 (+ g1 len + g2 vel),
  // bias = b0 + b1 len + b2 vel, clamped to act_frc
  int act_ntrn[DX_NU], act_qadr[DX_NU][2], act_dof[DX_NU][2], act_gaffine[DX_NU], act_baffine[DX_NU];
  float act_moment[DX_NU][2], act_gain[DX_NU][4], act_bias[DX_NU][4], act_frc[DX_NU][2];
  // implicitfast: D = -qDeriv (damping + actuator velocity derivatives), the
  // integrator solves (M + dt D) qacc = qfrc_smooth + qfrc_constraint
  float impl_D[DX_NV][DX_NV];

  // convex hulls of mesh geoms (geom frame), hill-climbing graph -----------------
  int geom_hulladr[DX_NG];
  int geom_hullnum[DX_NG];
  int geom_lutadr[DX_NG];  // first hull_lut cell (engine.hip hull_start_table), -1: no table
  const MPCR_GMEM float4* hull_vert;  // xyz | degree (int bits in w)
  const MPCR_GMEM int2* hull_info;    // (adjacency start, count) per vertex
  const MPCR_GMEM float4* hull_adjv;  // neighbour xyz | (index | degree << 16) (bits in w): one load per neighbour
  const MPCR_GMEM float4* hull_lut;   // support start table records (as hull_adjv), MPCR_LUT_R cube-map cells per hull
  unsigned long long* prof;  // wave-level event counters (MPCR_PROFILE builds; else null)
  const MPCR_GMEM float4* hull_head;  // per vertex its first 8 neighbour records as hull_adjv, padded with NaN records:
                            // a climb round addresses them from the vertex index alone (no hull_info load)
  // polygon faces of polyhedron-pair geoms (mesh-mesh / box-mesh manifold) ----
  int geom_faceadr[DX_NG];   // first face, -1: none
  int geom_facenum[DX_NG];   // its face count
  int geom_cornadr[DX_NG];   // a box's 8 corners in hull_vert (bit k: + side of axis k), -1: none
  const MPCR_GMEM float4* face_plane;  // outward normal xyz | offset (n . x = offset), geom frame
  const MPCR_GMEM int2* face_vinfo;    // (first face_vert entry, count <= MPCR_FACE_MAXV)
  const MPCR_GMEM int* face_vert;      // hull_vert indices, counter-clockwise about the normal
  const MPCR_GMEM int2* vert_finfo;    // per hull vertex: (first vert_face entry, count)
  const MPCR_GMEM int* vert_face;      // face indices
  int geom_coneadr[DX_NG];   // first cone_cell record (CONE_CELLS per geom with faces), -1: none
  const MPCR_GMEM int2* cone_cell;     // (first cone_face entry, count) per cell
  const MPCR_GMEM int* cone_face;      // face indices, ascending within a cell: a superset of the faces the
                             // cone test can accept for any direction in the cell

  int ctrl_qposadr[DX_NCTRL], ctrl_dofadr[DX_NCTRL];

  // scene_robotiq_hande.xml features (wide variant) ----------------------------
  int cone;        // 0 pyramidal, 1 elliptic (condim-3 contacts: rows n, t1, t2)
  int nten;
  float impratio;
  float pair_cmu[DX_NP];    // elliptic cone slope: friction / sqrt(impratio)
  float body_visc[DX_NB][2];  // inertia-box viscosity: force = [0] v, torque = [1] w (at xipos)
  // spatial tendons: site body (device index, -1 static) and the site position
  // in that body's frame (static: in world)
  int ten_body[DX_NTEN][2], ten_limited[DX_NTEN];
  float ten_pos[DX_NTEN][2][4];
  float ten_range[DX_NTEN][2], ten_solref[DX_NTEN][2], ten_solimp[DX_NTEN][5], ten_margin[DX_NTEN], ten_invw[DX_NTEN];
};

}  // namespace mpcr

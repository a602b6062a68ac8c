// mpcr_device.h — fp32 device mirror of mpcr_model_t with the derived tables
// the wave-per-rollout kernel needs (static-body poses folded in, subtree /
// dof-chain bitmasks, collision-geom remap).  Built once per engine on the
// host (engine.cpp: build_dev_model) and read by the kernel with uniform
// (scalar-cache) loads.
#pragma once
#include <stdint.h>

namespace mpcr {

constexpr int WAVE = 64;
constexpr int DX_NB = 16;    // moving bodies
constexpr int DX_NV = 16;    // dofs (padded register width of the dense solves)
constexpr int DX_NQ = 24;
constexpr int DX_NJ = 16;
constexpr int DX_NG = 24;    // collision geoms (remapped)
constexpr int DX_NP = 256;   // pairs
constexpr int DX_NEQ = 4;
constexpr int DX_NCTRL = 8;
constexpr int DX_NTREE = 4;
constexpr int DX_MAXACT = 20;  // active contacts kept per step
constexpr int DX_MAXEFC = 96;  // constraint rows kept per step
constexpr int DX_NSLOT = 192;  // robot-masked contact slots

// body kinds for the kinematics pass
enum { BK_STATIC = 0, BK_FREE = 1, BK_HINGE = 2, BK_SLIDE = 3, BK_WELD = 4 };

struct DevModel {
  int nbody, njnt, nq, nv, ngeom, npair, neq, nslot;
  int nctrl, ntree, hande_body, tcp_body;
  int iterations, ls_iterations, disableflags, jump_rounds;
  int nhdof;  // number of dofs, rounded to the solve width
  int pad_[3];
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
  float dof_armature[DX_NV], dof_damping[DX_NV], dof_invweight0[DX_NV];

  float qpos_init[DX_NQ];
  float qvel_init[DX_NV];

  // collision geoms (remapped to the ones any pair uses) ----------------
  int geom_body[DX_NG], geom_type[DX_NG];
  float geom_pos[DX_NG][4], geom_quat[DX_NG][4], geom_size[DX_NG][4];
  float geom_rbound[DX_NG];

  // pairs ---------------------------------------------------------------
  int pair_g1[DX_NP], pair_g2[DX_NP], pair_func[DX_NP], pair_ncon[DX_NP];
  int pair_slotadr[DX_NP], pair_condim[DX_NP];
  float pair_friction[DX_NP], pair_margin[DX_NP];  // margin = includemargin (margin - gap)
  float pair_solref[DX_NP][2], pair_solimp[DX_NP][5];
  float pair_diag[DX_NP];        // tran invweight of the two bodies

  // joint equalities ------------------------------------------------------
  int eq_j1[DX_NEQ], eq_j2[DX_NEQ];
  float eq_data[DX_NEQ][5], eq_solref[DX_NEQ][2], eq_solimp[DX_NEQ][5], eq_diag[DX_NEQ];

  int ctrl_qposadr[DX_NCTRL], ctrl_dofadr[DX_NCTRL];
};

}  // namespace mpcr

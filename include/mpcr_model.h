/*
 * mpcr_model.h — flat, POD "compiled model" consumed by the rollout engine
 * (libmpcr) and by the CPU oracle (oracle/).
 *
 * The reference hands an mjx.Model pytree to every rollout
 * (SBP/mjx_planner.py:100-108: MjModel.from_xml_path -> mjx.put_model).  Our
 * boundary instead takes this fixed-capacity C struct, produced on the host by
 * manipulator_mujoco_amd/mjcf.py (the MJCF compiler) and serialised as a raw
 * little-endian blob (".mpcrm").  All quantities are SI / radians, quaternions
 * are (w, x, y, z), matrices row-major.  fp64 here; the engine builds its own
 * fp32 device mirror.
 *
 * Field names follow MuJoCo's mjModel so that the oracle and the kernels read
 * like the engine whose semantics they restate.
 */
#ifndef MPCR_MODEL_H_
#define MPCR_MODEL_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCR_MODEL_MAGIC   0x4d504352u /* 'MPCR' */
#define MPCR_MODEL_VERSION 9 /* v9: no support start table (the engine builds it) */

#define MPCR_MAX_BODY   48
#define MPCR_MAX_JNT    40
#define MPCR_MAX_DOF    32   /* dof bitmasks are 32-bit */
#define MPCR_MAX_NQ     48
#define MPCR_MAX_GEOM   128
#define MPCR_MAX_SITE   24
#define MPCR_MAX_PAIR   768
#define MPCR_MAX_EQ     8
#define MPCR_MAX_SLOT   512  /* robot-masked contact slots (cost_c) */
#define MPCR_MAX_CTRL   8    /* planner-controlled dofs (num_dof) */
#define MPCR_MAX_ACT    16   /* actuators */
#define MPCR_MAX_HULLV  8192 /* convex-hull vertices of all collision meshes */
#define MPCR_MAX_HULLA  49152 /* hull-graph adjacency entries */
/* support start table resolution: 6 cube faces x R x R cells per hull.  Not
   part of the blob since v9 -- the engine builds the table from hull_vert
   (engine.hip hull_start_table), so R is the library's build-time choice
   (round 5: 16 -> 128; 256 measured in round 6, DESIGN.md perf log) */
#ifndef MPCR_LUT_R
#define MPCR_LUT_R      128
#endif
#define MPCR_MAX_FACE   12288 /* polygon faces of the polyhedron-pair hulls and boxes */
#define MPCR_MAX_FACEV  49152 /* face polygon vertex entries (<= MPCR_FACE_MAXV each) */
#define MPCR_MAX_VFACE  65536 /* vertex -> incident face entries */
#define MPCR_FACE_MAXV  16    /* vertices kept per face polygon */
#define MPCR_MAX_TEN    4    /* spatial (site-site) tendons with limits */

/* joint types (MuJoCo mjtJoint) */
enum { MPCR_JNT_FREE = 0, MPCR_JNT_BALL = 1, MPCR_JNT_SLIDE = 2, MPCR_JNT_HINGE = 3 };
/* geom types (MuJoCo mjtGeom order; only these collide here) */
enum {
  MPCR_GEOM_PLANE = 0, MPCR_GEOM_SPHERE = 2, MPCR_GEOM_CAPSULE = 3, MPCR_GEOM_CYLINDER = 5, MPCR_GEOM_BOX = 6,
  MPCR_GEOM_MESH = 7
};
/* narrow-phase functions; pair_ncon gives the contact slots each one owns */
enum {
  MPCR_COL_PLANE_CAPSULE = 0, /* 2 slots: one per capsule end        */
  MPCR_COL_PLANE_BOX     = 1, /* 4 slots: the 4 deepest corners      */
  MPCR_COL_CAPSULE_CAPSULE = 2, /* 1 slot: closest segment points    */
  MPCR_COL_CAPSULE_BOX   = 3, /* 2 slots: closest point + far end    */
  MPCR_COL_BOX_BOX       = 4, /* 4 slots: SAT + face clipping        */
  MPCR_COL_PLANE_SPHERE  = 5, /* 1 slot                              */
  MPCR_COL_SPHERE_SPHERE = 6, /* 1 slot                              */
  MPCR_COL_SPHERE_CAPSULE = 7, /* 1 slot                             */
  MPCR_COL_SPHERE_BOX    = 8, /* 1 slot                              */
  MPCR_COL_CONVEX        = 9, /* 1 slot: general convex pair (capsule,
                                 cylinder, box, sphere, mesh hull) by
                                 Minkowski portal refinement (penetration) */
  MPCR_COL_PLANE_CONVEX  = 10, /* 1 slot: deepest support point along -n */
  MPCR_COL_NTYPES        = 11
};
/* equality types (mjtEq) */
enum { MPCR_EQ_CONNECT = 0, MPCR_EQ_JOINT = 2 };
/* friction cones (mjtCone) */
enum { MPCR_CONE_PYRAMIDAL = 0, MPCR_CONE_ELLIPTIC = 1 };
/* integrators (mjtIntegrator) */
enum { MPCR_INT_EULER = 0, MPCR_INT_IMPLICITFAST = 3 };
/* actuator gain / bias types (mjtGain / mjtBias) */
enum { MPCR_GAIN_FIXED = 0, MPCR_GAIN_AFFINE = 1 };
enum { MPCR_BIAS_NONE = 0, MPCR_BIAS_AFFINE = 1 };
/* disable flags (subset of mjtDisableBit semantics) */
enum {
  MPCR_DSBL_EULERDAMP = 1 << 0,
  MPCR_DSBL_REFSAFE   = 1 << 1,
  MPCR_DSBL_WARMSTART = 1 << 2,
  MPCR_DSBL_GRAVITY   = 1 << 3,
  MPCR_DSBL_CONTACT   = 1 << 4,
  MPCR_DSBL_LIMIT     = 1 << 5,
  MPCR_DSBL_EQUALITY  = 1 << 6,
  MPCR_DSBL_PASSIVE   = 1 << 7,
  MPCR_DSBL_FILTERPARENT = 1 << 8
};

typedef struct mpcr_model_t {
  uint32_t magic, version, nbytes, pad0;

  /* sizes */
  int32_t nbody, njnt, nq, nv, ngeom, nsite, npair, neq;
  int32_t ncon;        /* total contact slots (sum of pair_ncon)            */
  int32_t nslot;       /* robot-masked slots, i.e. S of SURVEY §8a-A6        */
  int32_t nctrl;       /* planner-controlled dofs (num_dof, = 6 for UR5e)    */
  int32_t hande_body;  /* body whose xquat is the eef rotation (-1: none)    */
  int32_t tcp_site;    /* site whose xpos is the eef position  (-1: none)    */
  int32_t iterations, ls_iterations, disableflags;
  int32_t integrator, cone;  /* MPCR_INT_*, MPCR_CONE_*                       */
  int32_t ntree;       /* kinematic trees (roots with dofs)                  */
  int32_t nu;          /* actuators                                          */
  int32_t nhullv, nhulla; /* convex-hull vertices / adjacency entries       */
  int32_t pad_sz;

  /* options (mjOption) and statistics */
  double timestep, tolerance, ls_tolerance, impratio, meaninertia;
  double gravity[3];
  double pad1;

  /* bodies (topological order, 0 = world) */
  int32_t body_parentid[MPCR_MAX_BODY];
  int32_t body_rootid[MPCR_MAX_BODY];
  int32_t body_weldid[MPCR_MAX_BODY];
  int32_t body_jntnum[MPCR_MAX_BODY];
  int32_t body_jntadr[MPCR_MAX_BODY];
  int32_t body_dofnum[MPCR_MAX_BODY];
  int32_t body_dofadr[MPCR_MAX_BODY];
  uint32_t body_dofmask[MPCR_MAX_BODY]; /* dofs on the path body..root      */
  double body_pos[MPCR_MAX_BODY][3];
  double body_quat[MPCR_MAX_BODY][4];
  double body_ipos[MPCR_MAX_BODY][3];
  double body_iquat[MPCR_MAX_BODY][4];
  double body_mass[MPCR_MAX_BODY];
  double body_inertia[MPCR_MAX_BODY][3];
  double body_gravcomp[MPCR_MAX_BODY];
  double body_invweight0[MPCR_MAX_BODY][2];

  /* joints */
  int32_t jnt_type[MPCR_MAX_JNT];
  int32_t jnt_qposadr[MPCR_MAX_JNT];
  int32_t jnt_dofadr[MPCR_MAX_JNT];
  int32_t jnt_bodyid[MPCR_MAX_JNT];
  int32_t jnt_limited[MPCR_MAX_JNT];
  double jnt_pos[MPCR_MAX_JNT][3];
  double jnt_axis[MPCR_MAX_JNT][3];
  double jnt_range[MPCR_MAX_JNT][2];
  double jnt_solref[MPCR_MAX_JNT][2];
  double jnt_solimp[MPCR_MAX_JNT][5];
  double jnt_margin[MPCR_MAX_JNT];
  double jnt_stiffness[MPCR_MAX_JNT];
  double jnt_springref[MPCR_MAX_JNT];
  int32_t jnt_actfrclimited[MPCR_MAX_JNT];
  double jnt_actfrcrange[MPCR_MAX_JNT][2];

  /* dofs */
  int32_t dof_bodyid[MPCR_MAX_DOF];
  int32_t dof_jntid[MPCR_MAX_DOF];
  int32_t dof_parentid[MPCR_MAX_DOF];
  int32_t dof_treeid[MPCR_MAX_DOF];
  double dof_armature[MPCR_MAX_DOF];
  double dof_damping[MPCR_MAX_DOF];
  double dof_invweight0[MPCR_MAX_DOF];

  /* reference / template state (mjx_data after forward at qpos0,
     SBP/mjx_planner.py:105-107) */
  double qpos0[MPCR_MAX_NQ];
  double qpos_init[MPCR_MAX_NQ];
  double qvel_init[MPCR_MAX_DOF];

  /* geoms */
  int32_t geom_type[MPCR_MAX_GEOM];
  int32_t geom_bodyid[MPCR_MAX_GEOM];
  int32_t geom_contype[MPCR_MAX_GEOM];
  int32_t geom_conaffinity[MPCR_MAX_GEOM];
  int32_t geom_condim[MPCR_MAX_GEOM];
  int32_t geom_robot[MPCR_MAX_GEOM];   /* 1 if named robot_0..robot_9      */
  double geom_pos[MPCR_MAX_GEOM][3];
  double geom_quat[MPCR_MAX_GEOM][4];
  double geom_size[MPCR_MAX_GEOM][3];
  double geom_rbound[MPCR_MAX_GEOM];

  /* sites */
  int32_t site_bodyid[MPCR_MAX_SITE];
  double site_pos[MPCR_MAX_SITE][3];
  double site_quat[MPCR_MAX_SITE][4];

  /* collision pairs (static candidate list after contype/weld/parent/exclude
     filtering, sorted by narrow-phase function) and their mixed parameters */
  int32_t pair_geom1[MPCR_MAX_PAIR];
  int32_t pair_geom2[MPCR_MAX_PAIR];
  int32_t pair_func[MPCR_MAX_PAIR];
  int32_t pair_ncon[MPCR_MAX_PAIR];
  int32_t pair_conadr[MPCR_MAX_PAIR];   /* first contact slot              */
  int32_t pair_slotadr[MPCR_MAX_PAIR];  /* first robot slot, -1 if unmasked */
  int32_t pair_condim[MPCR_MAX_PAIR];
  int32_t pad2;
  double pair_friction[MPCR_MAX_PAIR];  /* sliding friction (condim 3)     */
  double pair_solref[MPCR_MAX_PAIR][2];
  double pair_solimp[MPCR_MAX_PAIR][5];
  double pair_margin[MPCR_MAX_PAIR];
  double pair_gap[MPCR_MAX_PAIR];

  /* equality constraints */
  int32_t eq_type[MPCR_MAX_EQ];
  int32_t eq_obj1[MPCR_MAX_EQ];
  int32_t eq_obj2[MPCR_MAX_EQ];
  int32_t pad3;
  double eq_data[MPCR_MAX_EQ][6];  /* joint: polycoef[5]; connect: anchor in
                                      body1 | the same point in body2 at qpos0 */
  double eq_solref[MPCR_MAX_EQ][2];
  double eq_solimp[MPCR_MAX_EQ][5];

  /* planner-controlled dofs: qpos/qvel addresses of the num_dof joints
     (SBP/mjx_planner.py:254,267-270 use qpos[:num_dof], qvel[:num_dof]) */
  int32_t ctrl_qposadr[MPCR_MAX_CTRL];
  int32_t ctrl_dofadr[MPCR_MAX_CTRL];

  /* actuators (mjModel actuator_*): joint or fixed-tendon transmissions,
     flattened to at most 2 (dof, moment) entries; force = gain*ctrl + bias,
     gain = gainprm[0] (+ gainprm[1] len + gainprm[2] vel if affine), bias =
     biasprm[0] + biasprm[1] len + biasprm[2] vel, len / vel = moment . qpos /
     qvel; ctrl is the constant actuator_ctrl (the keyframe's) */
  int32_t act_ntrn[MPCR_MAX_ACT];
  int32_t act_dof[MPCR_MAX_ACT][2];
  int32_t act_qadr[MPCR_MAX_ACT][2];
  int32_t act_gaintype[MPCR_MAX_ACT];
  int32_t act_biastype[MPCR_MAX_ACT];
  int32_t act_ctrllimited[MPCR_MAX_ACT];
  int32_t act_forcelimited[MPCR_MAX_ACT];
  int32_t pad4;
  double act_moment[MPCR_MAX_ACT][2];
  double act_gainprm[MPCR_MAX_ACT][3];
  double act_biasprm[MPCR_MAX_ACT][3];
  double act_ctrlrange[MPCR_MAX_ACT][2];
  double act_forcerange[MPCR_MAX_ACT][2];
  double act_ctrl[MPCR_MAX_ACT];

  /* convex hulls of mesh geoms (geom frame) and their vertex graphs (the
     neighbours of every hull vertex, for hill-climbing support queries) */
  int32_t geom_hulladr[MPCR_MAX_GEOM];  /* first vertex, -1: no hull        */
  int32_t geom_hullnum[MPCR_MAX_GEOM];
  int32_t hull_adjadr[MPCR_MAX_HULLV];
  int32_t hull_adjnum[MPCR_MAX_HULLV];
  int32_t hull_adj[MPCR_MAX_HULLA];     /* global vertex indices            */
  double hull_vert[MPCR_MAX_HULLV][3];

  /* v5 (scene_robotiq_hande.xml) */
  /* fluid: mjOption viscosity / density, MuJoCo's inertia-box model per body
     (force -3 pi d eta v, torque -pi d^3 eta w at xipos, d = mean box side) */
  double viscosity, density;
  /* spatial tendons through two sites (no wrapping): length |x_s2 - x_s1|,
     length limits as constraint rows after the joint limits (mj_instantiateLimit) */
  int32_t nten, pad5;
  int32_t ten_site[MPCR_MAX_TEN][2];
  int32_t ten_limited[MPCR_MAX_TEN];
  double ten_range[MPCR_MAX_TEN][2];
  double ten_solref[MPCR_MAX_TEN][2];
  double ten_solimp[MPCR_MAX_TEN][5];
  double ten_margin[MPCR_MAX_TEN];
  double ten_invweight0[MPCR_MAX_TEN]; /* J_ten M^-1 J_ten^T at qpos0 */
  /* v7: polygon faces of the hulls and boxes of polyhedron pairs (mesh-mesh,
     box-mesh): the face-clipping contact manifold
     (mujoco-mjx 3.3.1 convex_convex: a reference face, the incident face
     clipped to it, up to 4 points).  Coplanar hull triangles are merged;
     vertices counter-clockwise about the outward normal, at most
     MPCR_FACE_MAXV kept per face; every vertex lists the faces it lies on. */
  int32_t nface, nfacev, nvface, pad6;
  int32_t geom_faceadr[MPCR_MAX_GEOM]; /* first face, -1: none             */
  int32_t geom_facenum[MPCR_MAX_GEOM];
  int32_t geom_cornadr[MPCR_MAX_GEOM]; /* a box's 8 corners in hull_vert (bit k: + side of axis k), -1 */
  int32_t face_vadr[MPCR_MAX_FACE];
  int32_t face_vnum[MPCR_MAX_FACE];
  int32_t face_vert[MPCR_MAX_FACEV];   /* global hull_vert indices         */
  int32_t vert_faceadr[MPCR_MAX_HULLV];
  int32_t vert_facenum[MPCR_MAX_HULLV];
  int32_t vert_face[MPCR_MAX_VFACE];   /* global face indices              */
  double face_plane[MPCR_MAX_FACE][4]; /* outward normal, offset: n.x = offset on the face (geom frame) */
} mpcr_model_t;

#ifdef __cplusplus
}
#endif
#endif /* MPCR_MODEL_H_ */

/*
 * mpcr_oracle.c — CPU restatement (fp64, scalar C) of the reference's hot
 * path, used ONLY as the parity checker (tests/, __graft_entry__.smoke(),
 * bench.py's cpu_baseline leg).  Never linked into libmpcr.
 *
 * What it restates:
 *   - the rollout / output timing of compute_rollout_single + mjx_step
 *     (SBP/mjx_planner.py:251-274): qvel[:6] <- thetadot_t, step, emit
 *     qpos[:6] post-integration and xquat[hande], site_xpos[tcp],
 *     contact.dist[mask] pre-integration (from forward);
 *   - compute_cost_single (SBP/mjx_planner.py:276-303);
 *   - mjx.step (third-party mujoco-mjx 3.3.1, called at :108,256; not in
 *     /root/reference): kinematics, COM quantities, CRB mass matrix with
 *     armature, RNE bias forces, passive damping + gravcomp, narrow-phase
 *     contacts, pyramidal contact / limit / joint-equality constraints with
 *     solref/solimp impedance, Newton solver (iterations=1, ls_iterations=5,
 *     warm start = better of qacc_warmstart and qacc_smooth), semi-implicit
 *     Euler (eulerdamp disabled);
 *   - the dual-arm features: joint springs, actuators
 *     (gain/bias affine, joint and fixed-tendon transmissions, ctrl/force
 *     clamps, joint actuator-force ranges), connect equalities, the
 *     implicitfast integrator (M - dt*qDeriv with damping and actuator
 *     velocity derivatives, no Coriolis) and general convex collision
 *     (capsule / cylinder / box / sphere / mesh convex hull) by Minkowski
 *     portal refinement (libccd's MPR, one contact per pair, the algorithm
 *     MuJoCo's general convex path used before nativeccd) + plane-convex;
 *   - the scene_robotiq_hande.xml features: elliptic
 *     friction cones with impratio (MuJoCo's three-zone primal cone cost in
 *     the Newton gradient, Hessian and an exact per-contact line search),
 *     inertia-box fluid viscosity, spatial (two-site) tendon length limits.
 *
 * PARITY STATUS: MuJoCo/MJX are not importable or buildable here
 * (SURVEY.md §0.2, §8c), so the physics restatement is pinned only by the
 * reference's own logged CPU-MuJoCo run (SBP/data/theta.csv + thetadot.csv,
 * tests/test_oracle.py::test_replay_*) and by analytic invariants; contact slot
 * layout and solver details are "parity unpinned" (DESIGN.md §Oracle).
 */
#include <math.h>
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mpcr_model.h"

#define NB MPCR_MAX_BODY
#define NV MPCR_MAX_DOF
#define MAXCON (4 * MPCR_MAX_PAIR)
#define MAXEFC 512
#define MINVAL 1e-15
#define MINIMP 0.0001
#define MAXIMP 0.9999
#define PI 3.14159265358979323846

typedef struct {
  double dist, pos[3], frame[9];
  int pair, active;
} ocontact;

typedef struct {
  /* state */
  double qpos[MPCR_MAX_NQ], qvel[NV], qacc[NV], qacc_warmstart[NV];
  /* position-dependent */
  double xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3], ximat[NB][9];
  double xanchor[MPCR_MAX_JNT][3], xaxis[MPCR_MAX_JNT][3];
  double subtree_com[NB][3], cinert[NB][10], crb[NB][10], cdof[NV][6];
  double geom_xpos[MPCR_MAX_GEOM][3], geom_xmat[MPCR_MAX_GEOM][9];
  double site_xpos[MPCR_MAX_SITE][3];
  double M[NV][NV], L[NV][NV];
  /* velocity-dependent */
  double cvel[NB][6], cdof_dot[NV][6];
  double qfrc_bias[NV], qfrc_passive[NV], qfrc_smooth[NV], qacc_smooth[NV];
  double qfrc_actuator[NV], qfrc_constraint[NV], efc_force[MAXEFC];
  /* contacts (all slots) */
  int ncon;
  ocontact con[MAXCON];
  /* constraints */
  int nefc, efc_eq[MAXEFC];
  /* efc_eq: 0 inequality (quadratic when jar < 0), 1 equality (always
     quadratic), 2 elliptic contact: the normal row owns rows r..r+efc_dim-1,
     3 elliptic friction row (evaluated by its normal row) */
  int efc_dim[MAXEFC];
  double efc_mu[MAXEFC], efc_fri[MAXEFC][2];
  double efc_J[MAXEFC][NV], efc_pos[MAXEFC], efc_margin[MAXEFC], efc_D[MAXEFC];
  double efc_aref[MAXEFC], efc_diag[MAXEFC], efc_vel[MAXEFC];
  double efc_solref[MAXEFC][2], efc_solimp[MAXEFC][5];
  int efc_trunc; /* constraint rows dropped for capacity (should stay 0) */
  int hint[MPCR_MAX_PAIR][2]; /* hull-climb start per pair and side (-1: none), kept across steps */
  double dbg[8]; /* solver record of the step (oracle_step_debug, the kernel's DBG_INFO) */
  double dbg_gs[64]; /* first Newton iteration's gradient | search direction */
  double* ls_dump; /* non-null: the first line search's inputs (oracle_ls_inputs) */
} odata;

static void reset_hints(odata* d) {
  for (int p = 0; p < MPCR_MAX_PAIR; p++) d->hint[p][0] = d->hint[p][1] = -1;
}

/* ------------------------------------------------------------------------ */
/* small math                                                                */

static void q2m(const double q[4], double m[9]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
static void qmul(double r[4], const double a[4], const double b[4]) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof(t));
}
static void qnorm(double q[4]) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
static void mulmv(double r[3], const double m[9], const double v[3]) {
  double t[3] = {m[0] * v[0] + m[1] * v[1] + m[2] * v[2], m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
                 m[6] * v[0] + m[7] * v[1] + m[8] * v[2]};
  memcpy(r, t, sizeof(t));
}
static void mulmtv(double r[3], const double m[9], const double v[3]) {
  double t[3] = {m[0] * v[0] + m[3] * v[1] + m[6] * v[2], m[1] * v[0] + m[4] * v[1] + m[7] * v[2],
                 m[2] * v[0] + m[5] * v[1] + m[8] * v[2]};
  memcpy(r, t, sizeof(t));
}
static void mulmm(double r[9], const double a[9], const double b[9]) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  memcpy(r, t, sizeof(t));
}
static void cross3(double r[3], const double a[3], const double b[3]) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  memcpy(r, t, sizeof(t));
}
static double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double norm3(const double a[3]) { return sqrt(dot3(a, a)); }
static void axisangle(double q[4], const double ax[3], double ang) {
  double s = sin(0.5 * ang);
  q[0] = cos(0.5 * ang); q[1] = ax[0] * s; q[2] = ax[1] * s; q[3] = ax[2] * s;
}
static double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* spatial algebra, MuJoCo layout: motion/force = [angular(3); linear(3)] and
   10-vector inertia {Ixx,Iyy,Izz,Ixy,Ixz,Iyz, m*cx,m*cy,m*cz, m} about the
   tree's subtree_com (mju_mulInertVec / mju_crossMotion / mju_crossForce). */
static void mul_inert_vec(double r[6], const double i[10], const double v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
static void cross_motion(double r[6], const double v[6], const double u[6]) {
  double a[3], b[3], c[3];
  cross3(a, v, u);
  cross3(b, v, u + 3);
  cross3(c, v + 3, u);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
static void cross_force(double r[6], const double v[6], const double f[6]) {
  double a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}

/* dense Cholesky (lower) of the leading n x n block; returns 0 on success */
static int chol(double L[NV][NV], const double A[NV][NV], int n) {
  for (int j = 0; j < n; j++) {
    double s = A[j][j];
    for (int k = 0; k < j; k++) s -= L[j][k] * L[j][k];
    if (s <= MINVAL) s = MINVAL;
    L[j][j] = sqrt(s);
    for (int i = j + 1; i < n; i++) {
      double t = A[i][j];
      for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k];
      L[i][j] = t / L[j][j];
    }
    for (int i = 0; i < j; i++) L[i][j] = 0;
  }
  return 0;
}
static void chol_solve(double x[NV], const double L[NV][NV], const double b[NV], int n) {
  double y[NV];
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < n; k++) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
}

/* ------------------------------------------------------------------------ */
/* kinematics + COM quantities + CRB (mj_kinematics, mj_comPos, mj_crb)      */

static void kinematics(const mpcr_model_t* m, odata* d) {
  d->xpos[0][0] = d->xpos[0][1] = d->xpos[0][2] = 0;
  d->xquat[0][0] = 1; d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  q2m(d->xquat[0], d->xmat[0]);
  memcpy(d->xipos[0], d->xpos[0], sizeof(d->xpos[0]));
  memcpy(d->ximat[0], d->xmat[0], sizeof(d->xmat[0]));
  for (int b = 1; b < m->nbody; b++) {
    int p = m->body_parentid[b];
    double pos[3], quat[4], tmp[3];
    int j0 = m->body_jntadr[b], nj = m->body_jntnum[b];
    if (nj > 0 && m->jnt_type[j0] == MPCR_JNT_FREE) {
      int a = m->jnt_qposadr[j0];
      memcpy(pos, d->qpos + a, 3 * sizeof(double));
      memcpy(quat, d->qpos + a + 3, 4 * sizeof(double));
      qnorm(quat);
      memcpy(d->xanchor[j0], pos, sizeof(pos));
      d->xaxis[j0][0] = 0; d->xaxis[j0][1] = 0; d->xaxis[j0][2] = 1;
    } else {
      mulmv(tmp, d->xmat[p], m->body_pos[b]);
      for (int k = 0; k < 3; k++) pos[k] = d->xpos[p][k] + tmp[k];
      qmul(quat, d->xquat[p], m->body_quat[b]);
      for (int j = j0; j < j0 + nj; j++) {
        double R[9], qa = d->qpos[m->jnt_qposadr[j]] - m->qpos0[m->jnt_qposadr[j]];
        q2m(quat, R);
        mulmv(d->xaxis[j], R, m->jnt_axis[j]);
        mulmv(tmp, R, m->jnt_pos[j]);
        for (int k = 0; k < 3; k++) d->xanchor[j][k] = tmp[k] + pos[k];
        if (m->jnt_type[j] == MPCR_JNT_SLIDE) {
          for (int k = 0; k < 3; k++) pos[k] += d->xaxis[j][k] * qa;
        } else if (m->jnt_type[j] == MPCR_JNT_HINGE) {
          double ql[4];
          axisangle(ql, m->jnt_axis[j], qa);
          qmul(quat, quat, ql);
          q2m(quat, R);
          mulmv(tmp, R, m->jnt_pos[j]);
          for (int k = 0; k < 3; k++) pos[k] = d->xanchor[j][k] - tmp[k];
        }
      }
      qnorm(quat);
    }
    memcpy(d->xpos[b], pos, sizeof(pos));
    memcpy(d->xquat[b], quat, sizeof(quat));
    q2m(quat, d->xmat[b]);
    mulmv(tmp, d->xmat[b], m->body_ipos[b]);
    for (int k = 0; k < 3; k++) d->xipos[b][k] = d->xpos[b][k] + tmp[k];
    double Ri[9];
    q2m(m->body_iquat[b], Ri);
    mulmm(d->ximat[b], d->xmat[b], Ri);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    double tmp[3], R[9];
    mulmv(tmp, d->xmat[b], m->geom_pos[g]);
    for (int k = 0; k < 3; k++) d->geom_xpos[g][k] = d->xpos[b][k] + tmp[k];
    q2m(m->geom_quat[g], R);
    mulmm(d->geom_xmat[g], d->xmat[b], R);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    double tmp[3];
    mulmv(tmp, d->xmat[b], m->site_pos[s]);
    for (int k = 0; k < 3; k++) d->site_xpos[s][k] = d->xpos[b][k] + tmp[k];
  }
}

static void com_pos(const mpcr_model_t* m, odata* d) {
  double sm[NB], smc[NB][3];
  for (int b = 0; b < m->nbody; b++) {
    sm[b] = m->body_mass[b];
    for (int k = 0; k < 3; k++) smc[b][k] = m->body_mass[b] * d->xipos[b][k];
  }
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    sm[p] += sm[b];
    for (int k = 0; k < 3; k++) smc[p][k] += smc[b][k];
  }
  for (int b = 0; b < m->nbody; b++)
    for (int k = 0; k < 3; k++) d->subtree_com[b][k] = sm[b] > MINVAL ? smc[b][k] / sm[b] : d->xipos[b][k];
  /* cinert: inertia about subtree_com[root], world orientation (mju_inertCom) */
  memset(d->cinert[0], 0, sizeof(d->cinert[0]));
  for (int b = 1; b < m->nbody; b++) {
    const double* R = d->ximat[b];
    const double* I = m->body_inertia[b];
    double mass = m->body_mass[b], dif[3], full[9];
    for (int k = 0; k < 3; k++) dif[k] = d->xipos[b][k] - d->subtree_com[m->body_rootid[b]][k];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        full[3 * i + j] = R[3 * i] * I[0] * R[3 * j] + R[3 * i + 1] * I[1] * R[3 * j + 1] + R[3 * i + 2] * I[2] * R[3 * j + 2];
    double dd = dot3(dif, dif);
    double* c = d->cinert[b];
    c[0] = full[0] + mass * (dd - dif[0] * dif[0]);
    c[1] = full[4] + mass * (dd - dif[1] * dif[1]);
    c[2] = full[8] + mass * (dd - dif[2] * dif[2]);
    c[3] = full[1] - mass * dif[0] * dif[1];
    c[4] = full[2] - mass * dif[0] * dif[2];
    c[5] = full[5] - mass * dif[1] * dif[2];
    c[6] = mass * dif[0]; c[7] = mass * dif[1]; c[8] = mass * dif[2];
    c[9] = mass;
  }
  /* cdof (mju_dofCom) */
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j], d0 = m->jnt_dofadr[j];
    const double* com = d->subtree_com[m->body_rootid[b]];
    double off[3];
    for (int k = 0; k < 3; k++) off[k] = com[k] - d->xanchor[j][k];
    switch (m->jnt_type[j]) {
      case MPCR_JNT_FREE:
        for (int i = 0; i < 3; i++) {
          double* c = d->cdof[d0 + i];
          memset(c, 0, 6 * sizeof(double));
          c[3 + i] = 1;
        }
        d0 += 3; /* fall through to the rotational part */
      case MPCR_JNT_BALL:
        for (int i = 0; i < 3; i++) {
          double ax[3] = {d->xmat[b][i], d->xmat[b][3 + i], d->xmat[b][6 + i]};
          double* c = d->cdof[d0 + i];
          memcpy(c, ax, sizeof(ax));
          cross3(c + 3, ax, off);
        }
        break;
      case MPCR_JNT_SLIDE: {
        double* c = d->cdof[d0];
        c[0] = c[1] = c[2] = 0;
        memcpy(c + 3, d->xaxis[j], 3 * sizeof(double));
        break;
      }
      default: {
        double* c = d->cdof[d0];
        memcpy(c, d->xaxis[j], 3 * sizeof(double));
        cross3(c + 3, d->xaxis[j], off);
      }
    }
  }
}

static void crb(const mpcr_model_t* m, odata* d) {
  memcpy(d->crb, d->cinert, sizeof(double) * 10 * m->nbody);
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[p][k] += d->crb[b][k];
  }
  int nv = m->nv;
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) d->M[i][j] = 0;
  for (int i = 0; i < nv; i++) {
    double f[6];
    mul_inert_vec(f, d->crb[m->dof_bodyid[i]], d->cdof[i]);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      double v = 0;
      for (int k = 0; k < 6; k++) v += d->cdof[j][k] * f[k];
      d->M[i][j] = v;
      d->M[j][i] = v;
    }
    d->M[i][i] += m->dof_armature[i];
  }
  chol(d->L, d->M, nv);
}

/* translational Jacobian row-block of a world point attached to body b:
   jac[k][dof] (mj_jac) */
static void jac_point(const mpcr_model_t* m, const odata* d, int b, const double p[3], double jac[3][NV]) {
  const double* com = d->subtree_com[m->body_rootid[b]];
  double r[3] = {p[0] - com[0], p[1] - com[1], p[2] - com[2]};
  for (int i = 0; i < m->nv; i++) {
    if (b > 0 && (m->body_dofmask[b] >> i & 1u)) {
      double c[3];
      cross3(c, d->cdof[i], r);
      for (int k = 0; k < 3; k++) jac[k][i] = d->cdof[i][3 + k] + c[k];
    } else {
      jac[0][i] = jac[1][i] = jac[2][i] = 0;
    }
  }
}

/* ------------------------------------------------------------------------ */
/* velocity: mj_comVel, mj_passive, mj_rne                                   */

static void com_vel(const mpcr_model_t* m, odata* d) {
  memset(d->cvel[0], 0, sizeof(d->cvel[0]));
  for (int b = 1; b < m->nbody; b++) {
    double cv[6];
    memcpy(cv, d->cvel[m->body_parentid[b]], sizeof(cv));
    int j0 = m->body_jntadr[b];
    for (int j = j0; j < j0 + m->body_jntnum[b]; j++) {
      int d0 = m->jnt_dofadr[j];
      if (m->jnt_type[j] == MPCR_JNT_FREE) {
        for (int i = 0; i < 3; i++) memset(d->cdof_dot[d0 + i], 0, 6 * sizeof(double));
        for (int i = 0; i < 3; i++)
          for (int k = 0; k < 6; k++) cv[k] += d->cdof[d0 + i][k] * d->qvel[d0 + i];
        d0 += 3;
        for (int i = 0; i < 3; i++) cross_motion(d->cdof_dot[d0 + i], cv, d->cdof[d0 + i]);
        for (int i = 0; i < 3; i++)
          for (int k = 0; k < 6; k++) cv[k] += d->cdof[d0 + i][k] * d->qvel[d0 + i];
      } else if (m->jnt_type[j] == MPCR_JNT_BALL) {
        for (int i = 0; i < 3; i++) cross_motion(d->cdof_dot[d0 + i], cv, d->cdof[d0 + i]);
        for (int i = 0; i < 3; i++)
          for (int k = 0; k < 6; k++) cv[k] += d->cdof[d0 + i][k] * d->qvel[d0 + i];
      } else {
        cross_motion(d->cdof_dot[d0], cv, d->cdof[d0]);
        for (int k = 0; k < 6; k++) cv[k] += d->cdof[d0][k] * d->qvel[d0];
      }
    }
    memcpy(d->cvel[b], cv, sizeof(cv));
  }
}

static void passive(const mpcr_model_t* m, odata* d) {
  for (int i = 0; i < m->nv; i++) d->qfrc_passive[i] = 0;
  if (m->disableflags & MPCR_DSBL_PASSIVE) return;
  for (int i = 0; i < m->nv; i++) d->qfrc_passive[i] = -m->dof_damping[i] * d->qvel[i];
  /* joint springs (hinge / slide): -stiffness (q - springref) */
  for (int j = 0; j < m->njnt; j++) {
    if (m->jnt_stiffness[j] == 0 || (m->jnt_type[j] != MPCR_JNT_HINGE && m->jnt_type[j] != MPCR_JNT_SLIDE)) continue;
    d->qfrc_passive[m->jnt_dofadr[j]] -= m->jnt_stiffness[j] * (d->qpos[m->jnt_qposadr[j]] - m->jnt_springref[j]);
  }
  /* gravity compensation: -gravity*mass*gravcomp applied at xipos */
  for (int b = 1; b < m->nbody; b++) {
    double gc = m->body_gravcomp[b];
    if (gc == 0 || m->body_mass[b] == 0) continue;
    double f[3], jac[3][NV];
    for (int k = 0; k < 3; k++) f[k] = -m->gravity[k] * m->body_mass[b] * gc;
    jac_point(m, d, b, d->xipos[b], jac);
    for (int i = 0; i < m->nv; i++) d->qfrc_passive[i] += jac[0][i] * f[0] + jac[1][i] * f[1] + jac[2][i] * f[2];
  }
  /* fluid viscosity, MuJoCo's inertia-box model (mj_inertiaBoxFluidModel)
     with density 0: the body's equivalent inertia box gives the sphere
     diameter d = mean side; force -3 pi d eta v and torque -pi d^3 eta w at
     xipos.  Both are isotropic, so the world-frame velocities serve. */
  if (m->viscosity > 0)
    for (int b = 1; b < m->nbody; b++) {
      double mass = m->body_mass[b];
      if (mass < MINVAL) continue;
      const double* I = m->body_inertia[b];
      double diam = 0;
      for (int k = 0; k < 3; k++) {
        double x = I[(k + 1) % 3] + I[(k + 2) % 3] - I[k];
        diam += sqrt((x > MINVAL ? x : MINVAL) / mass * 6) / 3;
      }
      const double* cv = d->cvel[b];
      const double* com = d->subtree_com[m->body_rootid[b]];
      double r[3] = {d->xipos[b][0] - com[0], d->xipos[b][1] - com[1], d->xipos[b][2] - com[2]}, wr[3];
      cross3(wr, cv, r);
      double fl = -3 * PI * diam * m->viscosity, fa = -PI * diam * diam * diam * m->viscosity;
      double f[3], t[3], jac[3][NV];
      for (int k = 0; k < 3; k++) { f[k] = fl * (cv[3 + k] + wr[k]); t[k] = fa * cv[k]; }
      jac_point(m, d, b, d->xipos[b], jac);
      for (int i = 0; i < m->nv; i++) {
        double q = jac[0][i] * f[0] + jac[1][i] * f[1] + jac[2][i] * f[2];
        if (m->body_dofmask[b] >> i & 1u) q += d->cdof[i][0] * t[0] + d->cdof[i][1] * t[1] + d->cdof[i][2] * t[2];
        d->qfrc_passive[i] += q;
      }
    }
}

static void rne(const mpcr_model_t* m, odata* d) {
  double cacc[NB][6], cfrc[NB][6];
  memset(cacc[0], 0, sizeof(cacc[0]));
  if (!(m->disableflags & MPCR_DSBL_GRAVITY))
    for (int k = 0; k < 3; k++) cacc[0][3 + k] = -m->gravity[k];
  for (int b = 1; b < m->nbody; b++) {
    memcpy(cacc[b], cacc[m->body_parentid[b]], sizeof(cacc[b]));
    for (int i = m->body_dofadr[b]; i < m->body_dofadr[b] + m->body_dofnum[b]; i++)
      for (int k = 0; k < 6; k++) cacc[b][k] += d->cdof_dot[i][k] * d->qvel[i];
    double t1[6], t2[6];
    mul_inert_vec(cfrc[b], d->cinert[b], cacc[b]);
    mul_inert_vec(t1, d->cinert[b], d->cvel[b]);
    cross_force(t2, d->cvel[b], t1);
    for (int k = 0; k < 6; k++) cfrc[b][k] += t2[k];
  }
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p > 0)
      for (int k = 0; k < 6; k++) cfrc[p][k] += cfrc[b][k];
  }
  for (int i = 0; i < m->nv; i++) {
    double v = 0;
    for (int k = 0; k < 6; k++) v += d->cdof[i][k] * cfrc[m->dof_bodyid[i]][k];
    d->qfrc_bias[i] = v;
  }
}

/* actuation (mj_fwdActuation): force = gain ctrl + bias on the transmission
   length / velocity, clamped, mapped through the moments; joint-level
   actuator force ranges clamp the sum */
static void actuation(const mpcr_model_t* m, odata* d) {
  for (int i = 0; i < m->nv; i++) d->qfrc_actuator[i] = 0;
  for (int a = 0; a < m->nu; a++) {
    double len = 0, vel = 0;
    for (int k = 0; k < m->act_ntrn[a]; k++) {
      len += m->act_moment[a][k] * d->qpos[m->act_qadr[a][k]];
      vel += m->act_moment[a][k] * d->qvel[m->act_dof[a][k]];
    }
    double ctrl = m->act_ctrl[a];
    if (m->act_ctrllimited[a]) ctrl = clampd(ctrl, m->act_ctrlrange[a][0], m->act_ctrlrange[a][1]);
    const double* g = m->act_gainprm[a];
    const double* b = m->act_biasprm[a];
    double gain = m->act_gaintype[a] == MPCR_GAIN_AFFINE ? g[0] + g[1] * len + g[2] * vel : g[0];
    double bias = m->act_biastype[a] == MPCR_BIAS_AFFINE ? b[0] + b[1] * len + b[2] * vel : 0;
    double f = gain * ctrl + bias;
    if (m->act_forcelimited[a]) f = clampd(f, m->act_forcerange[a][0], m->act_forcerange[a][1]);
    for (int k = 0; k < m->act_ntrn[a]; k++) d->qfrc_actuator[m->act_dof[a][k]] += m->act_moment[a][k] * f;
  }
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_actfrclimited[j]) continue;
    int v = m->jnt_dofadr[j];
    d->qfrc_actuator[v] = clampd(d->qfrc_actuator[v], m->jnt_actfrcrange[j][0], m->jnt_actfrcrange[j][1]);
  }
}

/* implicitfast velocity derivative of the smooth force (mjd_smooth_vel
   without the RNE term): -damping on the diagonal + sum_a dforce/dvel m m^T */
static void qderiv(const mpcr_model_t* m, double D[NV][NV]) {
  for (int i = 0; i < m->nv; i++)
    for (int j = 0; j < m->nv; j++) D[i][j] = i == j ? -m->dof_damping[i] : 0;
  if (m->disableflags & MPCR_DSBL_PASSIVE)
    for (int i = 0; i < m->nv; i++) D[i][i] = 0;
  for (int a = 0; a < m->nu; a++) {
    double dv = 0;
    if (m->act_biastype[a] == MPCR_BIAS_AFFINE) dv += m->act_biasprm[a][2];
    if (m->act_gaintype[a] == MPCR_GAIN_AFFINE) {
      double ctrl = m->act_ctrl[a];
      if (m->act_ctrllimited[a]) ctrl = clampd(ctrl, m->act_ctrlrange[a][0], m->act_ctrlrange[a][1]);
      dv += m->act_gainprm[a][2] * ctrl;
    }
    for (int k = 0; k < m->act_ntrn[a]; k++)
      for (int l = 0; l < m->act_ntrn[a]; l++)
        D[m->act_dof[a][k]][m->act_dof[a][l]] += dv * m->act_moment[a][k] * m->act_moment[a][l];
  }
}

/* ------------------------------------------------------------------------ */
/* narrow phase (contact definitions shared with the HIP kernel: DESIGN.md   */
/* "Contact slot layout").  normal points from geom1 to geom2.              */

static void make_frame(double f[9], const double n[3]) {
  /* mju_makeFrame: x = normal, y from (0,1,0) or (0,0,1), z = x cross y */
  memcpy(f, n, 3 * sizeof(double));
  double y[3] = {0, 1, 0};
  if (fabs(n[1]) >= 0.5) { y[0] = 0; y[1] = 0; y[2] = 1; }
  double dd = dot3(n, y);
  for (int k = 0; k < 3; k++) y[k] -= dd * n[k];
  double ny = norm3(y);
  for (int k = 0; k < 3; k++) f[3 + k] = y[k] / ny;
  cross3(f + 6, f, f + 3);
}

static void set_contact(ocontact* c, double dist, const double pos[3], const double n[3]) {
  c->dist = dist;
  memcpy(c->pos, pos, 3 * sizeof(double));
  make_frame(c->frame, n);
}

static void col_plane_capsule(const odata* d, int gp, int gc, const double* sz, ocontact* out) {
  const double* R = d->geom_xmat[gp];
  double n[3] = {R[2], R[5], R[8]};
  const double* Rc = d->geom_xmat[gc];
  double ax[3] = {Rc[2], Rc[5], Rc[8]};
  double r = sz[0], hl = sz[1];
  for (int s = 0; s < 2; s++) {
    double sg = s == 0 ? 1.0 : -1.0, e[3], dif[3], pos[3];
    for (int k = 0; k < 3; k++) e[k] = d->geom_xpos[gc][k] + sg * hl * ax[k];
    for (int k = 0; k < 3; k++) dif[k] = e[k] - d->geom_xpos[gp][k];
    double dist = dot3(n, dif) - r;
    for (int k = 0; k < 3; k++) pos[k] = e[k] - n[k] * (r + 0.5 * dist);
    set_contact(&out[s], dist, pos, n);
  }
}

static void col_plane_box(const odata* d, int gp, int gb, const double* h, ocontact* out) {
  const double* R = d->geom_xmat[gp];
  double n[3] = {R[2], R[5], R[8]};
  const double* Rb = d->geom_xmat[gb];
  double dist[8], corner[8][3];
  for (int c = 0; c < 8; c++) {
    double l[3] = {(c & 1) ? h[0] : -h[0], (c & 2) ? h[1] : -h[1], (c & 4) ? h[2] : -h[2]}, w[3], dif[3];
    mulmv(w, Rb, l);
    for (int k = 0; k < 3; k++) corner[c][k] = d->geom_xpos[gb][k] + w[k];
    for (int k = 0; k < 3; k++) dif[k] = corner[c][k] - d->geom_xpos[gp][k];
    dist[c] = dot3(n, dif);
  }
  /* the 4 deepest corners, ascending depth order, ties by corner index */
  int used = 0;
  for (int s = 0; s < 4; s++) {
    int best = -1;
    for (int c = 0; c < 8; c++)
      if (!(used >> c & 1) && (best < 0 || dist[c] < dist[best])) best = c;
    used |= 1 << best;
    double pos[3];
    for (int k = 0; k < 3; k++) pos[k] = corner[best][k] - n[k] * 0.5 * dist[best];
    set_contact(&out[s], dist[best], pos, n);
  }
}

/* closest points between segments p1+s*d1 (s in [0,1]) and p2+t*d2 */
static void seg_seg(const double p1[3], const double d1[3], const double p2[3], const double d2[3],
                    double* sc, double* tc) {
  double r[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
  double a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  double s, t;
  if (a <= MINVAL && e <= MINVAL) { *sc = 0; *tc = 0; return; }
  if (a <= MINVAL) {
    s = 0; t = clampd(f / e, 0, 1);
  } else {
    double c = dot3(d1, r);
    if (e <= MINVAL) {
      t = 0; s = clampd(-c / a, 0, 1);
    } else {
      double b = dot3(d1, d2), den = a * e - b * b;
      s = den > 1e-12 * a * e ? clampd((b * f - c * e) / den, 0, 1) : 0;
      t = (b * s + f) / e;
      if (t < 0) { t = 0; s = clampd(-c / a, 0, 1); }
      else if (t > 1) { t = 1; s = clampd((b - c) / a, 0, 1); }
    }
  }
  *sc = s; *tc = t;
}

static void any_normal(double n[3], const double a[3]) {
  /* a unit vector perpendicular to a (fallback for coincident points) */
  double t[3] = {1, 0, 0};
  if (fabs(a[0]) > 0.9) { t[0] = 0; t[1] = 1; }
  cross3(n, a, t);
  double l = norm3(n);
  for (int k = 0; k < 3; k++) n[k] /= l;
}

static void col_capsule_capsule(const odata* d, int g1, int g2, const double* s1, const double* s2,
                                ocontact* out) {
  const double *R1 = d->geom_xmat[g1], *R2 = d->geom_xmat[g2];
  double a1[3] = {R1[2], R1[5], R1[8]}, a2[3] = {R2[2], R2[5], R2[8]};
  double p1[3], p2[3], d1[3], d2[3];
  for (int k = 0; k < 3; k++) {
    p1[k] = d->geom_xpos[g1][k] - s1[1] * a1[k]; d1[k] = 2 * s1[1] * a1[k];
    p2[k] = d->geom_xpos[g2][k] - s2[1] * a2[k]; d2[k] = 2 * s2[1] * a2[k];
  }
  double s, t, c1[3], c2[3], n[3];
  seg_seg(p1, d1, p2, d2, &s, &t);
  for (int k = 0; k < 3; k++) { c1[k] = p1[k] + s * d1[k]; c2[k] = p2[k] + t * d2[k]; n[k] = c2[k] - c1[k]; }
  double len = norm3(n);
  if (len < 1e-12) any_normal(n, a1);
  else for (int k = 0; k < 3; k++) n[k] /= len;
  double dist = len - s1[0] - s2[0], pos[3];
  for (int k = 0; k < 3; k++) pos[k] = c1[k] + n[k] * (s1[0] + 0.5 * dist);
  set_contact(&out[0], dist, pos, n);
}

/* signed distance of a box-local point to a box (half sizes h); returns the
   local normal pointing from the point towards the box surface region the
   point must move along to reach the box (from geom1 = point's owner to
   geom2 = box) and the closest/deepest box surface point. */
static double point_box(const double p[3], const double h[3], double nl[3], double q[3]) {
  double o[3], out2 = 0;
  for (int k = 0; k < 3; k++) {
    q[k] = clampd(p[k], -h[k], h[k]);
    o[k] = q[k] - p[k];
    out2 += o[k] * o[k];
  }
  if (out2 > 0) {
    double l = sqrt(out2);
    for (int k = 0; k < 3; k++) nl[k] = o[k] / l;
    return l;
  }
  /* inside: deepest face is the one with max(|p_k| - h_k); ties (within
     1 um) go to the lower axis and, for a point on the mid-plane of the box
     (a capsule pushed right through a thin box), to the + face -- the
     kernel's rule, so fp32 and fp64 pick the same face */
  int best = 0;
  double g = fabs(p[0]) - h[0];
  for (int k = 1; k < 3; k++)
    if (fabs(p[k]) - h[k] > g + 1e-6) { g = fabs(p[k]) - h[k]; best = k; }
  double sg = p[best] >= -1e-6 ? 1.0 : -1.0;
  nl[0] = nl[1] = nl[2] = 0;
  nl[best] = -sg;
  memcpy(q, p, 3 * sizeof(double));
  q[best] = sg * h[best];
  return g;
}

static void col_capsule_box(const odata* d, int gc, int gb, const double* sc, const double* h,
                            ocontact* out) {
  const double* Rc = d->geom_xmat[gc];
  const double* Rb = d->geom_xmat[gb];
  double ax[3] = {Rc[2], Rc[5], Rc[8]}, r = sc[0], hl = sc[1];
  double A[3], B[3], a[3], dd[3], tmp[3];
  for (int k = 0; k < 3; k++) {
    A[k] = d->geom_xpos[gc][k] - hl * ax[k] - d->geom_xpos[gb][k];
    B[k] = 2 * hl * ax[k];
  }
  mulmtv(a, Rb, A);
  mulmtv(dd, Rb, B);
  /* f(t) = sum_k max(|a_k + t dd_k| - h_k, 0)^2 is convex, C1, piecewise
     quadratic; f'(t) is monotone and piecewise linear between the knots
     t in {0, 1, (+-h_k - a_k)/dd_k}. */
  double knots[8];
  int nk = 0;
  knots[nk++] = 0;
  knots[nk++] = 1;
  for (int k = 0; k < 3; k++) {
    if (fabs(dd[k]) > MINVAL) {
      for (int sgn = -1; sgn <= 1; sgn += 2) {
        double t = (sgn * h[k] - a[k]) / dd[k];
        if (t > 0 && t < 1) knots[nk++] = t;
      }
    }
  }
  double tlo = -1, thi = 2, flo = 0, fhi = 0;
  for (int i = 0; i < nk; i++) {
    double t = knots[i], fp = 0;
    for (int k = 0; k < 3; k++) {
      double x = a[k] + t * dd[k], e = fabs(x) - h[k];
      if (e > 0) fp += 2 * dd[k] * (x > 0 ? e : -e);
    }
    if (fp < 0) { if (t > tlo) { tlo = t; flo = fp; } }
    else { if (t < thi) { thi = t; fhi = fp; } }
  }
  double ts;
  if (tlo < 0) ts = 0;
  else if (thi > 1) ts = 1;
  else ts = fhi - flo > 0 ? tlo - flo * (thi - tlo) / (fhi - flo) : tlo;
  double p[3], q[3], nl[3];
  for (int k = 0; k < 3; k++) p[k] = a[k] + ts * dd[k];
  double g = point_box(p, h, nl, q);
  /* a penetrating segment makes the minimiser above land on the box surface
     (the entry of f's zero interval), g = 0 up to rounding: anything within
     1 um of the surface takes the deepest-point path, so fp32 and fp64 agree
     on the branch (the kernel uses the same band) */
  if (g <= 1e-6) {
    /* segment reaches the box: deepest point of the convex, piecewise linear
       g(t) = max_k(|x_k(t)| - h_k) over its kinks */
    double cand[17];
    int nc = 0;
    cand[nc++] = 0;
    cand[nc++] = 1;
    for (int k = 0; k < 3; k++)
      if (fabs(dd[k]) > MINVAL) { double t = -a[k] / dd[k]; if (t > 0 && t < 1) cand[nc++] = t; }
    for (int i = 0; i < 3; i++)
      for (int j = i + 1; j < 3; j++)
        for (int si = -1; si <= 1; si += 2)
          for (int sj = -1; sj <= 1; sj += 2) {
            double den = si * dd[i] - sj * dd[j];
            if (fabs(den) > MINVAL) {
              double t = (h[i] - h[j] - si * a[i] + sj * a[j]) / den;
              if (t > 0 && t < 1) cand[nc++] = t;
            }
          }
    double gbest = 1e300, tbest = 0;
    for (int c = 0; c < nc; c++) {
      double gm = -1e300;
      for (int k = 0; k < 3; k++) {
        double e = fabs(a[k] + cand[c] * dd[k]) - h[k];
        if (e > gm) gm = e;
      }
      /* a flat minimum (the segment parallel to a face: every kink as deep)
         keeps the first candidate: a later one must be deeper by more than
         1 um (otherwise rounding picks a point anywhere along the segment) */
      if (gm < gbest - 1e-6) { gbest = gm; tbest = cand[c]; }
    }
    ts = tbest;
    for (int k = 0; k < 3; k++) p[k] = a[k] + ts * dd[k];
    g = point_box(p, h, nl, q);
  }
  /* The second contact (round 4): when the first point is on or in the box,
     the far end takes the same box face -- its distance to that face's plane,
     the segment clipped to the face's extent (the end moved back along the
     segment to where it leaves the face rectangle) -- as MJX's capsule-convex
     clipping keeps both contacts on one reference face.  Its own point_box
     (round 3) switched between the face's normal and the direction to the box
     edge as the end crossed the table's edge, a discontinuity fp32 and fp64
     took differently (the fp32 restatement's C4
     well-conditioned misses 12 -> 8).  A first point outside the box keeps
     point_box for the far end. */
  int fk = -1;
  double fsg = 0;
  if (g <= 0) {
    for (int k = 0; k < 3; k++) if (nl[k] != 0) { fk = k; fsg = -nl[k]; }
  }
  for (int s = 0; s < 2; s++) {
    double t = s == 0 ? ts : (ts < 0.5 ? 1.0 : 0.0);
    if (s == 1) {
      if (fk >= 0) {
        for (int j = 0; j < 3; j++) {
          if (j == fk || fabs(dd[j]) <= MINVAL) continue;
          const double x = a[j] + t * dd[j];
          if (fabs(x) > h[j]) {
            const double tb = ((x > 0 ? h[j] : -h[j]) - a[j]) / dd[j];
            t = ts < t ? fmin(t, fmax(tb, ts)) : fmax(t, fmin(tb, ts));
          }
        }
        for (int k = 0; k < 3; k++) p[k] = a[k] + t * dd[k];
        nl[0] = nl[1] = nl[2] = 0;
        nl[fk] = -fsg;
        memcpy(q, p, 3 * sizeof(double));
        q[fk] = fsg * h[fk];
        g = fsg * p[fk] - h[fk];
      } else {
        for (int k = 0; k < 3; k++) p[k] = a[k] + t * dd[k];
        g = point_box(p, h, nl, q);
      }
    }
    double n[3], pl[3], pos[3];
    mulmv(n, Rb, nl);
    for (int k = 0; k < 3; k++) pl[k] = 0.5 * (p[k] + r * nl[k] + q[k]);
    mulmv(tmp, Rb, pl);
    for (int k = 0; k < 3; k++) pos[k] = tmp[k] + d->geom_xpos[gb][k];
    set_contact(&out[s], g - r, pos, n);
  }
}

static void col_box_box(const odata* d, int ga, int gb, const double* ha, const double* hb,
                        double margin, ocontact* out) {
  const double *Ra = d->geom_xmat[ga], *Rb = d->geom_xmat[gb];
  double axA[3][3], axB[3][3], t[3];
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { axA[i][k] = Ra[3 * k + i]; axB[i][k] = Rb[3 * k + i]; }
  for (int k = 0; k < 3; k++) t[k] = d->geom_xpos[gb][k] - d->geom_xpos[ga][k];
  for (int s = 0; s < 4; s++) out[s].dist = 1e30;
  /* separating-axis test: 3 + 3 face axes, 9 edge axes */
  double best_face = -1e300, best_edge = -1e300, Lf[3] = {0, 0, 1}, Le[3] = {0, 0, 1};
  int face_id = -1, edge_i = -1, edge_j = -1;
  for (int ax = 0; ax < 6; ax++) {
    const double* L = ax < 3 ? axA[ax] : axB[ax - 3];
    double ra = 0, rb = 0;
    for (int k = 0; k < 3; k++) { ra += ha[k] * fabs(dot3(axA[k], L)); rb += hb[k] * fabs(dot3(axB[k], L)); }
    double sep = fabs(dot3(t, L)) - ra - rb;
    if (sep > best_face) { best_face = sep; face_id = ax; memcpy(Lf, L, sizeof(Lf)); }
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double L[3];
      cross3(L, axA[i], axB[j]);
      double l = norm3(L);
      if (l < 1e-6) continue;
      for (int k = 0; k < 3; k++) L[k] /= l;
      double ra = 0, rb = 0;
      for (int k = 0; k < 3; k++) { ra += ha[k] * fabs(dot3(axA[k], L)); rb += hb[k] * fabs(dot3(axB[k], L)); }
      double sep = fabs(dot3(t, L)) - ra - rb;
      if (sep > best_edge) { best_edge = sep; edge_i = i; edge_j = j; memcpy(Le, L, sizeof(Le)); }
    }
  double best = best_face > best_edge ? best_face : best_edge;
  out[0].dist = best; /* separation (used only if a masked slot asks for it) */
  if (best >= margin) return;
  int use_edge = edge_i >= 0 && best_edge > 0.95 * best_face + 1e-5;
  double n[3];
  const double* L = use_edge ? Le : Lf;
  double sg = dot3(t, L) >= 0 ? 1.0 : -1.0;
  for (int k = 0; k < 3; k++) n[k] = sg * L[k]; /* from A towards B */
  if (use_edge) {
    double pa[3], pb[3], da[3], db[3];
    for (int k = 0; k < 3; k++) { pa[k] = d->geom_xpos[ga][k]; pb[k] = d->geom_xpos[gb][k]; }
    for (int k = 0; k < 3; k++) {
      if (k != edge_i) {
        double s = dot3(n, axA[k]) >= 0 ? 1.0 : -1.0;
        for (int c = 0; c < 3; c++) pa[c] += s * ha[k] * axA[k][c];
      }
      if (k != edge_j) {
        double s = dot3(n, axB[k]) >= 0 ? -1.0 : 1.0;
        for (int c = 0; c < 3; c++) pb[c] += s * hb[k] * axB[k][c];
      }
    }
    for (int c = 0; c < 3; c++) {
      pa[c] -= ha[edge_i] * axA[edge_i][c]; da[c] = 2 * ha[edge_i] * axA[edge_i][c];
      pb[c] -= hb[edge_j] * axB[edge_j][c]; db[c] = 2 * hb[edge_j] * axB[edge_j][c];
    }
    double s, u, pos[3];
    seg_seg(pa, da, pb, db, &s, &u);
    for (int c = 0; c < 3; c++) pos[c] = 0.5 * (pa[c] + s * da[c] + pb[c] + u * db[c]);
    set_contact(&out[0], best_edge, pos, n);
    return;
  }
  /* face contact: reference box owns the face axis */
  int refA = face_id < 3, fi = refA ? face_id : face_id - 3;
  const double *cr = refA ? d->geom_xpos[ga] : d->geom_xpos[gb], *ci = refA ? d->geom_xpos[gb] : d->geom_xpos[ga];
  double (*axR)[3] = refA ? axA : axB, (*axI)[3] = refA ? axB : axA;
  const double *hr = refA ? ha : hb, *hi = refA ? hb : ha;
  double nf[3];
  for (int k = 0; k < 3; k++) nf[k] = refA ? n[k] : -n[k]; /* ref face normal towards incident box */
  int ki = 0;
  double bestdot = -1;
  for (int k = 0; k < 3; k++) {
    double v = fabs(dot3(axI[k], nf));
    if (v > bestdot) { bestdot = v; ki = k; }
  }
  double si = dot3(axI[ki], nf) > 0 ? -1.0 : 1.0;
  int u = (ki + 1) % 3, v = (ki + 2) % 3;
  double poly[8][3], tmpp[8][3];
  int np = 4;
  const double su[4] = {1, -1, -1, 1}, sv[4] = {1, 1, -1, -1};
  for (int c = 0; c < 4; c++)
    for (int k = 0; k < 3; k++)
      poly[c][k] = ci[k] + si * hi[ki] * axI[ki][k] + su[c] * hi[u] * axI[u][k] + sv[c] * hi[v] * axI[v][k];
  /* clip against the 4 side planes of the reference face */
  for (int pl = 0; pl < 4 && np > 0; pl++) {
    int ax = (fi + 1 + (pl >> 1)) % 3;
    double s = (pl & 1) ? -1.0 : 1.0;
    int nn = 0;
    for (int c = 0; c < np; c++) {
      const double *P = poly[c], *Q = poly[(c + 1) % np];
      double dp = s * (dot3(P, axR[ax]) - dot3(cr, axR[ax])) - hr[ax];
      double dq = s * (dot3(Q, axR[ax]) - dot3(cr, axR[ax])) - hr[ax];
      if (dp <= 0) { memcpy(tmpp[nn++], P, 3 * sizeof(double)); }
      if ((dp < 0 && dq > 0) || (dp > 0 && dq < 0)) {
        double w = dp / (dp - dq);
        for (int k = 0; k < 3; k++) tmpp[nn][k] = P[k] + w * (Q[k] - P[k]);
        nn++;
      }
    }
    np = nn;
    memcpy(poly, tmpp, sizeof(double) * 3 * np);
  }
  double depth[8];
  int keep[8], nkeep = 0;
  for (int c = 0; c < np; c++) {
    double rel[3];
    for (int k = 0; k < 3; k++) rel[k] = poly[c][k] - cr[k];
    depth[c] = hr[fi] - dot3(rel, nf);
    if (-depth[c] < margin) keep[nkeep++] = c;
  }
  if (nkeep == 0) return;
  int pick[4], npick;
  if (nkeep <= 4) {
    for (int c = 0; c < nkeep; c++) pick[c] = keep[c];
    npick = nkeep;
  } else {
    int d0 = 0;
    for (int c = 1; c < nkeep; c++)
      if (depth[keep[c]] > depth[keep[d0]]) d0 = c;
    for (int s = 0; s < 4; s++) pick[s] = keep[(d0 + s * nkeep / 4) % nkeep];
    npick = 4;
  }
  for (int s = 0; s < npick; s++) {
    int c = pick[s];
    double pos[3];
    for (int k = 0; k < 3; k++) pos[k] = poly[c][k] + nf[k] * 0.5 * depth[c];
    set_contact(&out[s], -depth[c], pos, n);
  }
}

/* ---- general convex: support functions + Minkowski portal refinement ---- */

/* world support point of geom g along dir (any length); *hint: hull vertex the
   previous query on this geom ended at (-1: none), where the climb starts */
/* ties in the support mapping resolve the same way in fp32 and fp64: a box /
   capsule / cylinder axis with |l_k| < SUP_TIE |l| contributes its face (or
   segment) centre, 0 (MuJoCo's mju_sign(0) = 0, widened to the fp32 rounding
   of a component that is exactly zero in fp64); the hull climb moves to the
   neighbour that beats the current vertex the most (strictly: MuJoCo's), or,
   with a band > 0 (oracle_set_floor(1, b)), to the first within b metres */
#define SUP_TIE_K 1e-6
#define SUP_BAND_K 1e-5 /* the round-2 band, kept for the experiments */
/* Which rules run MuJoCo-exact: a bit mask of EXACT_* below, set
   by oracle_set_exact; the others run at the kernel's values (oracle_set_floor).
   The default is MuJoCo's Newton stop test, its line search, ccd_tolerance
   1e-6 and strict support maxima; two fp32-robust rules stay the kernel's:
   the support-axis tie above (EXACT_SUP: mju_sign) and the manifold picks
   among near-equal candidates (EXACT_PICK: exact argmax -- a resting flat
   face has exactly coplanar vertices, whose fp32 values tie by rounding).
   Global: set before a run, not while one is in flight.  DESIGN.md §Parity
   lists what each rule moves. */
static int g_exact = 1 | 2 | 4;
#define EXACT_NEWTON 1  /* Newton stop without the 1e-6 relative improvement floor */
#define EXACT_LS 2      /* line search without the 1e-6 relative bracket floor */
#define EXACT_MPR 4     /* MPR gap tolerance = ccd_tolerance 1e-6 */
#define EXACT_SUP 8     /* strict support maxima (no tie band / axis tie) */
#define EXACT_PICK 16   /* manifold / box picks by exact argmax */
void oracle_set_exact(int mask) { g_exact = mask; }
int oracle_get_exact(void) { return g_exact; }
/* the kernel's values of the rules (oracle_set_floor: experiments that size
   them against the exact mode) */
static double g_floor[4] = {1e-6 /* Newton */, 0.0 /* support band: strict climb */, SUP_TIE_K, 1e-5 /* MPR */};
void oracle_set_floor(int which, double v) { if (which >= 0 && which < 4) g_floor[which] = v; }
#define SUP_TIE ((g_exact & EXACT_SUP) ? 0.0 : g_floor[2])
#define SUP_BAND ((g_exact & EXACT_SUP) ? 0.0 : g_floor[1])
static __thread long g_tie_stats[8]; /* diagnostic: |l_k| / |l| of the support axis ties (oracle_tie_stats) */
void oracle_tie_stats(long* out, int reset) {
  if (out) memcpy(out, g_tie_stats, sizeof(g_tie_stats));
  if (reset) memset(g_tie_stats, 0, sizeof(g_tie_stats));
}
static double tie_sign(double lk, double ln) {
  if (fabs(lk) < 1e-6 * ln) {
    const double r = fabs(lk) / (ln > 0 ? ln : 1);
    g_tie_stats[r == 0 ? 0 : r < 1e-15 ? 1 : r < 1e-12 ? 2 : r < 1e-9 ? 3 : 4]++;
  }
  /* exact: MuJoCo's mju_sign (0 for an exactly zero component, as
     mjccd_support's box / capsule / cylinder cases) */
  if ((g_exact & EXACT_SUP) || g_floor[2] < 0) return lk > 0 ? 1.0 : (lk < 0 ? -1.0 : 0.0);
  return fabs(lk) < g_floor[2] * ln ? 0.0 : (lk >= 0 ? 1.0 : -1.0);
}

/* cube-map cell of a local direction l (the start table's order): major
   axis (lowest on ties), its sign, then the other two components (cyclic
   order) over |l_axis| in R bins; the kernel's lut_cell in fp32 */
#define ORACLE_LUT_R 128 /* any resolution gives the same supports (the tie walk); the kernel's is MPCR_LUT_R */
static int lut_cell(const double l[3]) {
  const double a0 = fabs(l[0]), a1 = fabs(l[1]), a2 = fabs(l[2]);
  const int ax = (a0 >= a1 && a0 >= a2) ? 0 : (a1 >= a2 ? 1 : 2);
  const double la = fabs(l[ax]);
  if (!(la > 0)) return 0;
  const int R = ORACLE_LUT_R;
  int iu = (int)floor((l[(ax + 1) % 3] / la + 1.0) * 0.5 * R), iv = (int)floor((l[(ax + 2) % 3] / la + 1.0) * 0.5 * R);
  iu = iu < 0 ? 0 : (iu > R - 1 ? R - 1 : iu);
  iv = iv < 0 ? 0 : (iv > R - 1 ? R - 1 : iv);
  return (2 * ax + (l[ax] < 0)) * R * R + iu * R + iv;
}

/* Support start tables.  The model blob carries none since v9 (the engine
   builds its own, engine.hip hull_start_table); the oracle builds one per
   model on first use, by the same definition -- per hull and cube-map cell
   the vertex extreme along the cell centre, cells in scan order, each
   climbing (strict ascent) from the previous cell's vertex, then the lowest
   index among the exactly tied maxima along tied edges -- and keeps it for
   the process (at most ORACLE_LUT_CACHE models; past that, climbs start at
   the hull's first vertex: slower, the same supports).  Every entry point
   names its model once (use_model), so the queries read the table through
   thread-locals.  oracle_set_start_scramble(seed != 0): hashed vertices
   instead (tests/test_hull_ties.py). */
#define ORACLE_LUT_CACHE 32
typedef struct { uint64_t key; int32_t adr[MPCR_MAX_GEOM]; int32_t* cells; } lut_entry;
static lut_entry g_lut[ORACLE_LUT_CACHE];
static int g_nlut;
static pthread_mutex_t g_lut_mu = PTHREAD_MUTEX_INITIALIZER;
static uint64_t g_scramble;
static __thread const int32_t* t_lutadr;
static __thread const int32_t* t_cells;
void oracle_set_start_scramble(unsigned long long seed) { g_scramble = seed; }

static uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27; x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
static uint64_t hash_words(uint64_t h, const void* p, size_t nbytes) {
  const unsigned char* b = (const unsigned char*)p;
  for (size_t i = 0; i + 8 <= nbytes; i += 8) {
    uint64_t w;
    memcpy(&w, b + i, 8);
    h = mix64(h ^ w);
  }
  for (size_t i = nbytes & ~(size_t)7; i < nbytes; i++) h = mix64(h ^ b[i]);
  return h;
}

static void build_starts(const mpcr_model_t* m, lut_entry* e, uint64_t scramble) {
  const int R = ORACLE_LUT_R, nc = 6 * R * R;
  int n = 0;
  for (int g = 0; g < m->ngeom; g++) {
    e->adr[g] = (m->geom_hulladr[g] >= 0 && m->geom_hullnum[g] > 0) ? n : -1;
    if (e->adr[g] >= 0) n += nc;
  }
  e->cells = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
  if (!e->cells) return;
  int tied[256];
  for (int g = 0; g < m->ngeom; g++) {
    if (e->adr[g] < 0) continue;
    const int a = m->geom_hulladr[g], na = m->geom_hullnum[g];
    int32_t* out = e->cells + e->adr[g];
    int v = a;
    for (int c = 0; c < nc; c++) {
      if (scramble) { out[c] = a + (int)(mix64(scramble ^ ((uint64_t)g << 40) ^ (uint64_t)c) % (uint64_t)na); continue; }
      const int f = c / (R * R), iu = (c / R) % R, iv = c % R, ax = f / 2;
      double dd[3];
      dd[ax] = (f & 1) ? -1.0 : 1.0;
      dd[(ax + 1) % 3] = -1.0 + (2.0 * iu + 1.0) / R;
      dd[(ax + 2) % 3] = -1.0 + (2.0 * iv + 1.0) / R;
      double best = dot3(m->hull_vert[v], dd);
      for (;;) {
        int nb = v;
        for (int k = m->hull_adjadr[v]; k < m->hull_adjadr[v] + m->hull_adjnum[v]; k++) {
          const int u = m->hull_adj[k];
          const double du = dot3(m->hull_vert[u], dd);
          if (du > best) { best = du; nb = u; }
        }
        if (nb == v) break;
        v = nb;
      }
      int nt = 1, lo = v;
      tied[0] = v;
      for (int i = 0; i < nt && nt < 256; i++)
        for (int k = m->hull_adjadr[tied[i]]; k < m->hull_adjadr[tied[i]] + m->hull_adjnum[tied[i]] && nt < 256; k++) {
          const int u = m->hull_adj[k];
          if (!(dot3(m->hull_vert[u], dd) == best)) continue;
          int seen = 0;
          for (int j = 0; j < nt; j++) seen |= tied[j] == u;
          if (!seen) { tied[nt++] = u; if (u < lo) lo = u; }
        }
      out[c] = lo;
    }
  }
}

static void use_model(const mpcr_model_t* m) {
  t_lutadr = t_cells = NULL;
  if (m->nhullv <= 0) return;
  const uint64_t scramble = g_scramble;
  uint64_t h = mix64(0x6d70637273746172ull ^ scramble ^ ((uint64_t)m->ngeom << 32) ^ (uint64_t)m->nhullv);
  h = hash_words(h, m->geom_hulladr, sizeof(int32_t) * m->ngeom);
  h = hash_words(h, m->geom_hullnum, sizeof(int32_t) * m->ngeom);
  h = hash_words(h, m->hull_vert, sizeof(m->hull_vert[0]) * m->nhullv);
  h = hash_words(h, m->hull_adjadr, sizeof(int32_t) * m->nhullv);
  h = hash_words(h, m->hull_adj, sizeof(int32_t) * m->nhulla);
  pthread_mutex_lock(&g_lut_mu);
  lut_entry* e = NULL;
  for (int i = 0; i < g_nlut && !e; i++)
    if (g_lut[i].key == h) e = &g_lut[i];
  if (!e && g_nlut < ORACLE_LUT_CACHE) {
    e = &g_lut[g_nlut];
    build_starts(m, e, scramble);
    if (e->cells) { e->key = h; g_nlut++; } else e = NULL;
  }
  pthread_mutex_unlock(&g_lut_mu);
  if (e) { t_lutadr = e->adr; t_cells = e->cells; }
}

/* MPR work counters of the calling thread (diagnostic: tools/mpr_stats.py, workers = 1):
   0 calls, 1 support pairs, 2 climb rounds, 3 neighbour evaluations, 4 hits,
   polyhedron manifold: 5 clips that keep no point (the support-vertex contact), 8 calls, 9 candidate faces, 10 faces scanned for the
   cone, 11 calls reaching the clip, 12 reference-polygon vertices, 13
   incident-polygon vertices, 14 climb rounds, 15 support-vertex faces,
   16.. histogram of support pairs per call (capped at 47) */
static __thread long g_mpr_stats[64]; /* per thread: the checker's pool threads never share it */
/* Hull support ties (round 6).  The climb ends at a vertex no neighbour
   beats; when the direction is (within HULL_TIE metres) normal to an edge or
   a face of the hull, every vertex of it is a maximum and which one the
   climb reaches depends on where it started (the start table's cell, the
   pair's hint) and on the last bits of the dot products (fp32 and fp64 pick
   differently).  So the climb's last round also names the end v's
   lowest-index neighbour within HULL_TIE of v's value, and the support walks
   on to it while it is lower than the current vertex (the threshold fixed at
   the climb end's value): an edge's lower end, a triangle's lowest vertex,
   a polygon's lowest vertex unless the descent along its tied neighbours
   stops at a local minimum -- from whichever tied vertex the climb reached
   (tests/test_hull_ties.py), as an
   argmax over all vertices that takes the first of equal values (MJX's
   jnp.argmax support of a mesh) -- a support start table's resolution is a
   performance choice, not a parity change (VERDICT r5 item 1;
   tools/tie_start_independence.py).  HULL_TIE = 1e-7 m is ~1e-6 of the
   gripper hulls' extent (the box / capsule / cylinder axis tie's relative
   scale, tie_sign) and ~10x the fp32 rounding of a vertex projection; the
   kernel's sup_finish / tie_round do the same in fp32.  Queries whose caller
   uses the support value only (the SAT's separations, support_value) skip
   the walk: every tied vertex gives that value to within HULL_TIE.  Exact
   mode (EXACT_SUP): no tie rule. */
static double g_hull_tie = 1e-7;
static int g_hint_ge = 1; /* the hint on equal values (the kernel's start rule; 0: the table's) */
static __thread int g_from_hint;
static __thread long g_walk_kind[4]; /* walks by (start: table 0 / hint 1) + (climb moved 0 / stayed 2) */
void oracle_walk_kind(long* out, int reset) {
  if (out) memcpy(out, g_walk_kind, sizeof(g_walk_kind));
  if (reset) memset(g_walk_kind, 0, sizeof(g_walk_kind));
}
void oracle_set_hint_ge(int v) { g_hint_ge = v; }
void oracle_set_hull_tie(double v) { g_hull_tie = v; } /* experiments: 0 = the plain climb's end */
#define HULL_TIE ((g_exact & EXACT_SUP) ? 0.0 : g_hull_tie)
static __thread int g_value_only; /* support_value's queries: no tie walk */
static __thread int g_sup_kind; /* diagnostic: 0 MPR, 1 support vertex, 2 support value (SAT), 3 plane */
static __thread long g_tie_kind[4][2];
void oracle_tie_kind(long* out, int reset) {
  if (out) memcpy(out, g_tie_kind, sizeof(g_tie_kind));
  if (reset) memset(g_tie_kind, 0, sizeof(g_tie_kind));
}
/* the lowest-index neighbour of v whose value reaches lo (-1: none) */
static int tied_neighbour(const mpcr_model_t* m, int v, double lo, const double lu[3]) {
  int t = -1;
  for (int k = m->hull_adjadr[v]; k < m->hull_adjadr[v] + m->hull_adjnum[v]; k++) {
    const int u = m->hull_adj[k];
    if ((t < 0 || u < t) && dot3(m->hull_vert[u], lu) >= lo) t = u;
  }
  return t;
}
static __thread long g_walk_stats[4]; /* diagnostic: walks, jumps, walks past the first jump */
void oracle_walk_stats(long* out, int reset) {
  if (out) memcpy(out, g_walk_stats, sizeof(g_walk_stats));
  if (reset) memset(g_walk_stats, 0, sizeof(g_walk_stats));
}
static int hull_tie(const mpcr_model_t* m, int v, int t, double lo, const double lu[3]) {
  const int v0 = v;
  g_mpr_stats[6]++;
  g_walk_stats[0]++;
  for (int guard = 0; guard < 64 && t >= 0 && t < v; guard++) {
    v = t;
    t = tied_neighbour(m, v, lo, lu);
    g_walk_stats[1]++;
    if (guard == 0 && t >= 0 && t < v) g_walk_stats[2]++;

  }
  g_mpr_stats[7] += v != v0;
  g_tie_kind[g_sup_kind & 3][0]++;
  g_tie_kind[g_sup_kind & 3][1] += v != v0;
  return v;
}

/* world support point of geom g along dir (any length); *hint: hull vertex the
   previous query on this geom ended at (-1: none), where the climb starts */
static void support_rel(const mpcr_model_t* m, const odata* d, int g, const double dir[3], double out[3], int* hint,
                        const double* org);
static void support(const mpcr_model_t* m, const odata* d, int g, const double dir[3], double out[3], int* hint) {
  support_rel(m, d, g, dir, out, hint, NULL);
}
/* org (nullable): the support point relative to org, (geom centre - org)
   formed first (MPR works relative to the second geom's centre, as the kernel) */
static void support_rel(const mpcr_model_t* m, const odata* d, int g, const double dir[3], double out[3], int* hint,
                        const double* org) {
  const double* R = d->geom_xmat[g];
  const double* sz = m->geom_size[g];
  double l[3], p[3] = {0, 0, 0};
  mulmtv(l, R, dir);
  const double ln = norm3(l);
  switch (m->geom_type[g]) {
    case MPCR_GEOM_SPHERE: {
      if (ln > 0) for (int k = 0; k < 3; k++) p[k] = sz[0] * l[k] / ln;
      break;
    }
    case MPCR_GEOM_CAPSULE: {
      if (ln > 0) for (int k = 0; k < 3; k++) p[k] = sz[0] * l[k] / ln;
      p[2] += tie_sign(l[2], ln) * sz[1];
      break;
    }
    case MPCR_GEOM_CYLINDER: {
      double r = sqrt(l[0] * l[0] + l[1] * l[1]);
      if (r > fmax(SUP_TIE, 0.0) * ln) { p[0] = sz[0] * l[0] / r; p[1] = sz[0] * l[1] / r; }
      p[2] = tie_sign(l[2], ln) * sz[1];
      break;
    }
    case MPCR_GEOM_BOX:
      for (int k = 0; k < 3; k++) p[k] = tie_sign(l[k], ln) * sz[k];
      break;
    case MPCR_GEOM_MESH: { /* steepest-ascent hill climbing on the hull graph */
      double lu[3] = {0, 0, 0};
      if (ln > 0) for (int k = 0; k < 3; k++) lu[k] = l[k] / ln;
      /* start: the table vertex of l's cube-map cell, or the hint (where the
         previous query on this pair ended) when it reaches that by the band
         -- on equal values the hint, as the kernel (after a tie walk the hint
         is the tie's lowest index) */
      int v = t_cells && t_lutadr[g] >= 0 ? t_cells[t_lutadr[g] + lut_cell(l)] : m->geom_hulladr[g];
      double best = dot3(m->hull_vert[v], lu);
      if (*hint >= 0) {
        const double bh = dot3(m->hull_vert[*hint], lu);
        if (g_hint_ge == 2 ? bh >= best - HULL_TIE : (g_hint_ge ? bh >= best + SUP_BAND : bh > best + SUP_BAND)) {
          v = *hint; best = bh; g_from_hint = 1;
        }
      }
      const int v_start = v;
      int tmin = -1, tcnt = 0; /* the last round's lowest-index neighbour within HULL_TIE of v, their count */
      for (;;) {
        int nb = v;
        g_mpr_stats[2]++;
        g_mpr_stats[3] += m->hull_adjnum[v];
        double bn = best + SUP_BAND; /* a neighbour must beat this; ties within the band go to the first */
        tmin = -1;
        tcnt = 0;
        for (int k = m->hull_adjadr[v]; k < m->hull_adjadr[v] + m->hull_adjnum[v]; k++) {
          int u = m->hull_adj[k];
          double du = dot3(m->hull_vert[u], lu);
          if (du >= best - HULL_TIE) tcnt++;
          if (du >= best - HULL_TIE && (tmin < 0 || u < tmin)) tmin = u;
          if (du > bn) { bn = du + SUP_BAND; nb = u; }
        }
        if (nb == v) break;
        best = bn - SUP_BAND;
        v = nb;
      }
      if (HULL_TIE > 0 && !g_value_only && tmin >= 0 && tmin < v) {
        g_walk_kind[(g_from_hint ? 1 : 0) + (v == v_start ? 2 : 0)]++;
        g_walk_stats[3] += tcnt == 1;
        v = hull_tie(m, v, tmin, best - HULL_TIE, lu);
      }
      g_from_hint = 0;
      memcpy(p, m->hull_vert[v], sizeof(p));
      *hint = v;
      break;
    }
    default: break;
  }
  mulmv(out, R, p);
  for (int k = 0; k < 3; k++) out[k] += org ? d->geom_xpos[g][k] - org[k] : d->geom_xpos[g][k];
}

typedef struct { double v[3], a[3], b[3]; } mpt; /* v = a - b */

/* MPR's gap tolerance: 1e-5 m, not MuJoCo's ccd_tolerance 1e-6.  The
   refinement stops when a new support point gains less than tol over the
   portal; near the end the portal faces of two mesh hulls differ in normal by
   0.01-0.05 rad, so the answer hinges on which side of tol the last gap
   lands.  fp32 computes those gaps to ~3e-8 m (1e-7 on metre-sized boxes):
   at 1e-6 that decided a visible share of the dual arm's rollouts
   differently in the kernel and here, at 1e-5 it rarely does; the depth it
   leaves is within 1e-5 m of converged (both sides use the same value) */
#define MPR_TOL ((g_exact & EXACT_MPR) ? 1e-6 : g_floor[3]) /* MuJoCo's ccd_tolerance in the exact mode */
#define MPR_ITER 50
/* zero tests in metres (the kernel's kMprEps): lengths below 1.2e-7 m, two
   vectors parallel when one passes within it of the other's line, a point on
   a plane within it -- libccd tests lengths, areas and volumes against
   DBL_EPSILON alike, which cannot carry over to the fp32 kernel */
#define MPR_EPS 1.1920929e-07
static int iszero(double x) { return fabs(x) < MPR_EPS; }
static int off_plane(double x, const double c[3]) { return fabs(x) >= MPR_EPS * sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]); }

void oracle_mpr_stats(long* out, int reset) {
  if (out) memcpy(out, g_mpr_stats, sizeof(g_mpr_stats));
  if (reset) memset(g_mpr_stats, 0, sizeof(g_mpr_stats));
}
static void msupport(const mpcr_model_t* m, const odata* d, int g1, int g2, const double dir[3], mpt* o, int hint[2]) {
  g_mpr_stats[1]++;
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  support_rel(m, d, g1, dir, o->a, &hint[0], d->geom_xpos[g2]);
  support_rel(m, d, g2, nd, o->b, &hint[1], d->geom_xpos[g2]);
  for (int k = 0; k < 3; k++) o->v[k] = o->a[k] - o->b[k];
}
static void normalize3(double v[3]) {
  double n = norm3(v);
  if (n > 0) for (int k = 0; k < 3; k++) v[k] /= n;
}
static void portal_dir(const mpt p[4], double dir[3]) {
  double a[3], b[3];
  for (int k = 0; k < 3; k++) { a[k] = p[2].v[k] - p[1].v[k]; b[k] = p[3].v[k] - p[1].v[k]; }
  cross3(dir, a, b);
  normalize3(dir);
}
static int reach_tol(const mpt p[4], const mpt* v4, const double dir[3], double tol) {
  double d4 = dot3(v4->v, dir);
  double t = fmin(d4 - dot3(p[1].v, dir), fmin(d4 - dot3(p[2].v, dir), d4 - dot3(p[3].v, dir)));
  return t < tol;
}
static void expand(mpt p[4], const mpt* v4) {
  double x[3];
  cross3(x, v4->v, p[0].v);
  if (dot3(p[1].v, x) > 0) {
    if (dot3(p[2].v, x) > 0) p[1] = *v4; else p[3] = *v4;
  } else {
    if (dot3(p[3].v, x) > 0) p[2] = *v4; else p[1] = *v4;
  }
}
/* closest point of triangle (a, b, c) to the origin (Ericson 5.1.5) */
static void tri_closest(const double a[3], const double b[3], const double c[3], double out[3]) {
  double ab[3], ac[3], ap[3], bp[3], cp[3];
  for (int k = 0; k < 3; k++) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; ap[k] = -a[k]; bp[k] = -b[k]; cp[k] = -c[k]; }
  double d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) { memcpy(out, a, 3 * sizeof(double)); return; }
  double d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { memcpy(out, b, 3 * sizeof(double)); return; }
  double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    double t = d1 / (d1 - d3);
    for (int k = 0; k < 3; k++) out[k] = a[k] + t * ab[k];
    return;
  }
  double d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) { memcpy(out, c, 3 * sizeof(double)); return; }
  double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    double t = d2 / (d2 - d6);
    for (int k = 0; k < 3; k++) out[k] = a[k] + t * ac[k];
    return;
  }
  double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    double t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int k = 0; k < 3; k++) out[k] = b[k] + t * (c[k] - b[k]);
    return;
  }
  /* face region: the plane projection n (n.a) / |n|^2 -- Ericson's
     barycentric a + v ab + w ac loses the answer to cancellation in fp32
     when the triangle is large against its distance from the origin (MPR's
     final portal: cm-sized around a sub-mm penetration); the kernel does the same */
  double n[3];
  cross3(n, ab, ac);
  double s = dot3(n, a) / dot3(n, n);
  for (int k = 0; k < 3; k++) out[k] = n[k] * s;
  (void)va; (void)vb; (void)vc;
}

/* MPR penetration of geoms g1, g2: 1 and (depth, dir from g1 to g2, pos) if
   they overlap, else 0 */
static int mpr_impl(const mpcr_model_t* m, const odata* d, int g1, int g2, double* depth, double dir[3],
                    double pos[3], int* hint);
static int mpr(const mpcr_model_t* m, const odata* d, int g1, int g2, double* depth, double dir[3], double pos[3],
               int* hint) {
  const long s0 = g_mpr_stats[1];
  const int hit = mpr_impl(m, d, g1, g2, depth, dir, pos, hint);
  const long k = g_mpr_stats[1] - s0;
  g_mpr_stats[0]++;
  g_mpr_stats[4] += hit;
  g_mpr_stats[16 + (k < 0 ? 0 : (k < 47 ? k : 47))]++;
  return hit;
}
static int mpr_impl(const mpcr_model_t* m, const odata* d, int g1, int g2, double* depth, double dir[3],
                    double pos[3], int* hint) {
  const double tol = MPR_TOL;
  mpt p[4], v4;
  double va[3], vb[3], dd;
  /* phase 1: portal discovery; v0 = interior point of the difference */
  for (int k = 0; k < 3; k++) {
    p[0].a[k] = d->geom_xpos[g1][k] - d->geom_xpos[g2][k]; /* frame origin: g2's centre */
    p[0].b[k] = 0;
    p[0].v[k] = p[0].a[k];
  }
  if (iszero(p[0].v[0]) && iszero(p[0].v[1]) && iszero(p[0].v[2])) p[0].v[0] += 10 * MPR_EPS;
  for (int k = 0; k < 3; k++) dir[k] = -p[0].v[k];
  normalize3(dir);
  msupport(m, d, g1, g2, dir, &p[1], hint);
  dd = dot3(p[1].v, dir);
  if (iszero(dd) || dd < 0) return 0;
  cross3(dir, p[0].v, p[1].v);
  double thr = MPR_EPS * (norm3(p[0].v) + norm3(p[1].v));
  if (dot3(dir, dir) < thr * thr) { /* v1 on the ray from v0 through the origin */
    for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p[1].a[k] + p[1].b[k]) + d->geom_xpos[g2][k];
    if (iszero(p[1].v[0]) && iszero(p[1].v[1]) && iszero(p[1].v[2])) { /* touching at v1 */
      *depth = 0;
      dir[0] = dir[1] = dir[2] = 0;
    } else { /* origin on the v0-v1 segment */
      memcpy(dir, p[1].v, sizeof(double) * 3);
      *depth = norm3(dir);
      normalize3(dir);
    }
    return 1;
  }
  normalize3(dir);
  msupport(m, d, g1, g2, dir, &p[2], hint);
  dd = dot3(p[2].v, dir);
  if (iszero(dd) || dd < 0) return 0;
  for (int k = 0; k < 3; k++) { va[k] = p[1].v[k] - p[0].v[k]; vb[k] = p[2].v[k] - p[0].v[k]; }
  cross3(dir, va, vb);
  normalize3(dir);
  if (dot3(dir, p[0].v) > 0) {
    mpt t = p[1]; p[1] = p[2]; p[2] = t;
    for (int k = 0; k < 3; k++) dir[k] = -dir[k];
  }
  for (int guard = 0;; guard++) {
    if (guard > MPR_ITER) return 0;
    msupport(m, d, g1, g2, dir, &p[3], hint);
    dd = dot3(p[3].v, dir);
    if (iszero(dd) || dd < 0) return 0;
    int cont = 0;
    cross3(va, p[1].v, p[3].v);
    dd = dot3(va, p[0].v);
    if (dd < 0 && off_plane(dd, va)) { p[2] = p[3]; cont = 1; }
    if (!cont) {
      cross3(va, p[3].v, p[2].v);
      dd = dot3(va, p[0].v);
      if (dd < 0 && off_plane(dd, va)) { p[1] = p[3]; cont = 1; }
    }
    if (!cont) break;
    for (int k = 0; k < 3; k++) { va[k] = p[1].v[k] - p[0].v[k]; vb[k] = p[2].v[k] - p[0].v[k]; }
    cross3(dir, va, vb);
    normalize3(dir);
  }
  /* phase 2: refine until the portal encloses the origin */
  for (int it = 0;; it++) {
    portal_dir(p, dir);
    dd = dot3(dir, p[1].v);
    if (iszero(dd) || dd > 0) break;
    msupport(m, d, g1, g2, dir, &v4, hint);
    dd = dot3(v4.v, dir);
    if (!(iszero(dd) || dd > 0) || reach_tol(p, &v4, dir, tol) || it > MPR_ITER) return 0;
    expand(p, &v4);
  }
  /* phase 3: penetration depth / direction / position */
  for (int it = 0;; it++) {
    portal_dir(p, dir);
    msupport(m, d, g1, g2, dir, &v4, hint);
    if (reach_tol(p, &v4, dir, tol) || it > MPR_ITER) {
      double w[3];
      tri_closest(p[1].v, p[2].v, p[3].v, w);
      *depth = norm3(w);
      if (iszero(*depth)) dir[0] = dir[1] = dir[2] = 0;
      else for (int k = 0; k < 3; k++) dir[k] = w[k] / *depth;
      /* barycentric position of the origin in the tetrahedron (libccd findPos) */
      double pd[3], b[4], x[3], e1[3], e2[3];
      for (int k = 0; k < 3; k++) { e1[k] = p[2].v[k] - p[1].v[k]; e2[k] = p[3].v[k] - p[1].v[k]; }
      cross3(pd, e1, e2); /* portal normal, |pd| = twice the portal's area */
      cross3(x, p[2].v, p[3].v); b[0] = dot3(x, p[1].v);
      cross3(x, p[3].v, p[2].v); b[1] = dot3(x, p[0].v);
      cross3(x, p[0].v, p[1].v); b[2] = dot3(x, p[3].v);
      cross3(x, p[2].v, p[1].v); b[3] = dot3(x, p[0].v);
      double sum = b[0] + b[1] + b[2] + b[3];
      /* sum = 6 x the tetrahedron's volume: degenerate when v0 lies on the portal's plane */
      if (!off_plane(sum, pd) || sum < 0) {
        normalize3(pd);
        b[0] = 0;
        cross3(x, p[2].v, p[3].v); b[1] = dot3(x, pd);
        cross3(x, p[3].v, p[1].v); b[2] = dot3(x, pd);
        cross3(x, p[1].v, p[2].v); b[3] = dot3(x, pd);
        sum = b[1] + b[2] + b[3];
      }
      for (int k = 0; k < 3; k++) {
        double pa = 0, pb = 0;
        for (int i = 0; i < 4; i++) { pa += b[i] * p[i].a[k]; pb += b[i] * p[i].b[k]; }
        pos[k] = 0.5 * (pa + pb) / sum + d->geom_xpos[g2][k];
      }
      return 1;
    }
    expand(p, &v4);
  }
}

static int poly_manifold(const mpcr_model_t* m, odata* d, int pair, int g1, int g2, const double n[3], double depth,
                         ocontact* out);
static int caps_poly(const mpcr_model_t* m, odata* d, int g1, int g2, double depth, ocontact* out);
/* Experiment (ORACLE_CAPS_SAT=1 in the environment; not in the kernel, off by
   default): a capsule or cylinder penetrating a polyhedron deeper than
   POLY_DEEP takes the polyhedron's face axis of least penetration (MJX's
   capsule_convex SAT over face normals) instead of MPR's portal normal --
   tools/diag_f32.py measures what it does to the fp32 restatement's misses */
static int caps_sat_on(void) {
  static int v = -1;
  if (v < 0) { const char* e = getenv("ORACLE_CAPS_SAT"); v = e ? atoi(e) : 0; }
  return v;
}
static void col_convex(const mpcr_model_t* m, odata* d, int pair, int g1, int g2, ocontact* out) {
  double depth, n[3], pos[3];
  if (!mpr(m, d, g1, g2, &depth, n, pos, d->hint[pair])) return;
  if (n[0] == 0 && n[1] == 0 && n[2] == 0) n[2] = 1; /* touching: any frame */
  if (caps_sat_on() && depth > 5e-3 && caps_poly(m, d, g1, g2, depth, out)) return;
  /* polyhedron pairs: the face-clipping manifold when a face axis carries
     the contact, else MPR's single point */
  if (m->pair_ncon[pair] == 4 && depth > 0 && poly_manifold(m, d, pair, g1, g2, n, depth, out)) return;
  set_contact(out, -depth, pos, n);
}

/* argmax with a relative tie band, independent of scan order: the lowest
   index whose value lies within 1e-4 of the maximum's magnitude (+1e-12), so
   near-ties (symmetric hulls, fp32 vs fp64 rounding) resolve to the lowest
   vertex index in the oracle and the kernel alike (the kernel evaluates it as
   a wave max and a ballot over 64 vertices at a time) */
static int beats(double v, double best) { return v > best + ((g_exact & EXACT_PICK) ? 0.0 : 1e-4 * fabs(best) + 1e-12); }
static int near_max(double v, double mx) { return v >= mx - ((g_exact & EXACT_PICK) ? 0.0 : 1e-4 * fabs(mx) + 1e-12); }

/* plane - mesh: MJX's plane_convex manifold (mujoco-mjx 3.3.1,
   mjx/_src/collision_convex.py plane_convex + _manifold_points; MJX is the
   reference's rollout engine, SBP/mjx_planner.py:108,256).  Hull vertices
   that penetrate the plane and lie within 1 mm of the deepest one form the
   candidate set; of those: a = the first, b = the farthest from a, c = the
   farthest from the line ab (in the plane), d = the farthest from the edges
   bc / ac ("farthest": near_max's lowest index within the tie band).  Repeated picks are inactive (dist 1 in MJX, 1e30 here); every
   contact carries the plane normal and sits half-way through the
   penetration.  No penetrating vertex: slot 0 reports the deepest vertex's
   (non-negative) distance, slots 1-3 stay empty -- the restatement for
   margin 0 (the only margin the reference scenes use) */
static void col_plane_mesh(const mpcr_model_t* m, odata* d, int pair, int gp, int g, ocontact* out) {
  const double* R = d->geom_xmat[g];
  const double* Rp = d->geom_xmat[gp];
  double n[3] = {Rp[2], Rp[5], Rp[8]}, nn[3] = {-Rp[2], -Rp[5], -Rp[8]}, q[3], pos[3];
  g_sup_kind = 3;
  support(m, d, g, nn, q, &d->hint[pair][1]);
  g_sup_kind = 0;
  double dist0 = (q[0] - d->geom_xpos[gp][0]) * n[0] + (q[1] - d->geom_xpos[gp][1]) * n[1] +
                 (q[2] - d->geom_xpos[gp][2]) * n[2];
  if (dist0 >= 0) {
    for (int k = 0; k < 3; k++) pos[k] = q[k] - 0.5 * dist0 * n[k];
    set_contact(out, dist0, pos, n);
    return;
  }
  /* convex frame: nl = R^T n, plane point pl = R^T (x_plane - x_geom) */
  double nl[3], dx[3], pl[3];
  mulmtv(nl, R, n);
  for (int k = 0; k < 3; k++) dx[k] = d->geom_xpos[gp][k] - d->geom_xpos[g][k];
  mulmtv(pl, R, dx);
  const int v0 = m->geom_hulladr[g], nvh = m->geom_hullnum[g];
  const double thr = fmax(0.0, -dist0 - 1e-3);
#define SUP(i) ((pl[0] - m->hull_vert[i][0]) * nl[0] + (pl[1] - m->hull_vert[i][1]) * nl[1] + \
                (pl[2] - m->hull_vert[i][2]) * nl[2])
  int ia = -1, ilast = -1;
  for (int i = v0; i < v0 + nvh; i++)
    if (SUP(i) > thr) {
      if (ia < 0) ia = i;
      ilast = i;
    }
  if (ia < 0) { /* the climb's vertex is the only one (thr rounding) */
    for (int k = 0; k < 3; k++) pos[k] = q[k] - 0.5 * dist0 * n[k];
    set_contact(out, dist0, pos, n);
    return;
  }
  const double* a = m->hull_vert[ia];
  int ib = ia, ic = ia, id = ia;
  /* each pick: the maximum over the candidate set, then its first index
     within the tie band (near_max) */
#define PICK(EXPR, OUT)                                                  \
  do {                                                                   \
    double mx_ = -1;                                                     \
    for (int i = ia; i <= ilast; i++) {                                  \
      if (!(SUP(i) > thr)) continue;                                     \
      const double* v = m->hull_vert[i];                                 \
      const double e = (EXPR);                                           \
      if (e > mx_) mx_ = e;                                              \
    }                                                                    \
    for (int i = ia; i <= ilast; i++) {                                  \
      if (!(SUP(i) > thr)) continue;                                     \
      const double* v = m->hull_vert[i];                                 \
      if (near_max((EXPR), mx_)) { OUT = i; break; }                     \
    }                                                                    \
    best_ = mx_;                                                         \
  } while (0)
  double best_;
  PICK((a[0] - v[0]) * (a[0] - v[0]) + (a[1] - v[1]) * (a[1] - v[1]) + (a[2] - v[2]) * (a[2] - v[2]), ib);
  const double* b = m->hull_vert[ib];
  double amb[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]}, ab[3];
  cross3(ab, nl, amb);
  PICK(fabs((a[0] - v[0]) * ab[0] + (a[1] - v[1]) * ab[1] + (a[2] - v[2]) * ab[2]), ic);
  const double* c = m->hull_vert[ic];
  double amc[3] = {a[0] - c[0], a[1] - c[1], a[2] - c[2]}, bmc[3] = {b[0] - c[0], b[1] - c[1], b[2] - c[2]};
  double ac[3], bc[3];
  cross3(ac, nl, amc);
  cross3(bc, nl, bmc);
  /* MJX takes the argmax of concat(dist_bp, dist_ap): the bc edge wins ties */
  int ibp = ia, iap = ia;
  PICK(fabs((b[0] - v[0]) * bc[0] + (b[1] - v[1]) * bc[1] + (b[2] - v[2]) * bc[2]), ibp);
  const double bbp = best_;
  PICK(fabs((a[0] - v[0]) * ac[0] + (a[1] - v[1]) * ac[1] + (a[2] - v[2]) * ac[2]), iap);
  const double bap = best_;
#undef PICK
  id = beats(bap, bbp) ? iap : ibp;
  const int idx[4] = {ia, ib, ic, id};
  for (int s = 0; s < 4; s++) {
    int dup = 0;
    for (int t = 0; t < s; t++) dup |= idx[t] == idx[s];
    if (dup) continue;
    double w[3], dist = -SUP(idx[s]);
    mulmv(w, R, m->hull_vert[idx[s]]);
    for (int k = 0; k < 3; k++) pos[k] = w[k] + d->geom_xpos[g][k] - 0.5 * dist * n[k];
    set_contact(&out[s], dist, pos, n);
  }
#undef SUP
}

/* ---- polyhedron pairs (mesh-mesh, box-mesh): face-clipping manifold ------
   Restates mujoco-mjx 3.3.1 collision_convex.py convex_convex (MJX is the
   reference's rollout engine, SBP/mjx_planner.py:108,256): the separating
   axis of least penetration among face normals picks a reference face, the
   other geom's most anti-parallel face is clipped by the reference face's
   side planes, the clipped points below the reference plane are the
   contacts (normal = the reference face's, position half-way through the
   penetration), at most 4 of them by _manifold_points' picks.  Where MJX
   scans every face (and edge pair) of both hulls, the axis search here is
   seeded by MPR's normal n (g1 -> g2): the candidate axes are the faces on
   the support vertex of g1 along n and of g2 along -n (MPR's direction
   lies in those vertices' normal cones) and every face whose normal lies
   within ~20 degrees of n (resp. -n).  An edge contact -- no candidate
   face within 5 % of MPR's depth -- keeps MPR's single point.  Parity vs
   MJX unpinned (DESIGN.md §Dual-arm class). */

#define POLY_CONE_COS 0.94 /* ~20 degrees: the candidate faces' Gauss-map cone about MPR's normal */
/* a penetration deeper than POLY_DEEP between hulls of at most POLY_ALLF
   faces together scans every face (MJX's SAT): MPR's normal that seeds the
   cone is, that deep, the portal face it ended on -- fp32 and fp64 took
   portals 70 degrees apart on the Hand-E's interpenetrating finger pads and
   so different candidate lists (round 4) */
#define POLY_DEEP 5e-3
#define POLY_ALLF 512

/* world outward normal and offset (n . (x - c) = off) of face f of geom g,
   relative to the point c (the manifold works relative to g2's centre, as
   MPR and the kernel do: world coordinates would carry ~1e-7 m of fp32
   rounding into every separation, relative ones ~ulp(5 cm)) */
static void face_world(const mpcr_model_t* m, const odata* d, int g, int f, double nw[3], double* off,
                       const double* c) {
  const double* R = d->geom_xmat[g];
  mulmv(nw, R, m->face_plane[f]);
  const double dx[3] = {d->geom_xpos[g][0] - c[0], d->geom_xpos[g][1] - c[1], d->geom_xpos[g][2] - c[2]};
  *off = m->face_plane[f][3] + dot3(nw, dx);
}

/* hull vertex index of geom g's support point along dir (world): the mesh
   climb from *hint (updated), or the box corner (an exactly zero component
   takes the + side) */
static int support_vertex(const mpcr_model_t* m, const odata* d, int g, const double dir[3], int* hint) {
  if (m->geom_type[g] == MPCR_GEOM_BOX) {
    /* the corner on the side of each axis; an axis that ties (tie_sign: the
       kernel's band, or MuJoCo's exact zero under EXACT_SUP) takes the + side */
    double l[3];
    mulmtv(l, d->geom_xmat[g], dir);
    const double ln = sqrt(dot3(l, l));
    return m->geom_cornadr[g] + (tie_sign(l[0], ln) >= 0 ? 1 : 0) + (tie_sign(l[1], ln) >= 0 ? 2 : 0) +
           (tie_sign(l[2], ln) >= 0 ? 4 : 0);
  }
  double p[3];
  support(m, d, g, dir, p, hint);
  return *hint;
}

/* hull vertex v of geom g relative to c */
static void vert_world(const mpcr_model_t* m, const odata* d, int g, int v, double w[3], const double* c) {
  mulmv(w, d->geom_xmat[g], m->hull_vert[v]);
  for (int k = 0; k < 3; k++) w[k] += d->geom_xpos[g][k] - c[k];
}

/* support value of geom g along dir (unit), relative to c: max over its
   vertices of dir . (x - c) */
static double support_value(const mpcr_model_t* m, const odata* d, int g, const double dir[3], int* hint,
                            const double* c) {
  double p[3];
  g_value_only = 1; /* the value only: no tie walk (hull_tie) */
  support_rel(m, d, g, dir, p, hint, c);
  g_value_only = 0;
  return dot3(p, dir);
}

/* diagnostic (oracle_poly_probe): the last manifold decision on one pair --
   [0] calls, [1] MPR depth, [2] best face separation, [3] its candidate index
   (-1 none), [4] support-vertex candidates on g1, [5] all candidates, [6] support vertex g1, [7] g2,
   [8] result (0 edge / no points, 1 face manifold), [9] reference face,
   [10] incident face, [11] points kept, [12..14] MPR normal */
static __thread int g_probe_pair = -1;
static __thread double g_probe[16];
void oracle_poly_probe(int pair, double* out) {
  if (out) memcpy(out, g_probe, sizeof(g_probe));
  g_probe_pair = pair;
  memset(g_probe, 0, sizeof(g_probe));
}
#define PROBE(i, v) do { if (pair == g_probe_pair) g_probe[i] = (v); } while (0)

static int poly_manifold(const mpcr_model_t* m, odata* d, int pair, int g1, int g2, const double n[3], double depth,
                         ocontact* out) {
  PROBE(0, g_probe[0] + 1);
  PROBE(1, depth);
  PROBE(12, n[0]); PROBE(13, n[1]); PROBE(14, n[2]);
  PROBE(8, 0); PROBE(9, -1); PROBE(10, -1); PROBE(11, 0);
  /* climbs start from the pair's hints (where MPR's queries ended) and do not
     update them; every query starts afresh (the kernel runs them on parallel
     lanes) */
  const int h0 = d->hint[pair][0], h1 = d->hint[pair][1];
  int h;
  const double nn[3] = {-n[0], -n[1], -n[2]};
  const double* cg = d->geom_xpos[g2]; /* the frame's origin: g2's centre */
  const long climb0 = g_mpr_stats[2];
  g_mpr_stats[8]++;
  h = h0;
  g_sup_kind = 1;
  const int s1 = support_vertex(m, d, g1, n, &h);
  h = h1;
  const int s2 = support_vertex(m, d, g2, nn, &h);
  /* candidate reference faces, at most 64 (the kernel's lanes), in this
     order: g1's on s1, g2's on s2, then the faces whose outward normal lies
     within the Gauss-map cone of MPR's direction (g1: n . nf >= POLY_CONE_COS,
     g2 the same about -n; face index order, those already listed skipped) --
     MJX's SAT scans every face; the cone keeps the axis search independent of
     which of two near-flush face pairs MPR's portal ended on.  SAT separation
     along each outward face normal */
  const int allf = depth > POLY_DEEP && m->geom_facenum[g1] + m->geom_facenum[g2] <= POLY_ALLF;
  const int c1 = allf ? 0 : (m->vert_facenum[s1] < 64 ? m->vert_facenum[s1] : 64);
  const int c2 = allf ? 0 : (m->vert_facenum[s2] < 64 - c1 ? m->vert_facenum[s2] : 64 - c1);
  int fid[POLY_ALLF], side[POLY_ALLF], nc = 0;
  for (int k = 0; k < c1; k++) { fid[nc] = m->vert_face[m->vert_faceadr[s1] + k]; side[nc++] = 0; }
  for (int k = 0; k < c2; k++) { fid[nc] = m->vert_face[m->vert_faceadr[s2] + k]; side[nc++] = 1; }
  if (allf) { /* every face of g1, then of g2 */
    for (int sd = 0; sd < 2; sd++) {
      const int g = sd ? g2 : g1, fa = m->geom_faceadr[g];
      for (int f = fa; f < fa + m->geom_facenum[g]; f++) { fid[nc] = f; side[nc++] = sd; }
    }
  }
  for (int sd = 0; sd < 2 && !allf; sd++) {
    const int g = sd ? g2 : g1, fa = m->geom_faceadr[g], cs = sd ? c2 : c1;
    const int ls = sd ? m->vert_faceadr[s2] : m->vert_faceadr[s1];
    for (int f = fa; f < fa + m->geom_facenum[g] && nc < 64; f++) {
      double nf[3], off;
      face_world(m, d, g, f, nf, &off, cg);
      if ((sd ? -1.0 : 1.0) * dot3(nf, n) < POLY_CONE_COS) continue;
      int dup = 0;
      for (int k = 0; k < cs; k++) dup |= m->vert_face[ls + k] == f;
      if (!dup) { fid[nc] = f; side[nc++] = sd; }
    }
  }
  g_mpr_stats[9] += nc;
  g_mpr_stats[10] += m->geom_facenum[g1] + m->geom_facenum[g2];
  g_mpr_stats[15] += c1 + c2;
  double sep[POLY_ALLF];
  double mx = -1e300;
  for (int k = 0; k < nc; k++) {
    const int two = side[k], g = two ? g2 : g1, go = two ? g1 : g2;
    double nf[3], off, mnf[3];
    face_world(m, d, g, fid[k], nf, &off, cg);
    for (int c = 0; c < 3; c++) mnf[c] = -nf[c];
    h = two ? h0 : h1;
    g_sup_kind = 2;
    sep[k] = -support_value(m, d, go, mnf, &h, cg) - off; /* min over go of nf . x, minus the plane */
    g_sup_kind = 0;
    if (sep[k] > mx) mx = sep[k];
  }
  /* the maximum's tie band: the lowest face index (a flush face pair has the
     same separation from either side; order-free, as a wave min) */
  int kb = -1;
  for (int k = 0; k < nc; k++)
    if (near_max(sep[k], mx) && (kb < 0 || fid[k] < fid[kb])) kb = k;
  PROBE(2, kb >= 0 ? sep[kb] : 0); PROBE(3, kb); PROBE(4, c1); PROBE(5, nc); PROBE(6, s1); PROBE(7, s2);
  if (kb < 0 || -sep[kb] > 1.05 * depth + 1e-5) return 0; /* an edge axis carries the contact */
  const int best_f = fid[kb], gr = side[kb] ? g2 : g1, gi = side[kb] ? g1 : g2;
  double nr[3], offr;
  face_world(m, d, gr, best_f, nr, &offr, cg);
  /* incident face: the most anti-parallel face on gi's support vertex along -nr */
  const double mnr[3] = {-nr[0], -nr[1], -nr[2]};
  h = gi == g1 ? h0 : h1;
  g_sup_kind = 1;
  const int si = support_vertex(m, d, gi, mnr, &h);
  g_sup_kind = 0;
  const int ci = m->vert_facenum[si] < 64 ? m->vert_facenum[si] : 64;
  double al[64];
  mx = -1e300;
  for (int k = 0; k < ci; k++) {
    double nf[3], off;
    face_world(m, d, gi, m->vert_face[m->vert_faceadr[si] + k], nf, &off, cg);
    al[k] = -dot3(nf, nr);
    if (al[k] > mx) mx = al[k];
  }
  int inc_f = -1;
  for (int k = 0; k < ci && inc_f < 0; k++)
    if (near_max(al[k], mx)) inc_f = m->vert_face[m->vert_faceadr[si] + k];
  if (inc_f < 0) return 0;
  /* clip the incident polygon by the reference face's side planes */
  enum { MAXP = 2 * MPCR_FACE_MAXV + 2 };
  double poly[2][MAXP][3], ref[MPCR_FACE_MAXV][3];
  int np = m->face_vnum[inc_f], cur = 0;
  const int nrv = m->face_vnum[best_f];
  for (int k = 0; k < np; k++) vert_world(m, d, gi, m->face_vert[m->face_vadr[inc_f] + k], poly[0][k], cg);
  for (int k = 0; k < nrv; k++) vert_world(m, d, gr, m->face_vert[m->face_vadr[best_f] + k], ref[k], cg);
  g_mpr_stats[11]++;
  g_mpr_stats[12] += nrv;
  g_mpr_stats[13] += np;
  g_mpr_stats[14] += g_mpr_stats[2] - climb0;
  for (int e = 0; e < nrv && np > 0; e++) {
    const double* A = ref[e];
    const double* B = ref[e + 1 == nrv ? 0 : e + 1];
    double ed[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, sn[3];
    cross3(sn, ed, nr); /* outward side-plane normal (counter-clockwise polygon about nr) */
    int no = 0;
    for (int k = 0; k < np; k++) {
      const double* P = poly[cur][k];
      const double* Q = poly[cur][k + 1 == np ? 0 : k + 1];
      const double dp = sn[0] * (P[0] - A[0]) + sn[1] * (P[1] - A[1]) + sn[2] * (P[2] - A[2]);
      const double dq = sn[0] * (Q[0] - A[0]) + sn[1] * (Q[1] - A[1]) + sn[2] * (Q[2] - A[2]);
      if (dp <= 0 && no < MAXP) memcpy(poly[cur ^ 1][no++], P, sizeof(double) * 3);
      if (((dp < 0 && dq > 0) || (dp > 0 && dq < 0)) && no < MAXP) {
        const double w = dp / (dp - dq);
        for (int c = 0; c < 3; c++) poly[cur ^ 1][no][c] = P[c] + w * (Q[c] - P[c]);
        no++;
      }
    }
    np = no;
    cur ^= 1;
  }
  /* the clipped points below the reference plane */
  double pts[MAXP][3], dist[MAXP];
  int nk = 0;
  const double margin = m->pair_margin[pair] - m->pair_gap[pair];
  for (int k = 0; k < np; k++) {
    const double dk = dot3(nr, poly[cur][k]) - offr;
    if (dk < margin) { memcpy(pts[nk], poly[cur][k], sizeof(double) * 3); dist[nk++] = dk; }
  }
  PROBE(9, best_f); PROBE(10, inc_f); PROBE(11, nk);
  const double sg = gr == g1 ? 1.0 : -1.0; /* contact normal g1 -> g2 */
  const double cn[3] = {sg * nr[0], sg * nr[1], sg * nr[2]};
  if (nk == 0) {
    /* no clipped point below the reference plane (a small reference face over
       a deep penetration): the SAT axis still carries the contact -- one point
       at gi's support vertex along -nr, at its distance from the reference
       plane (MPR's own normal for a penetration this deep is the portal face
       it ends on, a path that fp32 and fp64 take differently) */
    g_mpr_stats[5]++;
    double P[3], pos[3];
    vert_world(m, d, gi, si, P, cg);
    const double dk = dot3(nr, P) - offr;
    if (!(dk < margin)) return 0;
    for (int c = 0; c < 3; c++) pos[c] = P[c] + cg[c] - 0.5 * dk * nr[c];
    set_contact(&out[0], dk, pos, cn);
    PROBE(8, 2);
    return 1;
  }
  PROBE(8, 1);
  /* at most 4: _manifold_points' picks (a = the first, b = the farthest from
     a, c = the farthest from line ab, d = the farthest from edge bc or ac;
     near_max's first index within the tie band) */
  int idx[4] = {0, 0, 0, 0}, cnt = nk < 4 ? nk : 4;
  if (nk <= 4) {
    for (int k = 0; k < nk; k++) idx[k] = k;
  } else {
    const double* a = pts[0];
    double mx, v;
#define PICK(EXPR, OUT)                                            \
    do {                                                           \
      mx = -1;                                                     \
      for (int k = 0; k < nk; k++) { const double* p = pts[k]; v = (EXPR); if (v > mx) mx = v; } \
      for (int k = 0; k < nk; k++) { const double* p = pts[k]; if (near_max((EXPR), mx)) { OUT = k; break; } } \
    } while (0)
    double best_bp, best_ap;
    PICK((a[0] - p[0]) * (a[0] - p[0]) + (a[1] - p[1]) * (a[1] - p[1]) + (a[2] - p[2]) * (a[2] - p[2]), idx[1]);
    const double* b = pts[idx[1]];
    double amb[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]}, ab[3];
    cross3(ab, nr, amb);
    PICK(fabs((a[0] - p[0]) * ab[0] + (a[1] - p[1]) * ab[1] + (a[2] - p[2]) * ab[2]), idx[2]);
    const double* c = pts[idx[2]];
    double amc[3] = {a[0] - c[0], a[1] - c[1], a[2] - c[2]}, bmc[3] = {b[0] - c[0], b[1] - c[1], b[2] - c[2]};
    double ac[3], bc[3];
    cross3(ac, nr, amc);
    cross3(bc, nr, bmc);
    int ibp = 0, iap = 0;
    PICK(fabs((b[0] - p[0]) * bc[0] + (b[1] - p[1]) * bc[1] + (b[2] - p[2]) * bc[2]), ibp);
    best_bp = mx;
    PICK(fabs((a[0] - p[0]) * ac[0] + (a[1] - p[1]) * ac[1] + (a[2] - p[2]) * ac[2]), iap);
    best_ap = mx;
#undef PICK
    idx[3] = beats(best_ap, best_bp) ? iap : ibp;
  }
  for (int s = 0; s < cnt; s++) {
    int dup = 0;
    for (int t = 0; t < s; t++) dup |= idx[t] == idx[s];
    if (dup) continue;
    const int k = idx[s];
    double pos[3];
    for (int c = 0; c < 3; c++) pos[c] = pts[k][c] + cg[c] - 0.5 * dist[k] * nr[c];
    set_contact(&out[s], dist[k], pos, cn);
  }
  return 1;
}

/* plane - cylinder (4 slots): MuJoCo's mjc_PlaneCylinder (mujoco 3.3.1
   engine_collision_primitive.c, restated): slot 0 the deepest rim point of the
   cap nearer the plane (always reported), then, when it penetrates, the rim
   point of the other cap on the same side, and two points of the near cap's
   rim 120 degrees either side of the first (an equilateral triangle with it).
   Normal = the plane's, positions half-way through the penetration. */
static void col_plane_cylinder(const mpcr_model_t* m, odata* d, int pair, int gp, int g, ocontact* out) {
  const double* R1 = d->geom_xmat[gp];
  const double* R2 = d->geom_xmat[g];
  const double* sz = m->geom_size[g];
  const double* x = d->geom_xpos[g];
  const double n[3] = {R1[2], R1[5], R1[8]};
  double ax[3] = {R2[2], R2[5], R2[8]}, dif[3], vec[3], pos[3];
  for (int k = 0; k < 3; k++) dif[k] = x[k] - d->geom_xpos[gp][k];
  double prjaxis = dot3(n, ax);
  if (prjaxis > 0) { /* the axis towards the plane */
    for (int k = 0; k < 3; k++) ax[k] = -ax[k];
    prjaxis = -prjaxis;
  }
  const double dist0 = dot3(dif, n);
  for (int k = 0; k < 3; k++) vec[k] = ax[k] * prjaxis - n[k]; /* radial direction towards the plane */
  const double len = norm3(vec);
  if (len < MINVAL) { vec[0] = R2[0]; vec[1] = R2[3]; vec[2] = R2[6]; }
  else for (int k = 0; k < 3; k++) vec[k] /= len;
  for (int k = 0; k < 3; k++) { vec[k] *= sz[0]; ax[k] *= sz[1]; }
  const double prjvec = dot3(vec, n);
  prjaxis *= sz[1];
  const double margin = m->pair_margin[pair] - m->pair_gap[pair];
  double dist = dist0 + prjaxis + prjvec;
  for (int k = 0; k < 3; k++) pos[k] = x[k] + vec[k] + ax[k] - 0.5 * dist * n[k];
  set_contact(&out[0], dist, pos, n);
  if (!(dist <= margin)) return;
  dist = dist0 - prjaxis + prjvec;
  if (dist <= margin) {
    for (int k = 0; k < 3; k++) pos[k] = x[k] + vec[k] - ax[k] - 0.5 * dist * n[k];
    set_contact(&out[1], dist, pos, n);
  }
  dist = dist0 + prjaxis - 0.5 * prjvec;
  if (dist <= margin) {
    double v1[3];
    cross3(v1, vec, ax);
    normalize3(v1);
    for (int k = 0; k < 3; k++) v1[k] *= sz[0] * sqrt(3.0) / 2;
    for (int sgn = 0; sgn < 2; sgn++) {
      const double sv = sgn ? -1.0 : 1.0;
      for (int k = 0; k < 3; k++) pos[k] = x[k] + sv * v1[k] + ax[k] - 0.5 * vec[k] - 0.5 * dist * n[k];
      set_contact(&out[2 + sgn], dist, pos, n);
    }
  }
}

static void col_plane_convex(const mpcr_model_t* m, odata* d, int pair, int gp, int g, ocontact* out) {
  if (m->geom_type[g] == MPCR_GEOM_MESH) {
    col_plane_mesh(m, d, pair, gp, g, out);
    return;
  }
  if (m->geom_type[g] == MPCR_GEOM_CYLINDER && m->pair_ncon[pair] == 4) {
    col_plane_cylinder(m, d, pair, gp, g, out);
    return;
  }
  const double* R = d->geom_xmat[gp];
  double n[3] = {R[2], R[5], R[8]}, nn[3] = {-R[2], -R[5], -R[8]}, p[3], pos[3];
  g_sup_kind = 3;
  support(m, d, g, nn, p, &d->hint[pair][1]);
  g_sup_kind = 0;
  double dist = (p[0] - d->geom_xpos[gp][0]) * n[0] + (p[1] - d->geom_xpos[gp][1]) * n[1] +
                (p[2] - d->geom_xpos[gp][2]) * n[2];
  for (int k = 0; k < 3; k++) pos[k] = p[k] - 0.5 * dist * n[k];
  set_contact(out, dist, pos, n);
}

/* diagnostic (oracle_narrow_stats): narrow-phase calls executed per pair
   function (after the culls), per thread -- what bench/flops_model.json
   credits per step */
static __thread long g_narrow_stats[16];
void oracle_narrow_stats(long* out, int reset) {
  if (out) memcpy(out, g_narrow_stats, sizeof(g_narrow_stats));
  if (reset) memset(g_narrow_stats, 0, sizeof(g_narrow_stats));
}

static void collision(const mpcr_model_t* m, odata* d) {
  d->ncon = m->ncon;
  for (int p = 0; p < m->npair; p++) {
    int g1 = m->pair_geom1[p], g2 = m->pair_geom2[p];
    ocontact* out = &d->con[m->pair_conadr[p]];
    for (int s = 0; s < m->pair_ncon[p]; s++) {
      out[s].dist = 1e30;
      out[s].pair = p;
      out[s].active = 0;
    }
    /* unmasked pairs only feed the solver: cull by bounding spheres (and, for
       the general convex functions, plane / box vs the other bounding sphere;
       all exact: a culled pair cannot touch) */
    if (m->pair_slotadr[p] < 0) {
      double dif[3];
      for (int k = 0; k < 3; k++) dif[k] = d->geom_xpos[g2][k] - d->geom_xpos[g1][k];
      if (m->geom_type[g1] != MPCR_GEOM_PLANE) {
        if (norm3(dif) > m->geom_rbound[g1] + m->geom_rbound[g2] + m->pair_margin[p]) continue;
        if (m->pair_func[p] == MPCR_COL_CONVEX &&
            (m->geom_type[g1] == MPCR_GEOM_BOX || m->geom_type[g2] == MPCR_GEOM_BOX)) {
          int b1 = m->geom_type[g1] == MPCR_GEOM_BOX, gb = b1 ? g1 : g2;
          double dd[3] = {b1 ? dif[0] : -dif[0], b1 ? dif[1] : -dif[1], b1 ? dif[2] : -dif[2]}, l[3], o2 = 0;
          mulmtv(l, d->geom_xmat[gb], dd);
          for (int k = 0; k < 3; k++) {
            double e = fabs(l[k]) - m->geom_size[gb][k];
            if (e > 0) o2 += e * e;
          }
          if (sqrt(o2) > m->geom_rbound[b1 ? g2 : g1] + m->pair_margin[p]) continue;
        }
      } else {
        const double* R = d->geom_xmat[g1];
        if (R[2] * dif[0] + R[5] * dif[1] + R[8] * dif[2] > m->geom_rbound[g2] + m->pair_margin[p]) continue;
      }
    }
    const double *s1 = m->geom_size[g1], *s2 = m->geom_size[g2];
    g_narrow_stats[m->pair_func[p] & 15]++;
    switch (m->pair_func[p]) {
      case MPCR_COL_PLANE_CAPSULE: col_plane_capsule(d, g1, g2, s2, out); break;
      case MPCR_COL_PLANE_BOX: col_plane_box(d, g1, g2, s2, out); break;
      case MPCR_COL_CAPSULE_CAPSULE: col_capsule_capsule(d, g1, g2, s1, s2, out); break;
      case MPCR_COL_CAPSULE_BOX: col_capsule_box(d, g1, g2, s1, s2, out); break;
      case MPCR_COL_BOX_BOX: col_box_box(d, g1, g2, s1, s2, m->pair_margin[p] - m->pair_gap[p], out); break;
      case MPCR_COL_CONVEX: col_convex(m, d, p, g1, g2, out); break;
      case MPCR_COL_PLANE_CONVEX: col_plane_convex(m, d, p, g1, g2, out); break;
      default: break;
    }
    for (int s = 0; s < m->pair_ncon[p]; s++) {
      out[s].pair = p;
      out[s].active = !(m->disableflags & MPCR_DSBL_CONTACT) && out[s].dist < m->pair_margin[p] - m->pair_gap[p];
    }
  }
}

/* ------------------------------------------------------------------------ */
/* constraints: equality, limits, pyramidal contacts + impedance             */

static void impedance(const double solimp[5], double pos, double margin, double* imp) {
  double dmin = clampd(solimp[0], MINIMP, MAXIMP), dmax = clampd(solimp[1], MINIMP, MAXIMP);
  double width = solimp[2], mid = solimp[3], power = solimp[4];
  if (dmin == dmax || width <= MINVAL) { *imp = 0.5 * (dmin + dmax); return; }
  double x = fabs((pos - margin) / width);
  if (x >= 1) { *imp = dmax; return; }
  if (x <= 0) { *imp = dmin; return; }
  double y;
  if (power == 1) y = x;
  else if (x <= mid) y = pow(x, power) / pow(mid, power - 1);
  else y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
  *imp = dmin + y * (dmax - dmin);
}

static int add_row(const mpcr_model_t* m, odata* d, int eq, double pos, double margin, double diag,
                   const double solref[2], const double solimp[5]) {
  if (d->nefc >= MAXEFC) { d->efc_trunc++; return -1; }
  int r = d->nefc++;
  d->efc_eq[r] = eq;
  d->efc_pos[r] = pos;
  d->efc_margin[r] = margin;
  d->efc_diag[r] = diag;
  d->efc_dim[r] = 1;
  memcpy(d->efc_solref[r], solref, 2 * sizeof(double));
  memcpy(d->efc_solimp[r], solimp, 5 * sizeof(double));
  for (int i = 0; i < m->nv; i++) d->efc_J[r][i] = 0;
  return r;
}

static void make_constraint(const mpcr_model_t* m, odata* d) {
  int nv = m->nv;
  d->nefc = 0;
  d->efc_trunc = 0;
  /* equalities in model order.  connect: 3 rows, anchor1 (body1) - anchor2
     (body2) in world; joint: q1 - qpos0_1 = poly(q2 - qpos0_2) */
  if (!(m->disableflags & MPCR_DSBL_EQUALITY))
    for (int e = 0; e < m->neq; e++) {
      if (m->eq_type[e] == MPCR_EQ_CONNECT) {
        int b1 = m->eq_obj1[e], b2 = m->eq_obj2[e];
        double p1[3], p2[3], t[3], j1[3][NV], j2[3][NV];
        mulmv(t, d->xmat[b1], m->eq_data[e]);
        for (int k = 0; k < 3; k++) p1[k] = d->xpos[b1][k] + t[k];
        mulmv(t, d->xmat[b2], m->eq_data[e] + 3);
        for (int k = 0; k < 3; k++) p2[k] = d->xpos[b2][k] + t[k];
        jac_point(m, d, b1, p1, j1);
        jac_point(m, d, b2, p2, j2);
        double diag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
        for (int k = 0; k < 3; k++) {
          int r = add_row(m, d, 1, p1[k] - p2[k], 0, diag, m->eq_solref[e], m->eq_solimp[e]);
          if (r < 0) continue;
          for (int i = 0; i < nv; i++) d->efc_J[r][i] = j1[k][i] - j2[k][i];
        }
        continue;
      }
      if (m->eq_type[e] != MPCR_EQ_JOINT) continue;
      int j1 = m->eq_obj1[e], j2 = m->eq_obj2[e];
      const double* c = m->eq_data[e];
      int a1 = m->jnt_qposadr[j1], d1 = m->jnt_dofadr[j1];
      double pos, deriv = 0, diag = m->dof_invweight0[d1];
      if (j2 >= 0) {
        int a2 = m->jnt_qposadr[j2];
        double dif = d->qpos[a2] - m->qpos0[a2];
        pos = d->qpos[a1] - m->qpos0[a1] - (c[0] + dif * (c[1] + dif * (c[2] + dif * (c[3] + dif * c[4]))));
        deriv = c[1] + dif * (2 * c[2] + dif * (3 * c[3] + dif * 4 * c[4]));
        diag += m->dof_invweight0[m->jnt_dofadr[j2]];
      } else {
        pos = d->qpos[a1] - m->qpos0[a1] - c[0];
      }
      int r = add_row(m, d, 1, pos, 0, diag, m->eq_solref[e], m->eq_solimp[e]);
      if (r < 0) continue;
      d->efc_J[r][d1] = 1;
      if (j2 >= 0) d->efc_J[r][m->jnt_dofadr[j2]] -= deriv;
    }
  /* joint limits (hinge / slide) */
  if (!(m->disableflags & MPCR_DSBL_LIMIT))
    for (int j = 0; j < m->njnt; j++) {
      if (!m->jnt_limited[j] || (m->jnt_type[j] != MPCR_JNT_HINGE && m->jnt_type[j] != MPCR_JNT_SLIDE)) continue;
      double q = d->qpos[m->jnt_qposadr[j]];
      int dof = m->jnt_dofadr[j];
      for (int side = 0; side < 2; side++) {
        double dist = side == 0 ? q - m->jnt_range[j][0] : m->jnt_range[j][1] - q;
        if (dist < m->jnt_margin[j]) {
          int r = add_row(m, d, 0, dist, m->jnt_margin[j], m->dof_invweight0[dof], m->jnt_solref[j], m->jnt_solimp[j]);
          if (r >= 0) d->efc_J[r][dof] = side == 0 ? 1 : -1;
        }
      }
    }
  /* spatial tendon limits (after the joint limits, mj_instantiateLimit):
     length |x_s2 - x_s1|, moment (x_s2 - x_s1)^T (J_s2 - J_s1) / length */
  if (!(m->disableflags & MPCR_DSBL_LIMIT))
    for (int t = 0; t < m->nten; t++) {
      if (!m->ten_limited[t]) continue;
      int s1 = m->ten_site[t][0], s2 = m->ten_site[t][1];
      double dif[3], j1[3][NV], j2[3][NV], jt[NV];
      for (int k = 0; k < 3; k++) dif[k] = d->site_xpos[s2][k] - d->site_xpos[s1][k];
      double len = norm3(dif), il = 1 / (len > MINVAL ? len : MINVAL);
      jac_point(m, d, m->site_bodyid[s1], d->site_xpos[s1], j1);
      jac_point(m, d, m->site_bodyid[s2], d->site_xpos[s2], j2);
      for (int i = 0; i < nv; i++) {
        double v = 0;
        for (int k = 0; k < 3; k++) v += dif[k] * il * (j2[k][i] - j1[k][i]);
        jt[i] = v;
      }
      for (int side = 0; side < 2; side++) {
        double dist = side == 0 ? len - m->ten_range[t][0] : m->ten_range[t][1] - len;
        if (dist < m->ten_margin[t]) {
          int r = add_row(m, d, 0, dist, m->ten_margin[t], m->ten_invweight0[t], m->ten_solref[t], m->ten_solimp[t]);
          if (r >= 0)
            for (int i = 0; i < nv; i++) d->efc_J[r][i] = side == 0 ? jt[i] : -jt[i];
        }
      }
    }
  /* contacts: pyramidal, condim 3 -> 4 rows J_n +- mu J_t{1,2}; condim 1 -> J_n;
     elliptic, condim 3 -> 3 rows J_n, J_t1, J_t2 (friction rows: pos 0) */
  for (int c = 0; c < d->ncon; c++) {
    ocontact* con = &d->con[c];
    if (!con->active) continue;
    int p = con->pair;
    int b1 = m->geom_bodyid[m->pair_geom1[p]], b2 = m->geom_bodyid[m->pair_geom2[p]];
    double j1[3][NV], j2[3][NV], jd[3][NV];
    jac_point(m, d, b1, con->pos, j1);
    jac_point(m, d, b2, con->pos, j2);
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < nv; i++) jd[k][i] = j2[k][i] - j1[k][i];
    double jf[3][NV];
    for (int a = 0; a < 3; a++)
      for (int i = 0; i < nv; i++)
        jf[a][i] = con->frame[3 * a] * jd[0][i] + con->frame[3 * a + 1] * jd[1][i] + con->frame[3 * a + 2] * jd[2][i];
    double tran = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    double mu = m->pair_friction[p], margin = m->pair_margin[p] - m->pair_gap[p];
    if (m->pair_condim[p] == 1) {
      int r = add_row(m, d, 0, con->dist, margin, tran, m->pair_solref[p], m->pair_solimp[p]);
      if (r >= 0)
        for (int i = 0; i < nv; i++) d->efc_J[r][i] = jf[0][i];
      continue;
    }
    if (m->cone == MPCR_CONE_ELLIPTIC) {
      if (d->nefc + 3 > MAXEFC) { d->efc_trunc += 3; continue; }
      for (int k = 0; k < 3; k++) {
        int r = add_row(m, d, k == 0 ? 2 : 3, k == 0 ? con->dist : 0, k == 0 ? margin : 0, tran,
                        m->pair_solref[p], m->pair_solimp[p]);
        for (int i = 0; i < nv; i++) d->efc_J[r][i] = jf[k][i];
        d->efc_dim[r] = k == 0 ? 3 : 0;
        d->efc_fri[r][0] = d->efc_fri[r][1] = mu;
      }
      continue;
    }
    for (int k = 1; k < 3; k++)
      for (int sgn = 1; sgn >= -1; sgn -= 2) {
        int r = add_row(m, d, 0, con->dist, margin, tran * (1 + mu * mu), m->pair_solref[p], m->pair_solimp[p]);
        if (r >= 0)
          for (int i = 0; i < nv; i++) d->efc_J[r][i] = jf[0][i] + sgn * mu * jf[k][i];
      }
  }
  /* impedance, regularisation and reference acceleration (mj_makeImpedance) */
  for (int r = 0; r < d->nefc; r++) {
    double v = 0;
    for (int i = 0; i < nv; i++) v += d->efc_J[r][i] * d->qvel[i];
    d->efc_vel[r] = v;
    double imp;
    impedance(d->efc_solimp[r], d->efc_pos[r], d->efc_margin[r], &imp);
    double R = (1 - imp) / imp * d->efc_diag[r];
    if (R < MINVAL) R = MINVAL;
    d->efc_D[r] = 1 / R;
    double K, B, tc = d->efc_solref[r][0], dr = d->efc_solref[r][1];
    double dmax = clampd(d->efc_solimp[r][1], MINIMP, MAXIMP);
    if (tc > 0) {
      if (!(m->disableflags & MPCR_DSBL_REFSAFE) && tc < 2 * m->timestep) tc = 2 * m->timestep;
      K = 1 / (dmax * dmax * tc * tc * dr * dr);
      B = 2 / (dmax * tc);
    } else {
      K = -tc / (dmax * dmax);
      B = -dr / dmax;
    }
    d->efc_aref[r] = -B * v - K * imp * (d->efc_pos[r] - d->efc_margin[r]);
  }
  /* elliptic contacts: friction R = R_n fri_0^2 / (fri_j^2 impratio), and the
     cone slope of the primal zones mu = fri_0 sqrt(R_t1 / R_n) */
  for (int r = 0; r < d->nefc; r++) {
    if (d->efc_eq[r] != 2) continue;
    double Rn = 1 / d->efc_D[r];
    for (int j = 1; j < d->efc_dim[r]; j++) {
      double fj = d->efc_fri[r][j - 1];
      d->efc_D[r + j] = 1 / (Rn * d->efc_fri[r][0] * d->efc_fri[r][0] / (fj * fj * m->impratio));
    }
    d->efc_mu[r] = d->efc_fri[r][0] * sqrt(d->efc_D[r] / d->efc_D[r + 1]);
  }
}

/* ------------------------------------------------------------------------ */
/* Newton solver (primal), one iteration + exact-quadratic line search       */

/* the line search's step sizes, point costs / derivatives and bracket
   arithmetic: mpcr_hp stays double in the fp32 build too (oracle_f32.c), as
   the dual-arm kernel keeps them in fp64 (rollout.hip LsReal: the point cost
   alpha^2 q2 + alpha q1 + q0 cancels the constant q0 to compare candidates
   that differ in the last fp32 bits); the row sums stay in the build's
   precision */
#ifndef MPCR_HP_DEFINED
typedef double mpcr_hp;
#endif
typedef struct { mpcr_hp alpha, cost, d0, d1; } lspt;

static void mulM(const mpcr_model_t* m, const odata* d, const double* x, double* y) {
  for (int i = 0; i < m->nv; i++) {
    double s = 0;
    for (int j = 0; j < m->nv; j++) s += d->M[i][j] * x[j];
    y[i] = s;
  }
}

/* Elliptic contact with normal row r (condim 3), MuJoCo's primal cone cost
   (mj_constraintUpdate): with N = mu jar_n, U_j = fri_j jar_tj, T = |U|,
     top    N >= mu T              satisfied, no cost;
     bottom mu N + T <= 0          0.5 sum_k D_k jar_k^2 (all rows quadratic);
     middle otherwise              0.5 Dm (N - mu T)^2, Dm = D_n / (mu^2 (1 + mu^2)).
   Returns the cost; f = -d cost / d jar, H = d^2 cost / d jar^2 (3 x 3). */
static double ell_update(const odata* d, int r, const double* jar, double f[3], double H[3][3]) {
  double mu = d->efc_mu[r], N = mu * jar[r], U[2], T = 0;
  for (int j = 0; j < 2; j++) { U[j] = d->efc_fri[r][j] * jar[r + 1 + j]; T += U[j] * U[j]; }
  T = sqrt(T);
  memset(H, 0, 9 * sizeof(double));
  if (N >= mu * T || (T <= 0 && N >= 0)) {
    f[0] = f[1] = f[2] = 0;
    return 0;
  }
  if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
    double c = 0;
    for (int k = 0; k < 3; k++) {
      f[k] = -d->efc_D[r + k] * jar[r + k];
      H[k][k] = d->efc_D[r + k];
      c += 0.5 * d->efc_D[r + k] * jar[r + k] * jar[r + k];
    }
    return c;
  }
  double Dm = d->efc_D[r] / (mu * mu * (1 + mu * mu)), phi = N - mu * T;
  /* grad phi = (mu, -mu fri_j U_j / T); hess phi_tt = -mu fri_j fri_k (delta_jk - U_j U_k / T^2) / T */
  double g[3] = {mu, -mu * d->efc_fri[r][0] * U[0] / T, -mu * d->efc_fri[r][1] * U[1] / T};
  for (int a = 0; a < 3; a++) f[a] = -Dm * phi * g[a];
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) H[a][b] = Dm * g[a] * g[b];
  for (int j = 0; j < 2; j++)
    for (int k = 0; k < 2; k++) {
      double h = -mu * d->efc_fri[r][j] * d->efc_fri[r][k] * ((j == k) - U[j] * U[k] / (T * T)) / T;
      H[1 + j][1 + k] += Dm * phi * h;
    }
  return 0.5 * Dm * phi * phi;
}

/* constraint cost and forces (f = -D jar on the quadratic rows, cone forces) */
static double efc_cost_force(const odata* d, const double* jar, double* f) {
  double c = 0;
  for (int r = 0; r < d->nefc; r++) {
    int t = d->efc_eq[r];
    if (t == 2) {
      double H[3][3];
      c += ell_update(d, r, jar, f + r, H);
    } else if (t == 1 || (t == 0 && jar[r] < 0)) {
      f[r] = -d->efc_D[r] * jar[r];
      c += 0.5 * d->efc_D[r] * jar[r] * jar[r];
    } else if (t == 0) {
      f[r] = 0;
    }
  }
  return c;
}

static double solver_cost(const mpcr_model_t* m, const odata* d, const double* qacc, const double* Ma,
                          const double* jar) {
  double gauss = 0, f[MAXEFC];
  for (int i = 0; i < m->nv; i++) gauss += (Ma[i] - d->qfrc_smooth[i]) * (qacc[i] - d->qacc_smooth[i]);
  return 0.5 * gauss + efc_cost_force(d, jar, f);
}

static void eval_jar(const mpcr_model_t* m, const odata* d, const double* x, double* jar) {
  for (int r = 0; r < d->nefc; r++) {
    double s = 0;
    for (int i = 0; i < m->nv; i++) s += d->efc_J[r][i] * x[i];
    jar[r] = s - d->efc_aref[r];
  }
}

/* cost and its first two alpha-derivatives of the elliptic contact at row r
   along jar + alpha jv (the zones re-evaluated at alpha) */
static void ell_line(const odata* d, int r, const double* jar, const double* jv, mpcr_hp alpha, double c[3]) {
  double x[3], v[3];
  for (int k = 0; k < 3; k++) { x[k] = jar[r + k] + alpha * jv[r + k]; v[k] = jv[r + k]; }
  double mu = d->efc_mu[r], N = mu * x[0], N1 = mu * v[0], U[2], W[2], T = 0, UW = 0, WW = 0;
  for (int j = 0; j < 2; j++) {
    U[j] = d->efc_fri[r][j] * x[1 + j];
    W[j] = d->efc_fri[r][j] * v[1 + j];
    T += U[j] * U[j];
    UW += U[j] * W[j];
    WW += W[j] * W[j];
  }
  T = sqrt(T);
  c[0] = c[1] = c[2] = 0;
  if (N >= mu * T || (T <= 0 && N >= 0)) return;
  if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
    for (int k = 0; k < 3; k++) {
      double D = d->efc_D[r + k];
      c[0] += 0.5 * D * x[k] * x[k];
      c[1] += D * x[k] * v[k];
      c[2] += D * v[k] * v[k];
    }
    return;
  }
  double Dm = d->efc_D[r] / (mu * mu * (1 + mu * mu));
  double T1 = UW / T, T2 = (WW - T1 * T1) / T;
  double phi = N - mu * T, phi1 = N1 - mu * T1, phi2 = -mu * T2;
  c[0] = 0.5 * Dm * phi * phi;
  c[1] = Dm * phi * phi1;
  c[2] = Dm * (phi1 * phi1 + phi * phi2);
}

static lspt ls_eval(const odata* d, const double qg[3], const double* jar, const double* jv, mpcr_hp alpha) {
  double q0 = qg[0], q1 = qg[1], q2 = qg[2], e[3] = {0, 0, 0};
  for (int r = 0; r < d->nefc; r++) {
    mpcr_hp x = jar[r] + alpha * jv[r];
    if (d->efc_eq[r] == 2) {
      double c[3];
      ell_line(d, r, jar, jv, alpha, c);
      for (int k = 0; k < 3; k++) e[k] += c[k];
      continue;
    }
    if (d->efc_eq[r] == 3) continue;
    if (d->efc_eq[r] == 1 || x < 0) {
      double D = d->efc_D[r];
      q0 += 0.5 * D * jar[r] * jar[r];
      q1 += D * jv[r] * jar[r];
      q2 += 0.5 * D * jv[r] * jv[r];
    }
  }
  lspt p;
  p.alpha = alpha;
  p.cost = alpha * alpha * q2 + alpha * q1 + q0 + e[0];
  p.d0 = 2 * alpha * q2 + q1 + e[1];
  p.d1 = 2 * (mpcr_hp)q2 + e[2];
  if (p.d1 == 0) p.d1 = MINVAL;
  return p;
}

static void solve(const mpcr_model_t* m, odata* d) {
  int nv = m->nv, nefc = d->nefc;
  if (nefc == 0) {
    memcpy(d->qacc, d->qacc_smooth, sizeof(double) * nv);
    for (int i = 0; i < nv; i++) d->qfrc_constraint[i] = 0;
    return;
  }
  double Ma[NV], jar[MAXEFC], qacc[NV];
  /* warm start: the better of qacc_warmstart and qacc_smooth */
  if (!(m->disableflags & MPCR_DSBL_WARMSTART)) {
    double Mw[NV], jw[MAXEFC], Ms[NV], js[MAXEFC];
    mulM(m, d, d->qacc_warmstart, Mw);
    eval_jar(m, d, d->qacc_warmstart, jw);
    mulM(m, d, d->qacc_smooth, Ms);
    eval_jar(m, d, d->qacc_smooth, js);
    double cw = solver_cost(m, d, d->qacc_warmstart, Mw, jw), cs = solver_cost(m, d, d->qacc_smooth, Ms, js);
    memcpy(qacc, cw < cs ? d->qacc_warmstart : d->qacc_smooth, sizeof(double) * nv);
    d->dbg[0] = cw < cs;
    d->dbg[1] = cw;
    d->dbg[2] = cs;
  } else {
    memcpy(qacc, d->qacc_smooth, sizeof(double) * nv);
  }
  mulM(m, d, qacc, Ma);
  eval_jar(m, d, qacc, jar);
  double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  double cost = solver_cost(m, d, qacc, Ma, jar), prev_cost = 1e300;
  for (int it = 0;; it++) {
    /* gradient and Newton direction with the Hessian of the active set */
    double grad[NV], H[NV][NV], Lh[NV][NV], Mgrad[NV], search[NV], f[MAXEFC];
    efc_cost_force(d, jar, f);
    for (int i = 0; i < nv; i++) {
      double qc = 0;
      for (int r = 0; r < nefc; r++) qc += d->efc_J[r][i] * f[r];
      grad[i] = Ma[i] - d->qfrc_smooth[i] - qc;
    }
    double gn = 0;
    for (int i = 0; i < nv; i++) gn += grad[i] * grad[i];
    gn = sqrt(gn);
    /* MuJoCo's stop test, plus the kernel's fp32 resolution floor (an
       improvement within 1e-6 of the cost ends the solve): the same rule on
       both sides, so neither iterates where the other cannot */
    if (it >= m->iterations || scale * (prev_cost - cost) < m->tolerance || scale * gn < m->tolerance ||
        (!(g_exact & EXACT_NEWTON) && prev_cost - cost <= g_floor[0] * fabs(cost)))
      break;
    for (int i = 0; i < nv; i++)
      for (int j = 0; j < nv; j++) {
        double h = d->M[i][j];
        for (int r = 0; r < nefc; r++)
          if (d->efc_eq[r] == 1 || (d->efc_eq[r] == 0 && jar[r] < 0))
            h += d->efc_J[r][i] * d->efc_D[r] * d->efc_J[r][j];
        H[i][j] = h;
      }
    /* cone Hessian blocks J_c^T H_c J_c of the elliptic contacts */
    for (int r = 0; r < nefc; r++) {
      if (d->efc_eq[r] != 2) continue;
      double fc[3], Hc[3][3];
      ell_update(d, r, jar, fc, Hc);
      for (int i = 0; i < nv; i++)
        for (int j = 0; j < nv; j++) {
          double h = 0;
          for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) h += d->efc_J[r + a][i] * Hc[a][b] * d->efc_J[r + b][j];
          H[i][j] += h;
        }
    }
    if (d->ls_dump && it == 0)
      for (int i = 0; i < nv; i++)
        for (int j = 0; j < nv; j++) d->ls_dump[8 + 4 * 512 + i * nv + j] = H[i][j];
    chol(Lh, H, nv);
    chol_solve(Mgrad, Lh, grad, nv);
    for (int i = 0; i < nv; i++) search[i] = -Mgrad[i];
    if (it == 0)
      for (int i = 0; i < nv; i++) { d->dbg_gs[i] = grad[i]; d->dbg_gs[32 + i] = search[i]; }
    /* line search (MJX-style bracketing on the piecewise quadratic) */
    double Mv[NV], jv[MAXEFC], sn = 0;
    mulM(m, d, search, Mv);
    for (int r = 0; r < nefc; r++) {
      double s = 0;
      for (int i = 0; i < nv; i++) s += d->efc_J[r][i] * search[i];
      jv[r] = s;
    }
    for (int i = 0; i < nv; i++) sn += search[i] * search[i];
    double gtol = m->tolerance * m->ls_tolerance * sqrt(sn) * m->meaninertia * (nv > 1 ? nv : 1);
    double gauss = 0, q1 = 0, q2 = 0;
    for (int i = 0; i < nv; i++) {
      gauss += (Ma[i] - d->qfrc_smooth[i]) * (qacc[i] - d->qacc_smooth[i]);
      q1 += search[i] * (Ma[i] - d->qfrc_smooth[i]);
      q2 += search[i] * Mv[i];
    }
    double qg[3] = {0.5 * gauss, q1, 0.5 * q2};
    if (d->ls_dump && it == 0) {
      d->ls_dump[0] = nefc; d->ls_dump[1] = qg[0]; d->ls_dump[2] = qg[1]; d->ls_dump[3] = qg[2];
      d->ls_dump[4] = gtol;
      for (int r = 0; r < nefc && r < 512; r++) {
        double* o = d->ls_dump + 8 + 4 * r;
        o[0] = jar[r]; o[1] = jv[r]; o[2] = d->efc_D[r]; o[3] = d->efc_eq[r];
      }
    }
    lspt p0 = ls_eval(d, qg, jar, jv, 0.0);
    lspt lo = ls_eval(d, qg, jar, jv, p0.alpha - p0.d0 / p0.d1);
    lspt hi;
    if (lo.d0 < p0.d0) { hi = p0; } else { hi = lo; lo = p0; }
    int swap = 1;
    for (int ls = 0; ls < m->ls_iterations; ls++) {
      if (!swap) break;
      if (it == 0) d->dbg[5] = ls;
      if (lo.d0 < 0 && lo.d0 > -gtol) break;
      if (hi.d0 > 0 && hi.d0 < gtol) break;
      /* the kernel's bracket floor: closed to 1e-6 relative */
      if (!(g_exact & EXACT_LS) && fabs(hi.alpha - lo.alpha) <= 1e-6 * fmax(fabs(lo.alpha), fabs(hi.alpha))) break;
      lspt lo_next = ls_eval(d, qg, jar, jv, lo.alpha - lo.d0 / lo.d1);
      lspt hi_next = ls_eval(d, qg, jar, jv, hi.alpha - hi.d0 / hi.d1);
      lspt mid = ls_eval(d, qg, jar, jv, 0.5 * (lo.alpha + hi.alpha));
      int s1 = lo.d0 > 0 || lo.d0 < lo_next.d0;
      if (s1) lo = lo_next;
      int s2 = mid.d0 < 0 && lo.d0 < mid.d0;
      if (s2) lo = mid;
      int s3 = hi.d0 < 0 || hi.d0 > hi_next.d0;
      if (s3) hi = hi_next;
      int s4 = mid.d0 > 0 && hi.d0 > mid.d0;
      if (s4) hi = mid;
      swap = s1 || s2 || s3 || s4;
    }
    int improved = lo.cost < p0.cost || hi.cost < p0.cost;
    mpcr_hp alpha = lo.cost < hi.cost ? lo.alpha : hi.alpha;
    if (it == 0) { d->dbg[3] = p0.cost; d->dbg[4] = alpha; d->dbg[6] = fmin(lo.cost, hi.cost); }
    d->dbg[7] = it + 1;
    if (improved) {
      for (int i = 0; i < nv; i++) { qacc[i] += alpha * search[i]; Ma[i] += alpha * Mv[i]; }
      for (int r = 0; r < nefc; r++) jar[r] += alpha * jv[r];
    }
    prev_cost = cost;
    cost = solver_cost(m, d, qacc, Ma, jar);
  }
  memcpy(d->qacc, qacc, sizeof(double) * nv);
  /* efc_force / qfrc_constraint at the final acceleration */
  for (int i = 0; i < nv; i++) d->qfrc_constraint[i] = 0;
  efc_cost_force(d, jar, d->efc_force);
  for (int r = 0; r < nefc; r++)
    for (int i = 0; i < nv; i++) d->qfrc_constraint[i] += d->efc_J[r][i] * d->efc_force[r];
}

/* ------------------------------------------------------------------------ */
/* step = forward + Euler (mj_step with eulerdamp disabled)                   */

/* diagnostic (oracle_set_round32, tools/stage_precision.py): round the
   outputs of the masked stages to fp32 -- which stage's fp32 precision moves
   the trajectories (bits: 1 kinematics, 2 COM / cinert / cdof, 4 mass matrix,
   8 contacts, 16 velocities, 32 passive + bias + actuator forces, 64
   constraint rows, 128 qacc_smooth, 256 qacc, 512 Euler state) */
static int g_round32 = 0;
void oracle_set_round32(int mask) { g_round32 = mask; }
static void r32v(double* x, int n) {
  for (int i = 0; i < n; i++) x[i] = (double)(float)x[i];
}
#define R32(bit, arr, n) do { if (g_round32 & (bit)) r32v((double*)(arr), (n)); } while (0)

static void forward(const mpcr_model_t* m, odata* d) {
  kinematics(m, d);
  R32(1, d->xpos, 3 * m->nbody); R32(1, d->xquat, 4 * m->nbody); R32(1, d->xmat, 9 * m->nbody);
  R32(1, d->xipos, 3 * m->nbody); R32(1, d->ximat, 9 * m->nbody); R32(1, d->xanchor, 3 * m->njnt);
  R32(1, d->xaxis, 3 * m->njnt); R32(1, d->geom_xpos, 3 * m->ngeom); R32(1, d->geom_xmat, 9 * m->ngeom);
  R32(1, d->site_xpos, 3 * m->nsite);
  com_pos(m, d);
  R32(2, d->subtree_com, 3 * m->nbody); R32(2, d->cinert, 10 * m->nbody); R32(2, d->cdof, 6 * m->nv);
  crb(m, d);
  if (g_round32 & 4) {
    for (int i = 0; i < m->nv; i++) r32v(d->M[i], m->nv);
    chol(d->L, d->M, m->nv);
  }
  collision(m, d);
  if (g_round32 & 8)
    for (int c = 0; c < d->ncon; c++) { r32v(&d->con[c].dist, 1); r32v(d->con[c].pos, 3); r32v(d->con[c].frame, 9); }
  com_vel(m, d);
  R32(16, d->cvel, 6 * m->nbody); R32(16, d->cdof_dot, 6 * m->nv);
  passive(m, d);
  rne(m, d);
  actuation(m, d);
  R32(32, d->qfrc_passive, m->nv); R32(32, d->qfrc_bias, m->nv); R32(32, d->qfrc_actuator, m->nv);
  make_constraint(m, d);
  if (g_round32 & 64)
    for (int r = 0; r < d->nefc; r++) { r32v(d->efc_J[r], m->nv); r32v(&d->efc_D[r], 1); r32v(&d->efc_aref[r], 1); }
  for (int i = 0; i < m->nv; i++) d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i] + d->qfrc_actuator[i];
  chol_solve(d->qacc_smooth, d->L, d->qfrc_smooth, m->nv);
  R32(128, d->qacc_smooth, m->nv);
  solve(m, d);
  R32(256, d->qacc, m->nv);
}

static void euler(const mpcr_model_t* m, odata* d) {
  double dt = m->timestep;
  if (m->integrator == MPCR_INT_IMPLICITFAST) {
    /* mj_implicitSkip: (M - dt qDeriv) qacc_i = qfrc_smooth + qfrc_constraint */
    double D[NV][NV], A[NV][NV], L[NV][NV], f[NV] = {0}, acc[NV];
    qderiv(m, D);
    for (int i = 0; i < m->nv; i++) {
      for (int j = 0; j < m->nv; j++) A[i][j] = d->M[i][j] - dt * D[i][j];
      f[i] = d->qfrc_smooth[i] + d->qfrc_constraint[i];
    }
    chol(L, A, m->nv);
    chol_solve(acc, L, f, m->nv);
    for (int i = 0; i < m->nv; i++) d->qvel[i] += dt * acc[i];
  } else {
    for (int i = 0; i < m->nv; i++) d->qvel[i] += dt * d->qacc[i];
  }
  for (int j = 0; j < m->njnt; j++) {
    int a = m->jnt_qposadr[j], v = m->jnt_dofadr[j];
    if (m->jnt_type[j] == MPCR_JNT_FREE) {
      for (int k = 0; k < 3; k++) d->qpos[a + k] += dt * d->qvel[v + k];
      a += 3; v += 3;
    }
    if (m->jnt_type[j] == MPCR_JNT_FREE || m->jnt_type[j] == MPCR_JNT_BALL) {
      /* mju_quatIntegrate: q <- q * exp(omega_local * dt) */
      double w[3] = {d->qvel[v], d->qvel[v + 1], d->qvel[v + 2]};
      double ang = norm3(w) * dt;
      double* q = d->qpos + a;
      if (ang > MINVAL) {
        double ax[3] = {w[0] * dt / ang, w[1] * dt / ang, w[2] * dt / ang}, dq[4];
        axisangle(dq, ax, ang);
        qmul(q, q, dq);
      }
      qnorm(q);
    } else {
      d->qpos[a] += dt * d->qvel[v];
    }
  }
  memcpy(d->qacc_warmstart, d->qacc, sizeof(double) * m->nv);
  R32(512, d->qpos, m->nq); R32(512, d->qvel, m->nv); R32(512, d->qacc_warmstart, m->nv);
}

/* ------------------------------------------------------------------------ */
/* exported API (ctypes)                                                      */

int oracle_model_size(void) { return (int)sizeof(mpcr_model_t); }
int oracle_data_size(void) { return (int)sizeof(odata); }

/* One mj_step from (qpos, qvel, qacc_warmstart), all updated in place.
   Optional outputs (NULL to skip): M (nv x nv), qfrc_bias, qfrc_passive,
   qacc (the solved acceleration), eef (7: tcp xpos, hande xquat, pre-step),
   dist (ncon slot distances, pre-step), nefc. */
int oracle_step(const mpcr_model_t* m, double* qpos, double* qvel, double* qacc_ws, double* M_out,
                double* bias_out, double* passive_out, double* qacc_out, double* eef_out, double* dist_out,
                int* nefc_out) {
  odata* d = (odata*)calloc(1, sizeof(odata));
  use_model(m);
  if (!d) return -1;
  memcpy(d->qpos, qpos, sizeof(double) * m->nq);
  memcpy(d->qvel, qvel, sizeof(double) * m->nv);
  memcpy(d->qacc_warmstart, qacc_ws, sizeof(double) * m->nv);
  reset_hints(d);
  forward(m, d);
  if (M_out)
    for (int i = 0; i < m->nv; i++)
      for (int j = 0; j < m->nv; j++) M_out[i * m->nv + j] = d->M[i][j];
  if (bias_out) memcpy(bias_out, d->qfrc_bias, sizeof(double) * m->nv);
  if (passive_out) memcpy(passive_out, d->qfrc_passive, sizeof(double) * m->nv);
  if (qacc_out) memcpy(qacc_out, d->qacc, sizeof(double) * m->nv);
  if (eef_out) {
    if (m->tcp_site >= 0) memcpy(eef_out, d->site_xpos[m->tcp_site], 3 * sizeof(double));
    if (m->hande_body >= 0) memcpy(eef_out + 3, d->xquat[m->hande_body], 4 * sizeof(double));
  }
  if (dist_out)
    for (int c = 0; c < m->ncon; c++) dist_out[c] = d->con[c].dist;
  if (nefc_out) *nefc_out = d->nefc;
  euler(m, d);
  memcpy(qpos, d->qpos, sizeof(double) * m->nq);
  memcpy(qvel, d->qvel, sizeof(double) * m->nv);
  memcpy(qacc_ws, d->qacc_warmstart, sizeof(double) * m->nv);
  int trunc = d->efc_trunc;
  free(d);
  return trunc ? 1 : 0;
}

/* parity debugging: world geom poses at qpos (xpos 3, xmat 9 per geom) and
   the oracle's MPR on one pair (out: hit, depth, dir 3, pos 3) */
int oracle_geom_poses(const mpcr_model_t* m, const double* qpos, double* xpos, double* xmat, int pair,
                      double* mpr_out) {
  odata* d = (odata*)calloc(1, sizeof(odata));
  use_model(m);
  if (!d) return -1;
  memcpy(d->qpos, qpos, sizeof(double) * m->nq);
  reset_hints(d);
  kinematics(m, d);
  for (int g = 0; g < m->ngeom; g++) {
    memcpy(xpos + 3 * g, d->geom_xpos[g], 3 * sizeof(double));
    memcpy(xmat + 9 * g, d->geom_xmat[g], 9 * sizeof(double));
  }
  if (pair >= 0 && mpr_out) {
    double depth = 0, dir[3] = {0, 0, 0}, pos[3] = {0, 0, 0};
    mpr_out[0] = mpr(m, d, m->pair_geom1[pair], m->pair_geom2[pair], &depth, dir, pos, d->hint[pair]);
    mpr_out[1] = depth;
    memcpy(mpr_out + 2, dir, sizeof(dir));
    memcpy(mpr_out + 5, pos, sizeof(pos));
  }
  free(d);
  return 0;
}

/* uniform in [-1, 1) from (seed, candidate, step, index): splitmix64 */
static double hash_unit(unsigned seed, int b, int t, int i) {
  uint64_t z = ((uint64_t)seed << 40) ^ ((uint64_t)(unsigned)b << 20) ^ ((uint64_t)(unsigned)t << 8) ^ (uint64_t)i;
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

/* parity debugging: one step like oracle_step, dumping the active contacts,
   the constraint rows, qacc_smooth and qacc in the kernel's DBG_* layout
   (manipulator_mujoco_amd/csrc/rollout.h: 48 contacts, 200 rows; 1234
   doubles) */
enum { ODBG_MAXCON = 48, ODBG_ROW = 2 + 8 * ODBG_MAXCON, ODBG_MAXROW = 200, ODBG_QAS = ODBG_ROW + 3 * ODBG_MAXROW,
       ODBG_QACC = ODBG_QAS + 32, ODBG_INFO = ODBG_QACC + 32, ODBG_N = ODBG_INFO + 8 + 64 + 112 };
int oracle_step_debug(const mpcr_model_t* m, const double* qpos, const double* qvel, const double* qacc_ws,
                      double* out) {
  odata* d = (odata*)calloc(1, sizeof(odata));
  use_model(m);
  if (!d) return -1;
  memcpy(d->qpos, qpos, sizeof(double) * m->nq);
  memcpy(d->qvel, qvel, sizeof(double) * m->nv);
  memcpy(d->qacc_warmstart, qacc_ws, sizeof(double) * m->nv);
  reset_hints(d);
  forward(m, d);
  memset(out, 0, sizeof(double) * ODBG_N);
  memcpy(out + ODBG_INFO, d->dbg, sizeof(d->dbg));
  memcpy(out + ODBG_INFO + 8, d->dbg_gs, sizeof(d->dbg_gs));
  int na = 0;
  for (int c = 0; c < d->ncon; c++) {
    const ocontact* k = &d->con[c];
    if (!k->active) continue;
    if (na < ODBG_MAXCON) {
      double* o = out + 2 + 8 * na;
      memcpy(o, k->pos, 3 * sizeof(double));
      o[3] = k->dist; o[4] = k->pair;
      o[5] = k->frame[0]; o[6] = k->frame[1]; o[7] = k->frame[2];
    }
    na++;
  }
  out[0] = na;
  out[1] = d->nefc;
  for (int r = 0; r < d->nefc && r < ODBG_MAXROW; r++) {
    out[ODBG_ROW + 3 * r] = d->efc_D[r];
    out[ODBG_ROW + 3 * r + 1] = d->efc_aref[r];
    out[ODBG_ROW + 3 * r + 2] = d->efc_vel[r];
  }
  memcpy(out + ODBG_QAS, d->qacc_smooth, sizeof(double) * m->nv);
  memcpy(out + ODBG_QACC, d->qacc, sizeof(double) * m->nv);
  free(d);
  return 0;
}

/* parity debugging: the inputs of the step's first Newton line search:
   out[0] nefc, out[1..3] the Gauss quadratic (q0, q1, q2), out[4] gtol,
   out[8 + 4 r ..] (jar, jv, D, efc_eq) per row, then the Newton Hessian nv x nv
   (8 + 4 * 512 + 32 * 32 doubles) */
int oracle_ls_inputs(const mpcr_model_t* m, const double* qpos, const double* qvel, const double* qacc_ws,
                     double* out) {
  odata* d = (odata*)calloc(1, sizeof(odata));
  use_model(m);
  if (!d) return -1;
  memcpy(d->qpos, qpos, sizeof(double) * m->nq);
  memcpy(d->qvel, qvel, sizeof(double) * m->nv);
  memcpy(d->qacc_warmstart, qacc_ws, sizeof(double) * m->nv);
  reset_hints(d);
  d->ls_dump = out;
  forward(m, d);
  free(d);
  return 0;
}

/* Rollout + cost for n candidates (compute_rollout_single +
   compute_cost_single, SBP/mjx_planner.py:265-303).
     thetadot : n x (nctrl*H), joint-major (A_thetadot @ xi, :348)
     q0       : nctrl initial joint positions
     w        : (w_pos, w_rot, w_col);  ptgt (3), qtgt (4, wxyz)
   outputs:
     cost4    : n x 4 (cost, cost_g, cost_r, cost_c)
     theta    : n x (nctrl*H) joint-major post-step qpos (nullable)
     slots    : n x H x nslot masked contact distances (nullable)
     eef      : n x H x 7 (tcp pos, hande quat) (nullable)
     info     : n x 3 ints (busiest step's rows, its active contacts, and
                the integer #{c < 0} term of cost_c, SBP/mjx_planner.py:296) */
int oracle_rollout(const mpcr_model_t* m, int n, int H, const double* thetadot, const double* q0,
                   const double* w, const double* ptgt, const double* qtgt, double* cost4, double* theta,
                   double* slots, double* eef, int* info, double noise, unsigned seed,
                   int index_base) {
  if (m->magic != MPCR_MODEL_MAGIC || m->nbytes != sizeof(mpcr_model_t)) return -2;
  odata* d = (odata*)calloc(1, sizeof(odata));
  use_model(m);
  double* cprev = (double*)calloc(m->nslot > 0 ? m->nslot : 1, sizeof(double));
  if (!d || !cprev) { free(d); free(cprev); return -1; }
  int nc = m->nctrl, status = 0;
  double qt[4];
  memcpy(qt, qtgt, sizeof(qt));
  double qtn = sqrt(qt[0] * qt[0] + qt[1] * qt[1] + qt[2] * qt[2] + qt[3] * qt[3]);
  for (int k = 0; k < 4; k++) qt[k] /= qtn;
  for (int b = 0; b < n; b++) {
    memset(d, 0, sizeof(odata));
    reset_hints(d);
    memcpy(d->qpos, m->qpos_init, sizeof(double) * m->nq);
    memcpy(d->qvel, m->qvel_init, sizeof(double) * m->nv);
    for (int j = 0; j < nc; j++) d->qpos[m->ctrl_qposadr[j]] = q0[j];
    double cg = 0, cr = 0, cc = 0;
    int maxrows = 0, maxact = 0, nneg = 0;
    const double* td = thetadot + (size_t)b * nc * H;
    for (int t = 0; t < H; t++) {
      for (int j = 0; j < nc; j++) d->qvel[m->ctrl_dofadr[j]] = td[j * H + t];
      forward(m, d);
      if (d->efc_trunc) status = 1;
      if (d->nefc > maxrows) maxrows = d->nefc;
      {
        int na = 0;
        for (int c = 0; c < m->ncon; c++) na += d->con[c].active;
        if (na > maxact) maxact = na;
      }
      /* eef pose and collision distances: pre-integration (from forward) */
      const double* p = m->tcp_site >= 0 ? d->site_xpos[m->tcp_site] : d->xpos[0];
      const double* q = m->hande_body >= 0 ? d->xquat[m->hande_body] : d->xquat[0];
      double dp[3] = {p[0] - ptgt[0], p[1] - ptgt[1], p[2] - ptgt[2]};
      cg += norm3(dp);
      double qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
      double dotq = fabs((q[0] * qt[0] + q[1] * qt[1] + q[2] * qt[2] + q[3] * qt[3]) / qn);
      cr += 2 * acos(clampd(dotq, -1, 1));
      if (eef) {
        double* e = eef + ((size_t)b * H + t) * 7;
        memcpy(e, p, 3 * sizeof(double));
        memcpy(e + 3, q, 4 * sizeof(double));
      }
      for (int pi = 0; pi < m->npair; pi++) {
        int sa = m->pair_slotadr[pi];
        if (sa < 0) continue;
        for (int s = 0; s < m->pair_ncon[pi]; s++) {
          double c = d->con[m->pair_conadr[pi] + s].dist;
          if (slots) slots[((size_t)b * H + t) * m->nslot + sa + s] = c;
          if (c < 0) { cc += 1; nneg++; }
          if (t > 0) {
            double g = cprev[sa + s] * (1 - 0.005) - c; /* y = 0.005, :287-291 */
            if (g > 0) cc += g;
          }
          cprev[sa + s] = c;
        }
      }
      euler(m, d);
      if (noise > 0) { /* conditioning probe: per-step relative state noise (tests/parity_util.py) */
        for (int i = 0; i < m->nq; i++) d->qpos[i] *= 1 + noise * hash_unit(seed, index_base + b, t, i);
        for (int i = 0; i < m->nv; i++) {
          d->qvel[i] *= 1 + noise * hash_unit(seed, index_base + b, t, 64 + i);
          d->qacc_warmstart[i] *= 1 + noise * hash_unit(seed, index_base + b, t, 128 + i);
        }
      }
      if (theta)
        for (int j = 0; j < nc; j++) theta[(size_t)b * nc * H + j * H + t] = d->qpos[m->ctrl_qposadr[j]];
    }
    cost4[4 * b + 0] = w[0] * cg + w[1] * cr + w[2] * cc;
    cost4[4 * b + 1] = cg;
    cost4[4 * b + 2] = cr;
    cost4[4 * b + 3] = cc;
    if (info) { info[3 * b] = maxrows; info[3 * b + 1] = maxact; info[3 * b + 2] = nneg; }
  }
  free(cprev);
  free(d);
  return status;
}

/* test hook: the elliptic cone of one condim-3 contact (rows 0..2) at jar, and
   its line function along jar + alpha jv (cost, d/dalpha, d2/dalpha2) */
int oracle_cone_eval(double mu, const double fri[2], const double D[3], const double jar[3], const double jv[3],
                     double alpha, double* cost, double f[3], double H[9], double line[3]) {
  odata* d = (odata*)calloc(1, sizeof(odata));
  if (!d) return -1;
  d->nefc = 3;
  for (int k = 0; k < 3; k++) {
    d->efc_eq[k] = k == 0 ? 2 : 3;
    d->efc_D[k] = D[k];
  }
  d->efc_dim[0] = 3;
  d->efc_mu[0] = mu;
  d->efc_fri[0][0] = fri[0];
  d->efc_fri[0][1] = fri[1];
  double Hc[3][3];
  *cost = ell_update(d, 0, jar, f, Hc);
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) H[3 * a + b] = Hc[a][b];
  ell_line(d, 0, jar, jv, alpha, line);
  free(d);
  return 0;
}

/* crash diagnostics (test infrastructure, MPCR_ORACLE_CRASH_BT=1 in oracle.lib()):
   print the C backtrace of a fault in the oracle, then die with the signal */
static void oracle_crash_bt(int sig) {
  void* buf[64];
  const int n = backtrace(buf, 64);
  static const char msg[] = "oracle: fatal signal, C backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(buf, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
void oracle_install_crash_bt(void) {
  signal(SIGSEGV, oracle_crash_bt);
  signal(SIGILL, oracle_crash_bt);
  signal(SIGBUS, oracle_crash_bt);
}



/* the experiment above (ORACLE_CAPS_SAT): capsule / cylinder against a
   polyhedron (mesh hull or box with face tables), relative to the
   polyhedron's centre; the face with the largest separation (lowest index
   within the near_max band) carries one contact, unless it is more than 5 %
   (+10 um) deeper than MPR's depth (an edge axis: MPR's point stays) */
static int caps_poly(const mpcr_model_t* m, odata* d, int g1, int g2, double depth, ocontact* out) {
  const int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const int round1 = t1 == MPCR_GEOM_CAPSULE || t1 == MPCR_GEOM_CYLINDER;
  const int round2 = t2 == MPCR_GEOM_CAPSULE || t2 == MPCR_GEOM_CYLINDER;
  const int poly1 = (t1 == MPCR_GEOM_MESH || t1 == MPCR_GEOM_BOX) && m->geom_faceadr[g1] >= 0;
  const int poly2 = (t2 == MPCR_GEOM_MESH || t2 == MPCR_GEOM_BOX) && m->geom_faceadr[g2] >= 0;
  int gc, gp;
  if (round1 && poly2) { gc = g1; gp = g2; }
  else if (round2 && poly1) { gc = g2; gp = g1; }
  else return 0;
  const int nf = m->geom_facenum[gp], fa = m->geom_faceadr[gp];
  if (nf <= 0 || nf > POLY_ALLF) return 0;
  const double* cg = d->geom_xpos[gp];
  const double* Rc = d->geom_xmat[gc];
  const double ax[3] = {Rc[2], Rc[5], Rc[8]};
  const double r = m->geom_size[gc][0], hl = m->geom_size[gc][1];
  const double cc[3] = {d->geom_xpos[gc][0] - cg[0], d->geom_xpos[gc][1] - cg[1], d->geom_xpos[gc][2] - cg[2]};
  const int cyl = m->geom_type[gc] == MPCR_GEOM_CYLINDER;
  double sep[POLY_ALLF], mx = -1e300;
  for (int k = 0; k < nf; k++) {
    double nw[3], off;
    face_world(m, d, gp, fa + k, nw, &off, cg);
    const double na = dot3(nw, ax);
    /* the round geom's support along -nw: its deepest point into the face plane */
    double lo = dot3(nw, cc) - hl * fabs(na);
    lo -= cyl ? r * sqrt(fmax(0.0, 1.0 - na * na)) : r;
    sep[k] = lo - off;
    if (sep[k] > mx) mx = sep[k];
  }
  int bf = -1;
  for (int k = 0; k < nf && bf < 0; k++)
    if (near_max(sep[k], mx)) bf = k;
  if (bf < 0 || sep[bf] < -depth * 1.05 - 1e-5) return 0;
  double nw[3], off;
  face_world(m, d, gp, fa + bf, nw, &off, cg);
  const double na = dot3(nw, ax);
  /* the deepest point of the round geom (an end, or the nearer end's rim) */
  const double sa = na > 0 ? -1.0 : (na < 0 ? 1.0 : 0.0);
  double e[3], rim[3] = {0, 0, 0};
  for (int k = 0; k < 3; k++) e[k] = cc[k] + sa * hl * ax[k];
  if (cyl) {
    double t[3];
    for (int k = 0; k < 3; k++) t[k] = nw[k] - na * ax[k];
    const double tl = norm3(t);
    if (tl > 1e-12) for (int k = 0; k < 3; k++) rim[k] = -r * t[k] / tl;
  } else {
    for (int k = 0; k < 3; k++) rim[k] = -r * nw[k];
  }
  const double dist = sep[bf];
  double pos[3], n[3];
  for (int k = 0; k < 3; k++) {
    pos[k] = e[k] + rim[k] - 0.5 * dist * nw[k] + cg[k];
    n[k] = gp == g2 ? -nw[k] : nw[k]; /* geom1 -> geom2 */
  }
  set_contact(out, dist, pos, n);
  return 1;
}

/*
 * oracle_physics.c — fp64 CPU restatement of the build's physics step
 * (gym.simulate counterpart).  TEST
 * INFRASTRUCTURE ONLY: linked by tests/ and bench.py's cpu_baseline leg.
 *
 * PARITY UNPINNED vs the reference: the reference physics is the closed
 * isaacgym/PhysX binary.  This file restates the algorithm documented in
 * DESIGN.md §Physics using an independent formulation from the HIP kernels:
 *
 *   - spatial vectors expressed at one point o per actor (the root origin at
 *     the start of the substep), world-aligned; motion = [w; v], force = [n; f]
 *   - composite-rigid-body algorithm for the joint-space inertia M, RNEA for the
 *     bias C(q, v), dense Cholesky for M~^-1 (GPU: articulated-body recursion)
 *   - implicit joint damping/stiffness: M~ = M + diag(armature + h b + h^2 k),
 *     tau = tau_act - b qd - k (q + h qd)
 *   - velocity-level PGS with speculative contacts: rows in the order
 *     [contact: normal, t1, t2]* then joint limits [lower, upper] per DOF;
 *     pos_iters sweeps (physx.num_position_iterations, Ant.yaml:53)
 *   - semi-implicit Euler; root quaternion by the exact exponential map
 *   - hand tasks (SURVEY.md §8(a) A4-A8 for ShadowHand): PD position drives
 *     (implicit spring/damper toward the target; an explicit +-effort force
 *     when the explicit estimate saturates), fixed tendons as explicit
 *     soft-limit springs + dampers, and one free rigid box per env whose
 *     6 velocity columns [w; v_com] join the articulation's in one
 *     block-diagonal system (contacts couple them)
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* Scalar type of the physics restatement: fp64 for the checker (default).  -DORC_FP32 builds the
 * fp32 variant that bench.py times as the CPU baseline (liboracle_f32.so), with the float libm. */
#ifdef ORC_FP32
typedef float real;
#define sqrt sqrtf
#define fabs fabsf
#define fmin fminf
#define sin sinf
#define cos cosf
#define tanh tanhf
#else
typedef double real;
#endif

#include "oracle.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXN MG_MAX_NODES
#define MAXV (MG_MAX_NODES + 12)
#define OBJ_NODE (-2) /* contact side on the free object */
#define MAXC 64
#define MAXR (3 * MAXC + 2 * MG_MAX_NODES)
#define MPR_TOL 1e-7  /* portal reached the boundary (m) */
#define CVX_MARGIN 1e-3 /* rounding of box cores against the egg (m) */
#define BOX_BLEND 1e-3  /* point_box: the band (m) over which an interior point's normal blends faces */
#define MPR_EPS 1e-12 /* origin-side tests */
/* the explicit MJCF pairs' contact threshold (0: MuJoCo margin 0); moved only by orc_step_flips */
static __thread double orc_pair_offset = 0.0;
/* orc_step_flips: seg_box_sat reports a tie of its two least push-out faces within orc_tie_delta */
static __thread double orc_tie_delta = -1.0;
static __thread int orc_tie_hit = 0;
/* orc_step_flips: a narrowphase decision within its tolerance band of the threshold (bit 16), and the contact
 * being pushed has an ill-conditioned normal (bit 32: the direction of a core distance below NORMAL_ILL that
 * the geometry does not pin -- an end point or a box edge / corner at the closest point) */
static __thread int orc_amb_hit = 0;  /* bit 16 for the whole step (an ambiguous decision that made no contact) */
static __thread int orc_amb_pend = 0; /* an ambiguous decision in the current geom-object candidate set */
static __thread int orc_ill_next = 0;
static __thread int orc_pb_ill = 0;   /* the last point_box: outside, two or more axes clamped, nearer than NORMAL_ILL */
static __thread int orc_cvx_ill = 0;  /* the last cvx_contact: an MPR depth below NORMAL_ILL */
static __thread int orc_hull_ill = 0; /* the last hull_core_contacts: a GJK distance below NORMAL_ILL */
#define NORMAL_ILL 5e-4
/* orc_step_flips bit 64: the angular-velocity cap clipped a hinge rate to an interval end whose fp32 value is
 * ill-conditioned: disc = b^2 - |w_p|^2 + W^2 carries the rounding of W^2-sized terms (~2 eps32 W^2), so the end
 * point -b +- sqrt(disc) is off by ~eps32 W^2 / sq; flagged when that exceeds CAP_ILL_TOL (rad/s) */
static __thread int orc_cap_hit = 0;
#define CAP_ILL_TOL 1e-3
/* the hull narrowphase's decision thresholds, scaled by orc_step_flips' variants (1 = the build's) */
static __thread struct { double fe, ang, cop; int seam, face; double marg; } orc_hv = {1.0, 1.0, 1.0, 0, -1, 0.0};

typedef real v3[3];

/* ---------------------------------------------------------------- small math */
static void cross3(const real* a, const real* b, real* o) {
  real x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
static real dot3(const real* a, const real* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void quat_to_mat(const real* q, real R[3][3]) {
  real x = q[0], y = q[1], z = q[2], w = q[3];
  R[0][0] = 1 - 2 * (y * y + z * z); R[0][1] = 2 * (x * y - z * w); R[0][2] = 2 * (x * z + y * w);
  R[1][0] = 2 * (x * y + z * w); R[1][1] = 1 - 2 * (x * x + z * z); R[1][2] = 2 * (y * z - x * w);
  R[2][0] = 2 * (x * z - y * w); R[2][1] = 2 * (y * z + x * w); R[2][2] = 1 - 2 * (x * x + y * y);
}
static void mat_to_quat(real R[3][3], real* q) {
  real tr = R[0][0] + R[1][1] + R[2][2];
  if (tr > 0) {
    real s = sqrt(tr + 1.0) * 2;
    q[3] = 0.25 * s; q[0] = (R[2][1] - R[1][2]) / s; q[1] = (R[0][2] - R[2][0]) / s; q[2] = (R[1][0] - R[0][1]) / s;
  } else if (R[0][0] > R[1][1] && R[0][0] > R[2][2]) {
    real s = sqrt(1.0 + R[0][0] - R[1][1] - R[2][2]) * 2;
    q[3] = (R[2][1] - R[1][2]) / s; q[0] = 0.25 * s; q[1] = (R[0][1] + R[1][0]) / s; q[2] = (R[0][2] + R[2][0]) / s;
  } else if (R[1][1] > R[2][2]) {
    real s = sqrt(1.0 + R[1][1] - R[0][0] - R[2][2]) * 2;
    q[3] = (R[0][2] - R[2][0]) / s; q[0] = (R[0][1] + R[1][0]) / s; q[1] = 0.25 * s; q[2] = (R[1][2] + R[2][1]) / s;
  } else {
    real s = sqrt(1.0 + R[2][2] - R[0][0] - R[1][1]) * 2;
    q[3] = (R[1][0] - R[0][1]) / s; q[0] = (R[0][2] + R[2][0]) / s; q[1] = (R[1][2] + R[2][1]) / s; q[2] = 0.25 * s;
  }
}
static void matmul3(real A[3][3], real B[3][3], real C[3][3]) {
  real T[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) T[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
  memcpy(C, T, sizeof(T));
}
static void matvec3(real A[3][3], const real* v, real* o) {
  real x = A[0][0] * v[0] + A[0][1] * v[1] + A[0][2] * v[2];
  real y = A[1][0] * v[0] + A[1][1] * v[1] + A[1][2] * v[2];
  real z = A[2][0] * v[0] + A[2][1] * v[1] + A[2][2] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
static void mattvec3(real A[3][3], const real* v, real* o) {
  real x = A[0][0] * v[0] + A[1][0] * v[1] + A[2][0] * v[2];
  real y = A[0][1] * v[0] + A[1][1] * v[1] + A[2][1] * v[2];
  real z = A[0][2] * v[0] + A[1][2] * v[1] + A[2][2] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
static void axis_angle_mat(const real* a, real ang, real R[3][3]) {
  real c = cos(ang), s = sin(ang), t = 1 - c, x = a[0], y = a[1], z = a[2];
  R[0][0] = t * x * x + c; R[0][1] = t * x * y - s * z; R[0][2] = t * x * z + s * y;
  R[1][0] = t * x * y + s * z; R[1][1] = t * y * y + c; R[1][2] = t * y * z - s * x;
  R[2][0] = t * x * z - s * y; R[2][1] = t * y * z + s * x; R[2][2] = t * z * z + c;
}
static void quat_mul_d(const real* a, const real* b, real* o) {
  real x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  real y = a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0];
  real z = a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3];
  real w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}

/* spatial algebra (6-vectors: angular first) */
static void crm(const real* v, const real* m, real* o) { /* v x m (motion) */
  real a[3], b[3], c[3];
  cross3(v, m, a);
  cross3(v, m + 3, b);
  cross3(v + 3, m, c);
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2];
  o[3] = b[0] + c[0]; o[4] = b[1] + c[1]; o[5] = b[2] + c[2];
}
static void crf(const real* v, const real* f, real* o) { /* v x* f (force) */
  real a[3], b[3], c[3];
  cross3(v, f, a);
  cross3(v + 3, f + 3, b);
  cross3(v, f + 3, c);
  o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2];
  o[3] = c[0]; o[4] = c[1]; o[5] = c[2];
}
static real dot6(const real* a, const real* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
static void mat6vec(real I[6][6], const real* v, real* o) {
  for (int i = 0; i < 6; i++) {
    real s = 0;
    for (int j = 0; j < 6; j++) s += I[i][j] * v[j];
    o[i] = s;
  }
}

/* ---------------------------------------------------------------- per-actor state */
typedef struct {
  real p[3], q[4];     /* root pose */
  real nu0[6];         /* root spatial velocity at root origin [w; v_o] */
  real qj[MAXN], qd[MAXN];
  real op[3], oq[4];   /* free object pose (COM = origin) */
  real ow[3], ov[3];   /* object angular / COM linear velocity (world) */
  real of[3];          /* applied force on the object COM (apply_rigid_body_force_tensors) */
  int of_local;          /* LOCAL_SPACE: of is in the object frame at the start of each substep */
  const real* gmu;     /* DR: friction per geom, [num_geoms] = the object's; NULL = sim friction */
  const float* tgt;      /* PD targets (nD) or NULL */
  int sat[MAXN];         /* drive saturated in the last substep */
  real ttend[MAXN];    /* tendon generalized force of the last substep */
} astate;

typedef struct {
  real R[MAXN][3][3], x[MAXN][3];
  real S[MAXN][6];
  real I[MAXN][6][6];
  real Iw[MAXN][3][3]; /* rotational inertia about the COM, world axes (link damping) */
  real V[MAXN][6];
  real o[3];
  real oR[3][3], op[3]; /* free object pose */
} kin;

typedef struct {
  int nodeA, nodeB, geomA, geomB;
  real p[3], n[3], d;
  int ill;   /* ill-conditioned normal (orc_step_flips bit 32) */
  int amb;   /* made by a geom-object candidate set with a decision in its ambiguity band (bit 16) */
} contact;

static int nv_of(const mg_model* m) { return (m->fixed_base ? 0 : 6) + m->num_dofs; }
static int nvt_of(const mg_model* m) { return nv_of(m) + (m->obj_type ? 6 : 0); } /* + object columns */
static int dof_col(const mg_model* m, int node) { return (m->fixed_base ? 0 : 6) + node - 1; }

static void load_state(const mg_model* m, const float* root, const float* dof, astate* s) {
  for (int k = 0; k < 3; k++) s->p[k] = root[k];
  real nq = 0;
  for (int k = 0; k < 4; k++) { s->q[k] = root[3 + k]; nq += s->q[k] * s->q[k]; }
  nq = sqrt(nq);
  for (int k = 0; k < 4; k++) s->q[k] /= nq;
  memset(s->nu0, 0, sizeof(s->nu0));
  if (!m->fixed_base) {
    real R[3][3], cw[3], wxc[3];
    quat_to_mat(s->q, R);
    real c[3] = {m->body_com[0][0], m->body_com[0][1], m->body_com[0][2]};
    matvec3(R, c, cw);
    real w[3] = {root[10], root[11], root[12]};
    cross3(w, cw, wxc);
    for (int k = 0; k < 3; k++) { s->nu0[k] = w[k]; s->nu0[3 + k] = root[7 + k] - wxc[k]; }
  }
  for (int i = 1; i < m->num_nodes; i++) { s->qj[i] = dof[2 * (i - 1)]; s->qd[i] = dof[2 * (i - 1) + 1]; }
}

static void store_state(const mg_model* m, const astate* s, float* root, float* dof) {
  if (!m->fixed_base) {
    real R[3][3], cw[3], wxc[3];
    quat_to_mat(s->q, R);
    real c[3] = {m->body_com[0][0], m->body_com[0][1], m->body_com[0][2]};
    matvec3(R, c, cw);
    cross3(s->nu0, cw, wxc);
    for (int k = 0; k < 3; k++) {
      root[k] = (float)s->p[k];
      root[7 + k] = (float)(s->nu0[3 + k] + wxc[k]);
      root[10 + k] = (float)s->nu0[k];
    }
    for (int k = 0; k < 4; k++) root[3 + k] = (float)s->q[k];
  }
  for (int i = 1; i < m->num_nodes; i++) {
    dof[2 * (i - 1)] = (float)s->qj[i];
    dof[2 * (i - 1) + 1] = (float)s->qd[i];
  }
}

static void forward_kinematics(const mg_model* m, const astate* s, kin* k) {
  quat_to_mat(s->q, k->R[0]);
  for (int c = 0; c < 3; c++) { k->x[0][c] = s->p[c]; k->o[c] = s->p[c]; }
  for (int i = 1; i < m->num_nodes; i++) {
    int par = m->parent[i];
    real r0[4] = {m->r0[i][0], m->r0[i][1], m->r0[i][2], m->r0[i][3]};
    real R0[3][3], Rp0[3][3], tp[3];
    quat_to_mat(r0, R0);
    matmul3(k->R[par], R0, Rp0);
    real t[3] = {m->t[i][0], m->t[i][1], m->t[i][2]};
    matvec3(k->R[par], t, tp);
    real ax[3] = {m->axis[i][0], m->axis[i][1], m->axis[i][2]};
    if (m->jtype[i] == MG_JT_HINGE) {
      real Rj[3][3];
      axis_angle_mat(ax, s->qj[i], Rj);
      matmul3(Rp0, Rj, k->R[i]);
      for (int c = 0; c < 3; c++) k->x[i][c] = k->x[par][c] + tp[c];
    } else {
      real sw[3];
      memcpy(k->R[i], Rp0, sizeof(Rp0));
      matvec3(Rp0, ax, sw);
      for (int c = 0; c < 3; c++) k->x[i][c] = k->x[par][c] + tp[c] + sw[c] * s->qj[i];
    }
  }
  /* motion subspaces at o */
  for (int i = 1; i < m->num_nodes; i++) {
    real ax[3] = {m->axis[i][0], m->axis[i][1], m->axis[i][2]}, sw[3], r[3], rxs[3];
    matvec3(k->R[i], ax, sw);
    if (m->jtype[i] == MG_JT_HINGE) {
      for (int c = 0; c < 3; c++) r[c] = k->x[i][c] - k->o[c];
      cross3(r, sw, rxs);
      for (int c = 0; c < 3; c++) { k->S[i][c] = sw[c]; k->S[i][3 + c] = rxs[c]; }
    } else {
      for (int c = 0; c < 3; c++) { k->S[i][c] = 0; k->S[i][3 + c] = sw[c]; }
    }
  }
  /* spatial inertias at o */
  for (int i = 0; i < m->num_nodes; i++) {
    real mass = m->mass[i];
    real cl[3] = {m->com[i][0], m->com[i][1], m->com[i][2]}, cw[3], c[3];
    matvec3(k->R[i], cl, cw);
    for (int a = 0; a < 3; a++) c[a] = k->x[i][a] + cw[a] - k->o[a];
    const float* in = m->inertia[i];
    real Il[3][3] = {{in[0], in[3], in[4]}, {in[3], in[1], in[5]}, {in[4], in[5], in[2]}};
    real T[3][3], Iw[3][3], Rt[3][3];
    matmul3(k->R[i], Il, T);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) Rt[a][b] = k->R[i][b][a];
    matmul3(T, Rt, Iw);
    memcpy(k->Iw[i], Iw, sizeof(Iw));
    real cc = dot3(c, c);
    real cx[3][3] = {{0, -c[2], c[1]}, {c[2], 0, -c[0]}, {-c[1], c[0], 0}};
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        k->I[i][a][b] = Iw[a][b] + mass * ((a == b ? cc : 0.0) - c[a] * c[b]);
        k->I[i][a][3 + b] = mass * cx[a][b];
        k->I[i][3 + a][b] = mass * cx[b][a];
        k->I[i][3 + a][3 + b] = (a == b) ? mass : 0.0;
      }
  }
  if (m->obj_type) {
    quat_to_mat(s->oq, k->oR);
    for (int c = 0; c < 3; c++) k->op[c] = s->op[c];
  }
  /* velocities */
  for (int c = 0; c < 6; c++) k->V[0][c] = m->fixed_base ? 0.0 : s->nu0[c];
  for (int i = 1; i < m->num_nodes; i++)
    for (int c = 0; c < 6; c++) k->V[i][c] = k->V[m->parent[i]][c] + k->S[i][c] * s->qd[i];
}

/* per-DOF implicit spring/damper of the substep: tau = tadd - b qd - k (q - ref + h qd),
 * diagonal += armature + h b + h^2 k.  Drives (drive_kp > 0): k = kp toward the target, b = joint
 * damping, unless the explicit estimate kp (tgt - q) - b qd exceeds the effort limit: then a constant
 * +-limit force and no implicit terms (PhysX clamps the drive force, shadow_hand.py:241-242). */
typedef struct {
  real k, b, ref, tadd;
  int sat;
} dofterm;

static dofterm dof_term(const mg_model* m, const astate* s, int i) {
  dofterm t = {m->stiffness[i], m->damping[i], 0.0, 0.0, 0};
  real kp = m->drive_kp[i];
  if (kp > 0.0) {
    real tgt = s->tgt ? s->tgt[i - 1] : 0.0;
    real fe = kp * (tgt - s->qj[i]) - m->damping[i] * s->qd[i];
    real F = m->effort_limit[i];
    if (fabs(fe) > F) {
      t.k = 0.0; t.b = 0.0; t.tadd = fe > 0 ? F : -F; t.sat = 1;
    } else {
      t.k = kp; t.ref = tgt;
    }
  }
  return t;
}

/* fixed tendons: length L = sum c q, force f = -ks (L - clamp(L, lo, hi)) - kd dL/dt (explicit) */
static void tendon_forces(const mg_model* m, const astate* s, real* tau /* per node */) {
  for (int i = 0; i < m->num_nodes; i++) tau[i] = 0.0;
  for (int t = 0; t < m->num_tendons; t++) {
    int n0 = m->tendon_dof[t][0] + 1, n1 = m->tendon_dof[t][1] + 1;
    real c0 = m->tendon_coef[t][0], c1 = m->tendon_coef[t][1];
    real L = c0 * s->qj[n0] + c1 * s->qj[n1];
    real Ld = c0 * s->qd[n0] + c1 * s->qd[n1];
    real lo = m->tendon_range[t][0], hi = m->tendon_range[t][1];
    real cl = L < lo ? lo : (L > hi ? hi : L);
    real f = -m->tendon_limit_stiffness[t] * (L - cl) - m->tendon_damping[t] * Ld;
    tau[n0] += c0 * f;
    tau[n1] += c1 * f;
  }
}

/* joint-space inertia (CRBA) incl. implicit diagonal, h = substep.  hc = h x link angular damping: the
 * implicit part of the damping couple -c I_w w on every link, M~ += h c sum_i Ja_i^T I_w,i Ja_i (added to
 * the links' rotational blocks before the composite pass) */
static void mass_matrix(const mg_model* m, const kin* k, real h, real* M, const real* diag, int ld, real hc) {
  int nv = ld, nn = m->num_nodes;
  real Ic[MAXN][6][6];
  memcpy(Ic, k->I, sizeof(real) * 36 * nn);
  if (hc != 0.0)
    for (int i = 0; i < nn; i++)
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Ic[i][a][b] += hc * k->Iw[i][a][b];
  for (int i = nn - 1; i >= 1; i--) {
    int p = m->parent[i];
    for (int a = 0; a < 6; a++)
      for (int b = 0; b < 6; b++) Ic[p][a][b] += Ic[i][a][b];
  }
  memset(M, 0, sizeof(real) * nv * nv);
  if (!m->fixed_base)
    for (int a = 0; a < 6; a++)
      for (int b = 0; b < 6; b++) M[a * nv + b] = Ic[0][a][b];
  for (int i = 1; i < nn; i++) {
    real F[6];
    mat6vec(Ic[i], k->S[i], F);
    int ci = dof_col(m, i);
    M[ci * nv + ci] = dot6(k->S[i], F) + (diag ? diag[i] : m->armature[i] + h * m->damping[i] + h * h * m->stiffness[i]);
    int j = m->parent[i];
    while (j > 0) {
      int cj = dof_col(m, j);
      real v = dot6(k->S[j], F);
      M[ci * nv + cj] = v;
      M[cj * nv + ci] = v;
      j = m->parent[j];
    }
    if (!m->fixed_base)
      for (int a = 0; a < 6; a++) { M[ci * nv + a] = F[a]; M[a * nv + ci] = F[a]; }
  }
}

/* bias forces C(q,v) incl. gravity (RNEA with qdd = 0) and the link damping couples c I_w w (cd = c) */
static void bias_forces(const mg_model* m, const kin* k, const astate* s, const real* g, real* C, real cd) {
  int nn = m->num_nodes, nv = nv_of(m); /* C has at least nv entries */
  real A[MAXN][6], f[MAXN][6];
  for (int c = 0; c < 6; c++) A[0][c] = 0;
  for (int i = 1; i < nn; i++) {
    real sq[6], t[6];
    for (int c = 0; c < 6; c++) sq[c] = k->S[i][c] * s->qd[i];
    crm(k->V[i], sq, t);
    for (int c = 0; c < 6; c++) A[i][c] = A[m->parent[i]][c] + t[c];
  }
  for (int i = 0; i < nn; i++) {
    real IA[6], IV[6], vIV[6];
    mat6vec((real(*)[6])k->I[i], A[i], IA);
    mat6vec((real(*)[6])k->I[i], k->V[i], IV);
    crf(k->V[i], IV, vIV);
    /* gravity: force m g at COM; moment about o = c x m g */
    real mass = m->mass[i];
    real cl[3] = {m->com[i][0], m->com[i][1], m->com[i][2]}, cw[3], c[3], mg[3], n[3];
    matvec3((real(*)[3])k->R[i], cl, cw);
    for (int a = 0; a < 3; a++) { c[a] = k->x[i][a] + cw[a] - k->o[a]; mg[a] = mass * g[a]; }
    cross3(c, mg, n);
    for (int a = 0; a < 3; a++) { f[i][a] = IA[a] + vIV[a] - n[a]; f[i][3 + a] = IA[3 + a] + vIV[3 + a] - mg[a]; }
    if (cd != 0.0) {
      real Iww[3];
      matvec3((real(*)[3])k->Iw[i], k->V[i], Iww);
      for (int a = 0; a < 3; a++) f[i][a] += cd * Iww[a];
    }
  }
  for (int i = nn - 1; i >= 1; i--)
    for (int c = 0; c < 6; c++) f[m->parent[i]][c] += f[i][c];
  memset(C, 0, sizeof(real) * nv);
  if (!m->fixed_base)
    for (int c = 0; c < 6; c++) C[c] = f[0][c];
  for (int i = 1; i < nn; i++) C[dof_col(m, i)] = dot6(k->S[i], f[i]);
}

static int cholesky(real* A, int n) {
  for (int j = 0; j < n; j++) {
    real s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    if (s <= 0) return -1;
    real d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      real t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  return 0;
}
static void chol_solve(const real* L, int n, real* b) {
  for (int i = 0; i < n; i++) {
    real s = b[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * b[k];
    b[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    real s = b[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * b[k];
    b[i] = s / L[i * n + i];
  }
}

/* ---------------------------------------------------------------- collision */
static void geom_world(const mg_model* m, const kin* k, int g, real* c, real R[3][3]) {
  int nd = m->geom_node[g];
  real pl[3] = {m->geom_pos[g][0], m->geom_pos[g][1], m->geom_pos[g][2]}, pw[3];
  matvec3((real(*)[3])k->R[nd], pl, pw);
  for (int a = 0; a < 3; a++) c[a] = k->x[nd][a] + pw[a];
  real gq[4] = {m->geom_quat[g][0], m->geom_quat[g][1], m->geom_quat[g][2], m->geom_quat[g][3]}, Rg[3][3];
  quat_to_mat(gq, Rg);
  matmul3((real(*)[3])k->R[nd], Rg, R);
}

static int push_contact(contact* out, int n, int cap, int nodeA, int gA, int nodeB, int gB, const real* p,
                        const real* nrm, real d) {
  if (n >= cap) return n;
  contact* c = &out[n];
  c->nodeA = nodeA; c->geomA = gA; c->nodeB = nodeB; c->geomB = gB;
  for (int a = 0; a < 3; a++) { c->p[a] = p[a]; c->n[a] = nrm[a]; }
  c->d = d;
  c->ill = orc_ill_next;
  c->amb = 0;
  orc_ill_next = 0;
  return n + 1;
}

/* sphere (center c, radius r) vs ground plane z = 0 */
static int sphere_plane(contact* out, int n, int cap, int node, int g, const real* c, real r, real off) {
  real d = c[2] - r;
  if (d < off) {
    real p[3] = {c[0], c[1], c[2] - r}, nz[3] = {0, 0, 1};
    n = push_contact(out, n, cap, node, g, -1, -1, p, nz, d);
  }
  return n;
}

static void closest_seg_seg(const real* p1, const real* q1, const real* p2, const real* q2, real* s_out,
                            real* t_out) {
  real d1[3], d2[3], r[3];
  for (int a = 0; a < 3; a++) { d1[a] = q1[a] - p1[a]; d2[a] = q2[a] - p2[a]; r[a] = p1[a] - p2[a]; }
  real a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  real s, t;
  real eps = 1e-12;
  if (a <= eps && e <= eps) { s = t = 0; }
  else if (a <= eps) { s = 0; t = f / e; t = t < 0 ? 0 : (t > 1 ? 1 : t); }
  else {
    real c = dot3(d1, r);
    if (e <= eps) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
    else {
      real b = dot3(d1, d2), den = a * e - b * b;
      s = den > eps ? (b * f - c * e) / den : 0.0;
      s = s < 0 ? 0 : (s > 1 ? 1 : s);
      t = (b * s + f) / e;
      if (t < 0) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
      else if (t > 1) { t = 1; s = (b - c) / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
    }
  }
  *s_out = s; *t_out = t;
}

/* segment (or point) endpoints + radius for sphere/capsule geoms */
static int geom_segment(const mg_model* m, const kin* k, int g, real* a, real* b, real* r) {
  real c[3], R[3][3];
  geom_world(m, k, g, c, R);
  int ty = m->geom_type[g];
  if (ty == MG_GT_SPHERE) {
    for (int i = 0; i < 3; i++) a[i] = b[i] = c[i];
    *r = m->geom_size[g][0];
    return 1;
  }
  if (ty == MG_GT_CAPSULE) {
    real hl = m->geom_size[g][1];
    for (int i = 0; i < 3; i++) { a[i] = c[i] - R[i][2] * hl; b[i] = c[i] + R[i][2] * hl; }
    *r = m->geom_size[g][0];
    return 1;
  }
  return 0;
}

/* ---- narrowphase against the free object's box (object frame: R = oR, center = op) */

/* signed distance of point pl (box frame) to a box of half extents hb: outside -> distance to the
 * closest point cb, normal away from the box; inside -> minus the smallest face depth (ties: x, y, z
 * order), normal = that face's outward normal, cb = the projection onto that face */
static real point_box(const real* pl, const real* hb, real* nb, real* cb) {
  real q[3];
  int out = 0;
  orc_pb_ill = 0;
  for (int a = 0; a < 3; a++) {
    q[a] = pl[a] < -hb[a] ? -hb[a] : (pl[a] > hb[a] ? hb[a] : pl[a]);
    if (q[a] != pl[a]) out++;
  }
  if (out) {
    real d[3] = {pl[0] - q[0], pl[1] - q[1], pl[2] - q[2]};
    real l = sqrt(dot3(d, d));
    orc_pb_ill = out >= 2 && l < NORMAL_ILL;
    for (int a = 0; a < 3; a++) { nb[a] = d[a] / l; cb[a] = q[a]; }
    return l;
  }
  /* inside: the depth is the nearest face's; the normal blends the faces within BOX_BLEND of the nearest one
   * (weight 1 - (depth - nearest) / BOX_BLEND), so it turns continuously across the box's medial planes instead
   * of jumping to whichever face rounding makes nearest; the surface point is p moved out along it by the depth */
  real e[6], dmin = 1e300;
  for (int a = 0; a < 3; a++) {
    e[2 * a] = hb[a] - pl[a];
    e[2 * a + 1] = hb[a] + pl[a];
  }
  for (int i = 0; i < 6; i++) dmin = fmin(dmin, e[i]);
  real n[3], nl = 0.0;
  for (int a = 0; a < 3; a++) {
    n[a] = fmax(0.0, 1.0 - (e[2 * a] - dmin) / BOX_BLEND) - fmax(0.0, 1.0 - (e[2 * a + 1] - dmin) / BOX_BLEND);
    nl += n[a] * n[a];
  }
  if (nl < 1e-12) { /* opposite faces cancel (a thin box entered at its middle): the nearest face, +x +y +z first */
    int i = 0;
    while (i < 5 && e[i] != dmin) i++;
    n[0] = n[1] = n[2] = 0.0;
    n[i / 2] = (i & 1) ? -1.0 : 1.0;
  } else {
    nl = sqrt(nl);
    for (int a = 0; a < 3; a++) n[a] /= nl;
  }
  for (int a = 0; a < 3; a++) {
    nb[a] = n[a];
    cb[a] = pl[a] + n[a] * dmin;
  }
  return -dmin;
}

/* closest parameter t in [0,1] of segment a + t u (box frame) to the box: f(t) = sum_k
 * max(|a_k + t u_k| - h_k, 0)^2 is convex piecewise quadratic; it is minimised exactly on each
 * interval between the (sorted) slab crossings.  If the segment passes through the box
 * (Liang-Barsky), returns the middle of the inside portion and *inside = 1. */
static real seg_box_t(const real* a, const real* u, const real* hb, int* inside) {
  real t0 = 0.0, t1 = 1.0;
  int hit = 1;
  for (int k = 0; k < 3 && hit; k++) {
    if (fabs(u[k]) < 1e-12) {
      if (a[k] < -hb[k] || a[k] > hb[k]) hit = 0;
    } else {
      real ta = (-hb[k] - a[k]) / u[k], tb = (hb[k] - a[k]) / u[k];
      if (ta > tb) { real x = ta; ta = tb; tb = x; }
      if (ta > t0) t0 = ta;
      if (tb < t1) t1 = tb;
      if (t0 > t1) hit = 0;
    }
  }
  if (hit) { *inside = 1; return 0.5 * (t0 + t1); }
  *inside = 0;
  real bp[8];
  int nb = 0;
  bp[nb++] = 0.0;
  for (int k = 0; k < 3; k++) {
    if (fabs(u[k]) < 1e-12) continue;
    for (int sgn = -1; sgn <= 1; sgn += 2) {
      real t = (sgn * hb[k] - a[k]) / u[k];
      if (t > 0.0 && t < 1.0) bp[nb++] = t;
    }
  }
  bp[nb++] = 1.0;
  for (int i = 1; i < nb; i++) /* insertion sort */
    for (int j = i; j > 0 && bp[j] < bp[j - 1]; j--) { real x = bp[j]; bp[j] = bp[j - 1]; bp[j - 1] = x; }
  real best_t = 0.0, best_f = 1e300;
  for (int i = 0; i + 1 < nb; i++) {
    real lo = bp[i], hi = bp[i + 1], mid = 0.5 * (lo + hi), num = 0.0, den = 0.0;
    for (int k = 0; k < 3; k++) {
      real x = a[k] + mid * u[k];
      if (x > hb[k]) { num += (a[k] - hb[k]) * u[k]; den += u[k] * u[k]; }
      else if (x < -hb[k]) { num += (a[k] + hb[k]) * u[k]; den += u[k] * u[k]; }
    }
    real t = den > 0.0 ? -num / den : lo;
    t = t < lo ? lo : (t > hi ? hi : t);
    real f = 0.0;
    for (int k = 0; k < 3; k++) {
      real x = fabs(a[k] + t * u[k]) - hb[k];
      if (x > 0) f += x * x;
    }
    if (f < best_f) { best_f = f; best_t = t; }
  }
  return best_t;
}

/* A segment a + t u whose core has entered a box (seg_box_t's inside case): the contact is taken against the
 * face of least push-out of the WHOLE segment -- SAT over the box's face axes, delta(k, s) = hb_k - min(s a_k,
 * s (a_k + u_k)) for the face of outward normal s e_k, ties in x+ x- y+ y- z+ z- order -- at the segment end
 * deepest behind it.  The inside portion's midpoint (the rule before round 4) lies on a thin box's mid-plane by
 * construction when the segment pierces it (the reference's pen reset pose through the palm, shadow_hand.py:
 * 313-314, 625-629), so the face it was pushed through flipped with rounding; the whole segment's extents
 * decide robustly.  Returns the face (2 k + (s < 0)); *t = the deepest end (0 or 1). */
static int seg_box_sat(const real* a, const real* u, const real* hb, real* t) {
  int best = 0;
  real bd = 1e300, bd2 = 1e300;
  for (int f = 0; f < 6; f++) {
    const int k = f >> 1;
    const real sg = (f & 1) ? -1.0 : 1.0, e0 = sg * a[k], e1 = sg * (a[k] + u[k]);
    const real dl = hb[k] - (e0 < e1 ? e0 : e1);
    if (dl < bd) { bd2 = bd; bd = dl; best = f; }
    else if (dl < bd2) bd2 = dl;
  }
  if (bd2 - bd < orc_tie_delta) orc_tie_hit = 1;
  const int k = best >> 1;
  const real sg = (best & 1) ? -1.0 : 1.0;
  *t = sg * a[k] <= sg * (a[k] + u[k]) ? 0.0 : 1.0;
  return best;
}
/* signed distance of point P (box frame) along face f's outward normal from that face's plane (negative behind
 * it); nb = the normal, cb = P moved onto the plane */
static real box_face_point(const real* P, const real* hb, int f, real* nb, real* cb) {
  const int k = f >> 1;
  const real sg = (f & 1) ? -1.0 : 1.0;
  for (int a = 0; a < 3; a++) { nb[a] = a == k ? sg : 0.0; cb[a] = P[a]; }
  cb[k] = sg * hb[k];
  return sg * P[k] - hb[k];
}

static void to_obj(const kin* k, const real* pw, real* pl) {
  real d[3] = {pw[0] - k->op[0], pw[1] - k->op[1], pw[2] - k->op[2]};
  mattvec3((real(*)[3])k->oR, d, pl);
}
static void from_obj_dir(const kin* k, const real* dl, real* dw) { matvec3((real(*)[3])k->oR, dl, dw); }
static void from_obj_pt(const kin* k, const real* pl, real* pw) {
  matvec3((real(*)[3])k->oR, pl, pw);
  for (int a = 0; a < 3; a++) pw[a] += k->op[a];
}

/* ---- the convex-mesh geom (MG_GT_CONVEX): the model's hull_* tables, geom frame ----------------------
 * (ShadowHand's robot0:C_forearm = mesh robot0:forearm_cvx, robot.xml:8, shared_asset.xml:15; the hull's
 * 64 kept vertices and 124 outward face planes come from tools/build_models.py) */

/* largest plane distance of point pl (geom frame) over the hull's faces: the signed distance inside and
 * where a face is the nearest feature, a lower bound of the distance outside near edges and vertices;
 * *f = the face */
static real point_hull(const mg_model* m, const real* pl, int* f) {
  real best = -1e300;
  int bf = 0;
  for (int i = 0; i < m->hull_num_planes; i++) {
    const float* q = m->hull_plane[i];
    const real s = q[0] * pl[0] + q[1] * pl[1] + q[2] * pl[2] - q[3];
    if (s > best) { best = s; bf = i; }
  }
  *f = bf;
  return best;
}

/* broadphase of the hull geom (centre c, axes R, half extents hg = its bounding box) against a sphere
 * (centre w, radius r): 1 if the sphere comes within `off` of the box (the kernel applies the same test) */
static int hull_box_near(const real* c, real R[3][3], const real* hg, const real* w, real r, real off) {
  real d[3] = {w[0] - c[0], w[1] - c[1], w[2] - c[2]}, l[3], s = 0.0;
  mattvec3(R, d, l);
  for (int a = 0; a < 3; a++) {
    const real e = fabs(l[a]) - hg[a];
    if (e > 0) s += e * e;
  }
  return sqrt(s) - r < off;
}

/* Box-box edge-edge contact (object frame: the object box B at the origin, axis aligned, half extents hb;
 * the hand box A: centre c, axes = columns of R, half extents hg).  Separating-axis test over the 15 axes
 * (3 + 3 face normals, 9 edge cross products; an edge axis within ~11 deg of a face normal is left to the
 * face contacts); when the best axis (largest separation, or least
 * penetration) is an edge-edge axis by more than 1e-5 m over the best face axis and the separation is
 * below `off`, one contact at the closest points of the two supporting edges, provided both lie within
 * their edges (otherwise the vertex-face candidates cover the configuration).  Normal from B to A, gap =
 * the separation along it.  Returns 1 with *pt, *nrm, *d set, else 0. */
static int box_box_edge(const real* c, real R[3][3], const real* hg, const real* hb, real off, real* pt, real* nrm,
                        real* d) {
  real face = -1e300;
  for (int i = 0; i < 3; i++) { /* B's face axes e_i */
    real ra = 0.0;
    for (int k = 0; k < 3; k++) ra += hg[k] * fabs(R[i][k]);
    const real sep = fabs(c[i]) - hb[i] - ra;
    if (sep > face) face = sep;
  }
  for (int j = 0; j < 3; j++) { /* A's face axes a_j */
    const real t = R[0][j] * c[0] + R[1][j] * c[1] + R[2][j] * c[2];
    real rb = 0.0;
    for (int i = 0; i < 3; i++) rb += hb[i] * fabs(R[i][j]);
    const real sep = fabs(t) - hg[j] - rb;
    if (sep > face) face = sep;
  }
  /* edge axes L = e_i x a_j in closed form (the classic OBB test, R[i][j] = e_i . a_j):
   * L = (.., -R[i2][j] at i1, R[i1][j] at i2), |L|^2 = R[i1][j]^2 + R[i2][j]^2, T.L = T[i2] R[i1][j] - T[i1] R[i2][j],
   * B's radius hb[i1] |R[i2][j]| + hb[i2] |R[i1][j]|, A's hg[j1] |R[i][j2]| + hg[j2] |R[i][j1]| (L.a_k = e_i.(a_j x a_k)) */
  real best = -1e300, L[3] = {0, 0, 0};
  int bi = -1, bj = -1;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      const real ln = sqrt(R[i1][j] * R[i1][j] + R[i2][j] * R[i2][j]);
      if (ln < 1e-6) continue; /* parallel edges: the face axes decide */
      /* an axis within ~11 deg of a face normal of either box is a face configuration (a box resting
       * tilted on a face): the vertex-face contacts describe it */
      const real near = fmax(fmax(fabs(R[i1][j]), fabs(R[i2][j])), fmax(fabs(R[i][j1]), fabs(R[i][j2]))) / ln;
      if (near > 0.98) continue;
      const real tl = c[i2] * R[i1][j] - c[i1] * R[i2][j];
      const real rb = hb[i1] * fabs(R[i2][j]) + hb[i2] * fabs(R[i1][j]);
      const real ra = hg[j1] * fabs(R[i][j2]) + hg[j2] * fabs(R[i][j1]);
      const real sep = (fabs(tl) - ra - rb) / ln;
      if (sep > best) {
        const real sg = tl < 0 ? -1.0 : 1.0; /* orient L from B towards A */
        best = sep; bi = i; bj = j;
        L[i] = 0.0;
        L[i1] = -sg * R[i2][j] / ln;
        L[i2] = sg * R[i1][j] / ln;
      }
    }
  if (bi < 0 || !(best > face + 1e-5) || !(best < off)) return 0;
  /* B's supporting edge: parallel to e_bi, the corner towards +L; A's: parallel to a_bj, towards -L */
  real pb[3], pa[3], ub[3] = {0, 0, 0}, ua[3] = {R[0][bj], R[1][bj], R[2][bj]};
  ub[bi] = 1.0;
  for (int a = 0; a < 3; a++) pb[a] = a == bi ? 0.0 : (L[a] >= 0 ? hb[a] : -hb[a]);
  for (int a = 0; a < 3; a++) pa[a] = c[a];
  for (int k = 0; k < 3; k++) {
    if (k == bj) continue;
    const real s = (L[0] * R[0][k] + L[1] * R[1][k] + L[2] * R[2][k]) >= 0 ? -hg[k] : hg[k];
    for (int a = 0; a < 3; a++) pa[a] += s * R[a][k];
  }
  /* closest points of the lines pa + s ua and pb + t ub */
  real w0[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
  const real b = dot3(ua, ub), dd = dot3(ua, w0), e = dot3(ub, w0), den = 1.0 - b * b;
  if (den < 1e-12) return 0;
  const real sa = (b * e - dd) / den, tb = (e - b * dd) / den;
  if (fabs(sa) > hg[bj] || fabs(tb) > hb[bi]) return 0;
  for (int a = 0; a < 3; a++) {
    pt[a] = 0.5 * ((pa[a] + sa * ua[a]) + (pb[a] + tb * ub[a]));
    nrm[a] = L[a];
  }
  *d = best;
  return 1;
}

/* the hull against the object's core, exactly (defined with the convex narrowphase below) */
static int hull_object_exact(const mg_model* m, const kin* k, int g, const real* c, real R[3][3], real off,
                             contact* out, int n, int cap);

/* hand geom g (A) vs the object box (B); normal points from the object to the geom */
static int geom_object(const mg_model* m, const kin* k, int g, real off, contact* out, int n, int cap) {
  const real hb[3] = {m->obj_size[0], m->obj_size[1], m->obj_size[2]};
  int nd = m->geom_node[g], ty = m->geom_type[g];
  real c[3], R[3][3];
  geom_world(m, k, g, c, R);
  if (ty == MG_GT_SPHERE || ty == MG_GT_CAPSULE) {
    real r = m->geom_size[g][0], hl = ty == MG_GT_CAPSULE ? m->geom_size[g][1] : 0.0;
    real aw[3], bw[3], al[3], bl[3], u[3];
    for (int a = 0; a < 3; a++) { aw[a] = c[a] - R[a][2] * hl; bw[a] = c[a] + R[a][2] * hl; }
    to_obj(k, aw, al);
    to_obj(k, bw, bl);
    for (int a = 0; a < 3; a++) u[a] = bl[a] - al[a];
    int inside;
    real t = seg_box_t(al, u, hb, &inside), P[3], nb[3], cb[3];
    const int face = inside ? seg_box_sat(al, u, hb, &t) : -1;
    for (int a = 0; a < 3; a++) P[a] = al[a] + t * u[a];
    real sd = inside ? box_face_point(P, hb, face, nb, cb) : point_box(P, hb, nb, cb), d = sd - r;
    if (d < off) {
      real pm[3], pw[3], nw[3];
      for (int a = 0; a < 3; a++) pm[a] = 0.5 * ((P[a] - r * nb[a]) + cb[a]);
      from_obj_pt(k, pm, pw);
      from_obj_dir(k, nb, nw);
      orc_ill_next = !inside && orc_pb_ill;
      n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
    }
    return n;
  }
  if (ty == MG_GT_CONVEX) {
    const real hg[3] = {m->geom_size[g][0], m->geom_size[g][1], m->geom_size[g][2]};
    if (!hull_box_near(c, R, hg, k->op, sqrt(dot3(hb, hb)), off)) return n;
    /* the hull's vertices against the object */
    for (int v = 0; v < m->hull_num_verts; v++) {
      real l[3] = {m->hull_vert[v][0], m->hull_vert[v][1], m->hull_vert[v][2]}, w[3], pl[3];
      matvec3(R, l, w);
      for (int a = 0; a < 3; a++) w[a] += c[a];
      to_obj(k, w, pl);
      real nb[3], cb[3], d = point_box(pl, hb, nb, cb);
      if (d < off) {
        real pm[3], pw[3], nw[3];
        for (int a = 0; a < 3; a++) pm[a] = 0.5 * (pl[a] + cb[a]);
        from_obj_pt(k, pm, pw);
        from_obj_dir(k, nb, nw);
        orc_ill_next = orc_pb_ill;
        n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
      }
    }
    /* the object's vertices against the hull's faces (normal: minus the face normal) */
    for (int v = 0; v < 8; v++) {
      real l[3] = {(v & 1 ? 1 : -1) * hb[0], (v & 2 ? 1 : -1) * hb[1], (v & 4 ? 1 : -1) * hb[2]}, w[3], dl[3], pl[3];
      from_obj_pt(k, l, w);
      for (int a = 0; a < 3; a++) dl[a] = w[a] - c[a];
      mattvec3(R, dl, pl);
      int f;
      const real d = point_hull(m, pl, &f);
      if (d < off) {
        const real ng[3] = {m->hull_plane[f][0], m->hull_plane[f][1], m->hull_plane[f][2]};
        real pm[3], pw[3], nw[3];
        for (int a = 0; a < 3; a++) pm[a] = pl[a] - 0.5 * d * ng[a];
        matvec3(R, pm, pw);
        for (int a = 0; a < 3; a++) pw[a] += c[a];
        matvec3(R, ng, nw);
        for (int a = 0; a < 3; a++) nw[a] = -nw[a];
        n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
      }
    }
    /* edge against edge / edge across a face: the exact distance of the hull and the box */
    return hull_object_exact(m, k, g, c, R, off, out, n, cap);
  }
  if (ty != MG_GT_BOX) return n;
  const real hg[3] = {m->geom_size[g][0], m->geom_size[g][1], m->geom_size[g][2]};
  /* the geom's vertices against the object */
  for (int v = 0; v < 8; v++) {
    real l[3] = {(v & 1 ? 1 : -1) * hg[0], (v & 2 ? 1 : -1) * hg[1], (v & 4 ? 1 : -1) * hg[2]}, w[3], pl[3];
    matvec3(R, l, w);
    for (int a = 0; a < 3; a++) w[a] += c[a];
    to_obj(k, w, pl);
    real nb[3], cb[3], d = point_box(pl, hb, nb, cb);
    if (d < off) {
      real pm[3], pw[3], nw[3];
      for (int a = 0; a < 3; a++) pm[a] = 0.5 * (pl[a] + cb[a]);
      from_obj_pt(k, pm, pw);
      from_obj_dir(k, nb, nw);
      orc_ill_next = orc_pb_ill;
      n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
    }
  }
  /* the object's vertices against the geom box (normal flipped: geom -> object is -n) */
  for (int v = 0; v < 8; v++) {
    real l[3] = {(v & 1 ? 1 : -1) * hb[0], (v & 2 ? 1 : -1) * hb[1], (v & 4 ? 1 : -1) * hb[2]}, w[3], d3[3], pl[3];
    from_obj_pt(k, l, w);
    for (int a = 0; a < 3; a++) d3[a] = w[a] - c[a];
    mattvec3(R, d3, pl);
    real nb[3], cb[3], d = point_box(pl, hg, nb, cb);
    if (d < off) {
      real pm[3], pw[3], nw[3];
      for (int a = 0; a < 3; a++) pm[a] = 0.5 * (pl[a] + cb[a]);
      matvec3(R, pm, pw);
      for (int a = 0; a < 3; a++) pw[a] += c[a];
      matvec3(R, nb, nw);
      for (int a = 0; a < 3; a++) nw[a] = -nw[a];
      orc_ill_next = orc_pb_ill;
      n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
    }
  }
  /* edge against edge (the vertex-face tests above miss an edge resting across an edge) */
  {
    real cl[3], Rt[3][3], Rl[3][3], pe[3], ne[3], de;
    to_obj(k, c, cl);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) Rt[a][b] = k->oR[b][a];
    matmul3(Rt, R, Rl);
    if (box_box_edge(cl, Rl, hg, hb, off, pe, ne, &de)) {
      real pw[3], nw[3];
      from_obj_pt(k, pe, pw);
      from_obj_dir(k, ne, nw);
      n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, de);
    }
  }
  return n;
}

/* ---- convex narrowphase against the egg (ellipsoid) and the pen (capsule) objects ------------------
 * (ShadowHand objectType egg / pen, shadow_hand.py:86-100: open_ai_assets/hand/egg.xml = ellipsoid
 * 0.03 x 0.03 x 0.04, pen.xml = capsule r 0.008, half length 0.1).  Everything is evaluated in the
 * object frame (object centred at the origin).  Hand-geom cores: a segment (sphere/capsule core, the
 * radius is added afterwards) or a box.
 *
 * GJK distance (Gilbert-Johnson-Keerthi on the Minkowski difference A - B; closest point of the
 * simplex by Voronoi-region tests; stop when |v|^2 - v.w <= 1e-8 |v|^2 + 1e-24, a repeated support
 * point, no progress, or 64 iterations; fp64; early exit once a separating plane is farther than the
 * contact offset, since such a candidate is not a contact).  Box cores are rounded by a 1 mm margin
 * (CVX_MARGIN: edges and corners of a hand box become 1 mm round; penetrations shallower than that
 * stay with GJK).  Overlapping cores (the simplex encloses the origin) go to
 * MPR (below) for the penetration vector.  GJK's witnesses are then polished by alternating projections
 * (cvx_polish).  The HIP kernel (csrc/convex.hpp) runs the same algorithm in fp32. */
typedef struct {
  int kind;                    /* 0 segment [p0, p1], 1 box (c, R columns = axes, h) */
  real p0[3], p1[3];
  real c[3], R[3][3], h[3];
} cvx_shape;

static void cvx_support(const cvx_shape* A, const real* d, real* o) {
  if (A->kind == 0) {
    const real* s = dot3(A->p0, d) >= dot3(A->p1, d) ? A->p0 : A->p1;
    for (int a = 0; a < 3; a++) o[a] = s[a];
    return;
  }
  for (int a = 0; a < 3; a++) o[a] = A->c[a];
  for (int k = 0; k < 3; k++) {
    real dk = A->R[0][k] * d[0] + A->R[1][k] * d[1] + A->R[2][k] * d[2];
    real s = dk >= 0 ? A->h[k] : -A->h[k];
    for (int a = 0; a < 3; a++) o[a] += s * A->R[a][k];
  }
}

/* support point of the ellipsoid x^2/e0^2 + y^2/e1^2 + z^2/e2^2 = 1 in direction d */
static void ell_support(const real* e, const real* d, real* o) {
  real q[3] = {e[0] * e[0] * d[0], e[1] * e[1] * d[1], e[2] * e[2] * d[2]};
  real n = sqrt(q[0] * d[0] + q[1] * d[1] + q[2] * d[2]);
  if (n < 1e-30) { o[0] = o[1] = o[2] = 0.0; return; }
  for (int a = 0; a < 3; a++) o[a] = q[a] / n;
}

/* closest point of segment / triangle (Ericson, Real-Time Collision Detection 5.1.2 / 5.1.5) to the
 * origin as barycentric weights */
static void cvx_seg(const real* a, const real* b, real* lam) {
  real ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, den = dot3(ab, ab);
  real t = den > 0 ? -dot3(a, ab) / den : 0.0;
  t = t < 0 ? 0 : (t > 1 ? 1 : t);
  lam[0] = 1 - t; lam[1] = t;
}
static void cvx_tri(const real* a, const real* b, const real* c, real* lam) {
  real ab[3], ac[3];
  for (int k = 0; k < 3; k++) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; }
  lam[0] = lam[1] = lam[2] = 0.0;
  real d1 = -dot3(ab, a), d2 = -dot3(ac, a);
  if (d1 <= 0 && d2 <= 0) { lam[0] = 1; return; }
  real d3 = -dot3(ab, b), d4 = -dot3(ac, b);
  if (d3 >= 0 && d4 <= d3) { lam[1] = 1; return; }
  real vc = d1 * d4 - d3 * d2;
  /* the three edge cases divide by a length that is 0 only for coincident vertices (a == b, a == c, b == c,
   * e.g. an MPR portal whose support points repeat): then the vertex itself is the answer (no 0 / 0) */
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    real v = (d1 - d3) > 0 ? d1 / (d1 - d3) : 0;
    lam[0] = 1 - v; lam[1] = v; return;
  }
  real d5 = -dot3(ab, c), d6 = -dot3(ac, c);
  if (d6 >= 0 && d5 <= d6) { lam[2] = 1; return; }
  real vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    real w = (d2 - d6) > 0 ? d2 / (d2 - d6) : 0;
    lam[0] = 1 - w; lam[2] = w; return;
  }
  real va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    real den2 = (d4 - d3) + (d5 - d6);
    real w = den2 > 0 ? (d4 - d3) / den2 : 0;
    lam[1] = 1 - w; lam[2] = w; return;
  }
  real den = va + vb + vc;
  if (!(den > 0)) { real l2[2]; cvx_seg(a, b, l2); lam[0] = l2[0]; lam[1] = l2[1]; return; }
  real v = vb / den, w = vc / den;
  lam[0] = 1 - v - w; lam[1] = v; lam[2] = w;
}

/* closest point of the simplex W[0..n-1] to the origin; keeps the supporting vertices (W, P in
 * place, order preserved), returns 1 if the origin lies inside a (non-degenerate) tetrahedron */
static int cvx_simplex(real W[4][3], real P[4][3], int* n, real* v, real* lk) {
  real lam[4] = {0, 0, 0, 0};
  if (*n == 1) {
    lam[0] = 1;
  } else if (*n == 2) {
    cvx_seg(W[0], W[1], lam);
  } else if (*n == 3) {
    cvx_tri(W[0], W[1], W[2], lam);
  } else {
    static const int F[4][4] = {{0, 1, 2, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {1, 3, 2, 0}}; /* face + opposite */
    real best = 1e300;
    int any = 0;
    for (int f = 0; f < 4; f++) {
      const real *a = W[F[f][0]], *b = W[F[f][1]], *c = W[F[f][2]], *d = W[F[f][3]];
      real ab[3], ac[3], ad[3], nf[3];
      for (int k = 0; k < 3; k++) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; ad[k] = d[k] - a[k]; }
      cross3(ab, ac, nf);
      real sp = -dot3(nf, a), sd = dot3(nf, ad);
      real sc = dot3(ab, ab) + dot3(ac, ac) + dot3(ad, ad);
      int degenerate = sd * sd <= 1e-12 * sc * sc * sc;
      if (!(sp * sd < 0) && !degenerate) continue;
      any = 1;
      real l3[3], q[3];
      cvx_tri(a, b, c, l3);
      for (int k = 0; k < 3; k++) q[k] = l3[0] * a[k] + l3[1] * b[k] + l3[2] * c[k];
      real dq = dot3(q, q);
      if (dq < best) {
        best = dq;
        lam[0] = lam[1] = lam[2] = lam[3] = 0;
        lam[F[f][0]] = l3[0]; lam[F[f][1]] = l3[1]; lam[F[f][2]] = l3[2];
      }
    }
    if (!any) return 1;
  }
  int m = 0;
  v[0] = v[1] = v[2] = 0;
  real Wn[4][3], Pn[4][3];
  for (int i = 0; i < *n; i++) {
    if (!(lam[i] > 0)) continue;
    for (int k = 0; k < 3; k++) { v[k] += lam[i] * W[i][k]; Wn[m][k] = W[i][k]; Pn[m][k] = P[i][k]; }
    lk[m++] = lam[i];
  }
  memcpy(W, Wn, sizeof(real) * 3 * m);
  memcpy(P, Pn, sizeof(real) * 3 * m);
  *n = m;
  return 0;
}

/* GJK distance between core A and the ellipsoid e (origin-centred).  Returns 1 when separated, with
 * the closest points pa (on A), pb (on the ellipsoid) and the distance; 0 when the cores overlap. */
/* the core's point nearest the egg's centre in the egg-scaled metric (x / e): the segment's exact
 * minimiser of |p(t) / e|^2, or the box centre.  Returns 1 when that point lies inside the egg, i.e. the
 * cores certainly overlap (exact for a segment; sufficient for a box). */
static int cvx_core_point(const cvx_shape* A, const real* e, real* sp) {
  if (A->kind == 0) {
    real q0[3], qu[3];
    for (int a = 0; a < 3; a++) { q0[a] = A->p0[a] / e[a]; qu[a] = (A->p1[a] - A->p0[a]) / e[a]; }
    real den = dot3(qu, qu), t = den > 0 ? -dot3(q0, qu) / den : 0.0;
    t = t < 0 ? 0 : (t > 1 ? 1 : t);
    for (int a = 0; a < 3; a++) sp[a] = A->p0[a] + t * (A->p1[a] - A->p0[a]);
  } else {
    for (int a = 0; a < 3; a++) sp[a] = A->c[a];
  }
  real r2 = 0;
  for (int a = 0; a < 3; a++) r2 += (sp[a] / e[a]) * (sp[a] / e[a]);
  return r2 < 1.0;
}

static int cvx_gjk(const cvx_shape* A, const real* e, real cut, real* pa, real* pb, real* dist) {
  real W[4][3], P[4][3], v[3];
  if (A->kind == 0) { /* start from the segment point nearest the egg in its metric, towards the egg */
    real sp[3], gr[3], bs[3];
    cvx_core_point(A, e, sp);
    for (int a = 0; a < 3; a++) gr[a] = sp[a] / (e[a] * e[a]);
    ell_support(e, gr, bs);
    for (int a = 0; a < 3; a++) v[a] = sp[a] - bs[a];
  } else {
    for (int a = 0; a < 3; a++) v[a] = A->c[a];
  }
  if (dot3(v, v) < 1e-20) { v[0] = 0; v[1] = 0; v[2] = 1; }
  int n = 0;
  real vv = dot3(v, v);
  real lam[4] = {0, 0, 0, 0};
  for (int it = 0; it < 64; it++) {
    real nd[3] = {-v[0], -v[1], -v[2]}, a[3], b[3], w[3];
    cvx_support(A, nd, a);
    ell_support(e, v, b);
    for (int k = 0; k < 3; k++) w[k] = a[k] - b[k];
    const real vw = dot3(v, w);
    if (vw > 0 && vw * vw > vv * cut * cut) { /* separating plane farther than cut: no contact */
      *dist = vw / sqrt(vv);
      return 2;
    }
    if (n > 0 && vv - vw <= 1e-8 * vv + 1e-24) break;
    int dup = 0;
    for (int i = 0; i < n; i++) {
      real dd[3] = {W[i][0] - w[0], W[i][1] - w[1], W[i][2] - w[2]};
      if (dot3(dd, dd) <= 1e-24) dup = 1;
    }
    if (dup) break;
    for (int k = 0; k < 3; k++) { W[n][k] = w[k]; P[n][k] = a[k]; }
    n++;
    if (cvx_simplex(W, P, &n, v, lam)) return 0;
    real vn = dot3(v, v);
    if (vn <= 1e-20) return 0;
    int stall = it > 0 && vn >= vv * (1.0 - 1e-14); /* v starts at the centre difference */
    vv = vn;
    if (stall) break;
  }
  /* closest points: the kept simplex's weights applied to its A-side support points */
  for (int k = 0; k < 3; k++) {
    pa[k] = 0;
    for (int i = 0; i < n; i++) pa[k] += lam[i] * P[i][k];
    pb[k] = pa[k] - v[k];
  }
  *dist = sqrt(vv);
  return 1;
}

/* one contact between core A (+ radius rA) and the ellipsoid e, object frame: GJK, then the
 * shrunk-core retry, then the centre-direction fallback (see above).  Normal from the object to A. */
/* MPR penetration (Minkowski portal refinement, XenoCollide; fixed state: the interior point v0 and a
 * portal triangle v1 v2 v3, each with its A-side support point) for cores known to overlap.  Returns
 * 1 with the boundary point x of A - B nearest to where the refined portal meets the origin's side
 * (penetration vector: moving A by -x separates the cores) and the A-side witness pa; 0 if the portal
 * search degenerates. */
static void mpr_support(const cvx_shape* A, const real* e, const real* d, real* w, real* a) {
  real b[3], nd[3] = {-d[0], -d[1], -d[2]};
  cvx_support(A, d, a);
  ell_support(e, nd, b);
  for (int k = 0; k < 3; k++) w[k] = a[k] - b[k];
}
static void v3sub(const real* a, const real* b, real* o) { for (int k = 0; k < 3; k++) o[k] = a[k] - b[k]; }
static void v3unit(real* a) {
  real l = sqrt(dot3(a, a));
  if (l > 0) for (int k = 0; k < 3; k++) a[k] /= l;
}
static void v3cp(real* d, const real* s) { d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; }
static void mpr_portal_dir(real V[5][3], real* dir) {
  real a[3], b[3];
  v3sub(V[2], V[1], a);
  v3sub(V[3], V[1], b);
  cross3(a, b, dir);
  v3unit(dir);
}
/* replace one portal vertex by v4 so that the portal keeps facing the origin ray */
static void mpr_expand(real V[5][3], real Pa[5][3]) {
  real c[3];
  cross3(V[4], V[0], c);
  int k;
  if (dot3(V[1], c) > 0) k = dot3(V[2], c) > 0 ? 1 : 3;
  else k = dot3(V[3], c) > 0 ? 2 : 1;
  v3cp(V[k], V[4]);
  v3cp(Pa[k], Pa[4]);
}
static int mpr_reached(real V[5][3], const real* dir) {
  real d4 = dot3(V[4], dir);
  real m = fmin(d4 - dot3(V[1], dir), fmin(d4 - dot3(V[2], dir), d4 - dot3(V[3], dir)));
  return m <= MPR_TOL;
}
static int cvx_mpr(const cvx_shape* A, const real* e, real* x, real* pa) {
  real V[5][3], Pa[5][3], dir[3];
  if (A->kind == 0) for (int a = 0; a < 3; a++) V[0][a] = 0.5 * (A->p0[a] + A->p1[a]);
  else for (int a = 0; a < 3; a++) V[0][a] = A->c[a];
  if (dot3(V[0], V[0]) < 1e-20) { V[0][0] = 1e-6; V[0][1] = 0; V[0][2] = 0; }
  for (int k = 0; k < 3; k++) dir[k] = -V[0][k];
  v3unit(dir);
  mpr_support(A, e, dir, V[1], Pa[1]);
  if (dot3(V[1], dir) <= 0) return 0;
  cross3(V[0], V[1], dir);
  if (dot3(dir, dir) <= 1e-24) { /* the origin lies on the segment v0 - v1 */
    v3cp(x, V[1]);
    v3cp(pa, Pa[1]);
    return 1;
  }
  v3unit(dir);
  mpr_support(A, e, dir, V[2], Pa[2]);
  if (dot3(V[2], dir) <= 0) return 0;
  real va[3], vb[3];
  v3sub(V[1], V[0], va);
  v3sub(V[2], V[0], vb);
  cross3(va, vb, dir);
  v3unit(dir);
  if (dot3(dir, V[0]) > 0) {
    real t[3];
    v3cp(t, V[1]); v3cp(V[1], V[2]); v3cp(V[2], t);
    v3cp(t, Pa[1]); v3cp(Pa[1], Pa[2]); v3cp(Pa[2], t);
    for (int k = 0; k < 3; k++) dir[k] = -dir[k];
  }
  int it;
  for (it = 0; it < 64; it++) { /* discover a portal the origin ray passes through */
    mpr_support(A, e, dir, V[3], Pa[3]);
    if (dot3(V[3], dir) <= 0) return 0;
    real c[3];
    cross3(V[1], V[3], c);
    if (dot3(c, V[0]) < -MPR_EPS) {
      v3cp(V[2], V[3]); v3cp(Pa[2], Pa[3]);
    } else {
      cross3(V[3], V[2], c);
      if (dot3(c, V[0]) < -MPR_EPS) {
        v3cp(V[1], V[3]); v3cp(Pa[1], Pa[3]);
      } else {
        break;
      }
    }
    v3sub(V[1], V[0], va);
    v3sub(V[2], V[0], vb);
    cross3(va, vb, dir);
    v3unit(dir);
  }
  if (it == 64) return 0;
  for (it = 0; it < 64; it++) { /* refine until the portal encloses the origin */
    mpr_portal_dir(V, dir);
    if (dot3(V[1], dir) >= 0) break;
    mpr_support(A, e, dir, V[4], Pa[4]);
    if (dot3(V[4], dir) < 0 || mpr_reached(V, dir)) return 0;
    mpr_expand(V, Pa);
  }
  if (it == 64) return 0;
  for (it = 0;; it++) { /* push the portal onto the boundary */
    mpr_portal_dir(V, dir);
    mpr_support(A, e, dir, V[4], Pa[4]);
    if (mpr_reached(V, dir) || it >= 64) break;
    mpr_expand(V, Pa);
  }
  real lam[3];
  cvx_tri(V[1], V[2], V[3], lam);
  for (int k = 0; k < 3; k++) {
    x[k] = lam[0] * V[1][k] + lam[1] * V[2][k] + lam[2] * V[3][k];
    pa[k] = lam[0] * Pa[1][k] + lam[1] * Pa[2][k] + lam[2] * Pa[3][k];
  }
  return 1;
}

/* Exact penetration of a segment core [p0, p1] (or a point) overlapping the ellipsoid e (the minimum
 * translation): depth = min over unit n of max_k (h_E(n) - n.p_k), the translation of the core along n that
 * separates it.  The minimum is a vertex one -- the distance from an end inside the ellipsoid to the surface,
 * valid when the other end is not deeper along that normal -- or, when neither is, the edge one on the great
 * circle n.u = 0: the distance from the core's shadow point to the boundary of the ellipsoid's shadow ellipse in
 * the plane normal to u.  Each is the nearest-boundary-point problem of an interior point: b_i = s_i q_i / (s_i +
 * lam) with the root lam in (-min s_i, 0] of sum_i s_i q_i^2 / (s_i + lam)^2 = 1 (s = squared semi-axes), by
 * Newton's method from lam = 0 (the function is convex and decreasing there: one step lands left of the root,
 * the rest climb to it).  MPR's portal normal is a facet of a polytope approximation (a 1e-7 m change of the
 * state turned it by 1e-2 rad for a capsule 1 cm deep); this solution moves smoothly with the state away from
 * the medial axis, where orc_cvx_ill marks it.  The kernel (convex.hpp seg_mtd) runs the same in fp32: the result
 * is a smooth function of the state, with no portal decisions for fp32 to take differently. */
static real ell_root(int k, const real* s2, const real* q, real* smin_out) {
  real smin = s2[0];
  for (int i = 1; i < k; i++) smin = fmin(smin, s2[i]);
  real lam = 0.0;
  for (int it = 0; it < 64; it++) {
    real f = -1.0, fp = 0.0;
    for (int i = 0; i < k; i++) {
      const real den = s2[i] + lam, r = s2[i] * q[i] * q[i] / (den * den);
      f += r;
      fp -= 2.0 * r / den;
    }
    if (!(fp < 0.0)) break;
    real nl = lam - f / fp;
    if (!(nl > -smin)) nl = 0.5 * (lam - smin); /* keep clear of the pole */
    if (nl > 0.0) nl = 0.0;
    const real dl = fabs(nl - lam);
    lam = nl;
    if (dl <= 1e-14 * smin) break;
  }
  *smin_out = smin;
  return lam;
}
/* the vertex solution of an end p inside e: outward normal n, depth */
static int mtd_vertex(const real* e, const real* p, real* n, real* depth, int* ill) {
  const real s2[3] = {e[0] * e[0], e[1] * e[1], e[2] * e[2]};
  if (!(p[0] * p[0] / s2[0] + p[1] * p[1] / s2[1] + p[2] * p[2] / s2[2] < 1.0)) return 0;
  real smin;
  const real lam = ell_root(3, s2, p, &smin);
  real g[3];
  for (int i = 0; i < 3; i++) g[i] = p[i] / (s2[i] + lam);
  const real gl = sqrt(dot3(g, g));
  if (!(gl > 0.0) || !isfinite(gl)) return 0;
  for (int i = 0; i < 3; i++) n[i] = g[i] / gl;
  *depth = -lam * gl;
  *ill = (smin + lam) < 1e-3 * smin;
  return 1;
}
static int seg_mtd(const cvx_shape* A, const real* e, real* n, real* depth, real* pa) {
  real u[3];
  int ill = 0;
  v3sub(A->p1, A->p0, u);
  const real uu = dot3(u, u);
  /* a valid vertex solution (the other end not deeper along its normal) is the minimum -- both valid: equal
   * depths -- so the first valid one is taken */
  if (mtd_vertex(e, A->p0, n, depth, &ill) && (uu == 0.0 || dot3(n, u) >= 0.0)) {
    v3cp(pa, A->p0); orc_cvx_ill = ill;
    return 1;
  }
  if (!(uu > 0.0)) return 0;
  if (mtd_vertex(e, A->p1, n, depth, &ill) && dot3(n, u) <= 0.0) {
    v3cp(pa, A->p1); orc_cvx_ill = ill;
    return 1;
  }
  /* the edge: the plane normal to u, basis (w1, w2); the shadow ellipse's matrix S = P diag(s) P^T */
  real uh[3] = {u[0], u[1], u[2]}, a[3] = {0, 0, 0}, w1[3], w2[3];
  v3unit(uh);
  const int ax = fabs(uh[0]) <= fabs(uh[1]) ? (fabs(uh[0]) <= fabs(uh[2]) ? 0 : 2) : (fabs(uh[1]) <= fabs(uh[2]) ? 1 : 2);
  a[ax] = 1.0;
  cross3(uh, a, w1);
  v3unit(w1);
  cross3(uh, w1, w2);
  const real s2[3] = {e[0] * e[0], e[1] * e[1], e[2] * e[2]};
  real S00 = 0, S01 = 0, S11 = 0;
  for (int i = 0; i < 3; i++) {
    S00 += w1[i] * w1[i] * s2[i];
    S01 += w1[i] * w2[i] * s2[i];
    S11 += w2[i] * w2[i] * s2[i];
  }
  const real tr = 0.5 * (S00 + S11), df = 0.5 * (S00 - S11), rad = sqrt(df * df + S01 * S01);
  const real l2[2] = {tr + rad, tr - rad};
  real c0 = 1.0, c1 = 0.0; /* eigenvector of l2[0] in (w1, w2), from the row without cancellation: (df + rad, S01)
                              * for df >= 0, (S01, rad - df) otherwise (l2[0] - S00 = rad - df loses all of it in fp32
                              * when S01 is small and df > 0) */
  if (rad > 1e-30) {
    const real x = df >= 0 ? df + rad : S01, y = df >= 0 ? S01 : rad - df, yl = sqrt(x * x + y * y);
    if (yl > 1e-30) { c0 = x / yl; c1 = y / yl; }
  } else if (df < 0) { c0 = 0.0; c1 = 1.0; }
  const real q0 = dot3(w1, A->p0), q1 = dot3(w2, A->p0);
  const real q[2] = {c0 * q0 + c1 * q1, -c1 * q0 + c0 * q1};
  if (!(l2[1] > 0.0) || !(q[0] * q[0] / l2[0] + q[1] * q[1] / l2[1] < 1.0)) return 0;
  real smin;
  const real lam = ell_root(2, l2, q, &smin);
  const real g0 = q[0] / (l2[0] + lam), g1 = q[1] / (l2[1] + lam), gl = sqrt(g0 * g0 + g1 * g1);
  if (!(gl > 0.0) || !isfinite(gl)) return 0;
  const real m0 = (c0 * g0 - c1 * g1) / gl, m1 = (c1 * g0 + c0 * g1) / gl; /* back in (w1, w2) */
  for (int i = 0; i < 3; i++) n[i] = m0 * w1[i] + m1 * w2[i];
  *depth = -lam * gl;
  /* the core's point: the segment point nearest the ellipsoid's support point along n */
  real b[3], db[3];
  ell_support(e, n, b);
  v3sub(b, A->p0, db);
  real t = dot3(db, u) / uu;
  t = t < 0 ? 0 : (t > 1 ? 1 : t);
  for (int i = 0; i < 3; i++) pa[i] = A->p0[i] + t * u[i];
  orc_cvx_ill = (smin + lam) < 1e-3 * smin;
  return 1;
}

/* one contact between core A (+ radius rA) and the ellipsoid e, object frame: GJK when the cores are
 * apart, MPR penetration when they overlap, the centre direction if MPR degenerates.  Normal from the
 * object to A. */
static int cvx_finite(const real* p, const real* n, real d) {
  return isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]) && isfinite(n[0]) && isfinite(n[1]) && isfinite(n[2]) &&
         isfinite(d);
}

/* Exact closest points of core A and the ellipsoid (cvx_polish), from GJK's witnesses.  GJK converges linearly
 * against the curved surface and its stop rule leaves the witness direction accurate to about sqrt(GJK_REL) (the
 * fp32 kernel's 1e-6: 1e-3).  The polish solves the optimality conditions on the feature of A that holds GJK's
 * witness, by Newton's method on the ellipsoid point's Lagrange multiplier lam: b_i = e_i^2 a_i / (e_i^2 + lam),
 * so the separation a - b = lam a_i / (e_i^2 + lam) carries no cancellation at small gaps, and the egg's normal
 * at b is the direction of a_i / (e_i^2 + lam):
 *   vertex a:          sum_i b_i^2 / e_i^2 = 1                               (unknown lam)
 *   edge a0 + t u:     the same and (a - b) . u = 0                          (unknowns t, lam; 2 x 2 Newton)
 *   box face (n, h):   b = the egg's support point in -n, a = b projected onto the face (closed form)
 * An active set moves between them: a parameter that leaves its edge or face is clamped (face -> edge ->
 * vertex), and a clamped box axis through whose face the separation does not point is freed (vertex -> edge
 * -> face).  (Alternating projections between the two shapes contract the error along an edge nearly tangent
 * to the egg only by R / (R + gap) per round: measured, no use.)  The kernel (csrc/convex.hpp) runs the same
 * steps in fp32 with CVX_NEWTON iterations per solve; here each solve runs CVX_NEWTON_ORACLE. */
#ifdef ORC_FP32
#define CVX_NEWTON_ORACLE 6
#else
#define CVX_NEWTON_ORACLE 12
#endif

static real vtx_newton(const real* e2, const real* a, real lam, int iters) {
  for (int it = 0; it < iters; it++) {
    real F = -1, dF = 0;
    for (int i = 0; i < 3; i++) {
      const real q = 1 / (e2[i] + lam), t = e2[i] * a[i] * a[i] * q * q;
      F += t;
      dF -= 2 * t * q;
    }
    if (!(dF < 0)) break;
    const real ln = lam - F / dF;
    lam = ln > 0 ? ln : 0;
  }
  return lam;
}

/* (t, lam) for a(t) = a0 + t u: F1 = sum e2 a^2 q^2 - 1, F2 = (a - b) . u = sum lam q a u */
static void edge_newton(const real* e2, const real* a0, const real* u, real* t, real* lam, int iters) {
  for (int it = 0; it < iters; it++) {
    real F1 = -1, F1t = 0, F1l = 0, F2 = 0, F2t = 0, F2l = 0;
    for (int i = 0; i < 3; i++) {
      const real ai = a0[i] + *t * u[i], q = 1 / (e2[i] + *lam), w = e2[i] * ai * q * q; /* w = b_i q_i */
      F1 += ai * w;
      F1l -= 2 * ai * w * q;
      F1t += 2 * w * u[i];
      F2 += *lam * q * ai * u[i];
      F2l += u[i] * w;
      F2t += u[i] * u[i] * *lam * q;
    }
    const real det = F1t * F2l - F1l * F2t;
    if (!(det > 0)) break;
    *t += (F1l * F2 - F1 * F2l) / det;
    const real ln = *lam + (F2t * F1 - F1t * F2) / det;
    *lam = ln > 0 ? ln : 0;
  }
}

static void cvx_polish(const cvx_shape* A, const real* e, real* pa, real* pb, real* dist) {
  const int N = CVX_NEWTON_ORACLE;
  const real e2[3] = {e[0] * e[0], e[1] * e[1], e[2] * e[2]};
  real g[3] = {pb[0] / e2[0], pb[1] / e2[1], pb[2] / e2[2]};
  real dv[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
  const real gg = dot3(g, g);
  real lam = gg > 0 ? dot3(dv, g) / gg : 0;
  lam = lam > 0 ? lam : 0;
  real a[3], b[3];
  int face = 0;
  if (A->kind == 0) { /* segment: its interior, else the end on the side the interior solution left by */
    real u[3] = {A->p1[0] - A->p0[0], A->p1[1] - A->p0[1], A->p1[2] - A->p0[2]};
    const real uu = dot3(u, u);
    real w[3] = {pa[0] - A->p0[0], pa[1] - A->p0[1], pa[2] - A->p0[2]};
    real t = uu > 0 ? dot3(w, u) / uu : 0, l = lam;
    t = t < 0 ? 0 : (t > 1 ? 1 : t);
    const real t0 = t;
    if (uu > 0) edge_newton(e2, A->p0, u, &t, &l, N);
    if (uu > 0 && t > 0 && t < 1 && isfinite(t) && isfinite(l)) {
      lam = l;
    } else {
      t = (isfinite(t) ? t : t0) < 0.5 ? 0 : 1;
      for (int i = 0; i < 3; i++) a[i] = A->p0[i] + t * u[i];
      lam = vtx_newton(e2, a, lam, N);
    }
    for (int i = 0; i < 3; i++) a[i] = A->p0[i] + t * u[i];
  } else { /* box: active set over the axes clamped at +-h (sg), from GJK's witness */
    const real hmax = fmax(A->h[0], fmax(A->h[1], A->h[2])), tol = 1e-5 * hmax;
    real lc[3];
    int sg[3], done = 0;
    for (int k = 0; k < 3; k++) {
      lc[k] = A->R[0][k] * (pa[0] - A->c[0]) + A->R[1][k] * (pa[1] - A->c[1]) + A->R[2][k] * (pa[2] - A->c[2]);
      sg[k] = lc[k] >= A->h[k] - tol ? 1 : (lc[k] <= -A->h[k] + tol ? -1 : 0);
    }
    for (int pass = 0; pass < 6 && !done; pass++) {
      const int m = (sg[0] == 0) + (sg[1] == 0) + (sg[2] == 0);
      if (m == 3) { /* GJK's witness inside the box (an early stop on a simplex across it): start from the face
                     * whose outward normal is nearest the direction to the egg's witness */
        real dv[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]}, best = -1;
        int kb = 0;
        for (int k = 0; k < 3; k++) {
          const real dk = A->R[0][k] * dv[0] + A->R[1][k] * dv[1] + A->R[2][k] * dv[2];
          if (fabs(dk) > best) { best = fabs(dk); kb = k; }
        }
        const real dk = A->R[0][kb] * dv[0] + A->R[1][kb] * dv[1] + A->R[2][kb] * dv[2];
        sg[kb] = dk >= 0 ? 1 : -1;
        continue;
      }
      if (m == 2) {       /* face */
        const int k = sg[0] ? 0 : (sg[1] ? 1 : 2);
        real nf[3], mn[3];
        for (int i = 0; i < 3; i++) { nf[i] = sg[k] * A->R[i][k]; mn[i] = -nf[i]; }
        ell_support(e, mn, b);
        real bc[3] = {b[0] - A->c[0], b[1] - A->c[1], b[2] - A->c[2]};
        const real dd = dot3(nf, bc) - A->h[k];
        for (int i = 0; i < 3; i++) a[i] = b[i] - dd * nf[i];
        int moved = 0;
        for (int j = 0; j < 3; j++) {
          if (j == k) continue;
          const real lj = A->R[0][j] * (a[0] - A->c[0]) + A->R[1][j] * (a[1] - A->c[1]) + A->R[2][j] * (a[2] - A->c[2]);
          if (lj > A->h[j] || lj < -A->h[j]) { sg[j] = lj > 0 ? 1 : -1; moved = 1; }
        }
        if (moved) continue;
        face = 1;
        *dist = dd;
        done = 1;
        break;
      }
      real a0[3] = {A->c[0], A->c[1], A->c[2]};
      int jf = -1;
      for (int k = 0; k < 3; k++) {
        if (sg[k] == 0) { jf = k; continue; }
        for (int i = 0; i < 3; i++) a0[i] += sg[k] * A->h[k] * A->R[i][k];
      }
      if (m == 1) { /* edge along axis jf */
        real u[3] = {A->R[0][jf], A->R[1][jf], A->R[2][jf]}, t = lc[jf], l = lam;
        edge_newton(e2, a0, u, &t, &l, N);
        if (!(isfinite(t) && isfinite(l))) return;
        if (t > A->h[jf] || t < -A->h[jf]) { sg[jf] = t > 0 ? 1 : -1; continue; }
        lam = l;
        for (int i = 0; i < 3; i++) a[i] = a0[i] + t * u[i];
      } else { /* vertex */
        for (int i = 0; i < 3; i++) a[i] = a0[i];
        lam = vtx_newton(e2, a, lam, N);
      }
      /* optimal only if b - a (from A to the egg, along -a_i q_i) leaves A through every clamped face: an axis
       * it does not leave through is freed */
      real sv[3];
      for (int i = 0; i < 3; i++) sv[i] = -a[i] / (e2[i] + lam);
      const real sl = sqrt(dot3(sv, sv));
      int freed = 0;
      for (int k = 0; k < 3; k++) {
        if (sg[k] == 0) continue;
        const real comp = sg[k] * (A->R[0][k] * sv[0] + A->R[1][k] * sv[1] + A->R[2][k] * sv[2]);
        if (comp < -1e-6 * sl) { sg[k] = 0; freed = 1; lc[k] = 0; }
      }
      if (freed) {
        for (int k = 0; k < 3; k++) /* the free coordinates restart from the current point */
          if (sg[k] == 0) lc[k] = A->R[0][k] * (a[0] - A->c[0]) + A->R[1][k] * (a[1] - A->c[1]) + A->R[2][k] * (a[2] - A->c[2]);
        continue;
      }
      done = 1;
    }
    if (!done) return;
  }
  if (!face) {
    real sv[3];
    for (int i = 0; i < 3; i++) {
      const real q = 1 / (e2[i] + lam);
      b[i] = e2[i] * a[i] * q;
      sv[i] = lam * a[i] * q;
    }
    *dist = sqrt(dot3(sv, sv));
  }
  if (!(isfinite(a[0]) && isfinite(a[1]) && isfinite(a[2]) && isfinite(b[0]) && isfinite(b[1]) && isfinite(b[2]) &&
        isfinite(*dist)))
    return;
  for (int i = 0; i < 3; i++) { pa[i] = a[i]; pb[i] = b[i]; }
}

static void cvx_contact(const cvx_shape* A0, real rA, const real* e, real cut, real* pt, real* nrm,
                        real* d) {
  real pa[3], pb[3], dist, x[3];
  /* a box core is rounded by a 1 mm margin (at most half its smallest half extent): GJK then resolves
   * penetrations shallower than the margin (resting contacts), and MPR only runs for deeper ones */
  cvx_shape As = *A0;
  const cvx_shape* A = &As;
  if (As.kind == 1) {
    const real mg = fmin(CVX_MARGIN, 0.5 * fmin(As.h[0], fmin(As.h[1], As.h[2])));
    for (int a = 0; a < 3; a++) As.h[a] -= mg;
    rA += mg;
  }
  real sp[3];
  orc_cvx_ill = 0;
  const int g = cvx_core_point(A, e, sp) ? 0 : cvx_gjk(A, e, rA + cut, pa, pb, &dist); /* overlap: MPR */
  if (g == 2) { /* farther than rA + cut: only the (lower-bound) distance is meaningful */
    *d = dist - rA;
    nrm[0] = nrm[1] = 0; nrm[2] = 1;
    pt[0] = pt[1] = pt[2] = 0;
    return;
  }
  if (g && dist > 1e-9) {
    cvx_polish(A, e, pa, pb, &dist);
    /* the normal is the egg's surface normal at its witness point (the gradient of the implicit
     * function): better conditioned than (pa - pb) / dist when the gap is small */
    real gr[3] = {pb[0] / (e[0] * e[0]), pb[1] / (e[1] * e[1]), pb[2] / (e[2] * e[2])};
    real gl2 = dot3(gr, gr);
    for (int a = 0; a < 3; a++) nrm[a] = gl2 > 1e-30 ? gr[a] / sqrt(gl2) : (pa[a] - pb[a]) / dist;
    for (int a = 0; a < 3; a++) pt[a] = 0.5 * ((pa[a] - nrm[a] * rA) + pb[a]);
    *d = dist - rA;
    if (cvx_finite(pt, nrm, *d)) return;
  } else if (A->kind == 0) { /* a segment core: the exact penetration (no MPR fallback, as the kernel) */
    if (seg_mtd(A, e, nrm, &dist, pa)) {
      for (int a = 0; a < 3; a++) pt[a] = pa[a] + 0.5 * dist * nrm[a] - 0.5 * rA * nrm[a];
      *d = -dist - rA;
      if (cvx_finite(pt, nrm, *d)) return;
    }
  } else if (cvx_mpr(A, e, x, pa)) {
    real l = sqrt(dot3(x, x));
    if (l > 1e-9) {
      for (int a = 0; a < 3; a++) {
        nrm[a] = -x[a] / l;
        pt[a] = pa[a] - 0.5 * x[a] - nrm[a] * rA * 0.5;
      }
      *d = -l - rA;
      orc_cvx_ill = l < NORMAL_ILL;
      if (cvx_finite(pt, nrm, *d)) return;
    }
  }
  /* MPR degenerate, or a non-finite result of a degenerate simplex: the centre direction */
  real ca[3];
  if (A->kind == 0) for (int a = 0; a < 3; a++) ca[a] = 0.5 * (A->p0[a] + A->p1[a]);
  else for (int a = 0; a < 3; a++) ca[a] = A->c[a];
  real l = sqrt(dot3(ca, ca));
  if (l > 1e-12) for (int a = 0; a < 3; a++) nrm[a] = ca[a] / l;
  else { nrm[0] = 0; nrm[1] = 0; nrm[2] = 1; }
  for (int a = 0; a < 3; a++) pt[a] = 0.5 * ca[a];
  *d = -rA;
}

/* ---- the convex-mesh hull against the object's core, exactly (ShadowHand block / pen) --
 * The vertex-face candidates above (hull vertices against the object, the object's vertices / end spheres
 * against the hull's faces) miss the configurations whose closest features are both interior: a cube edge
 * across a hull edge, the pen across a ridge of the hull, the pen lying across a face its ends overhang.
 *
 * GJK on the Minkowski difference hull - core in the hull's geom frame, fp64: A = the hull (support: its
 * vertices, ties to the lowest index), B = the object's core: the cube shrunk by HULL_MARGIN and rounded by it
 * (the rounded core finds the features; an edge-edge contact is then placed on the sharp edges), or the pen's segment with the
 * pen's radius.  When the cores overlap, MPR from the interior point (hull vertex centroid - core centre) gives
 * the penetration (so with the 1 mm rounding a cube resting up to 1 mm deep stays with GJK, whose closest
 * features are unique; MPR's portal point is not).  The features at the witnesses decide: on the hull, the planes within HULL_FEAT_EPS of the
 * hull witness (1 = a face, 2 = an edge: their cross product its direction, >= 3 = a vertex); on the core, the
 * box's face planes through its witness (1, 2, 3), or the segment parameter (an end or the interior).
 *   * edge against edge: one contact, unless the edges are within 5 deg of parallel or one
 *     edge is within 2 deg of parallel to a face of the other shape (then the closest pair is not unique and
 *     the configuration is an edge lying on a face, whose ends are vertex-face candidates; for the pen, the
 *     face case below);
 *   * the pen's interior over a hull face (the face, or a face of the witness edge the pen lies parallel to):
 *     the segment, projected onto the face's plane, is clipped by every other plane of the hull to the part
 *     over the face, [t0, t1]; each end strictly inside the segment (an end of the pen over the face is its end
 *     sphere's candidate) is a contact with the face's normal and its own plane gap.  A pen lying flat across a
 *     face rests on two points, and the contacts move continuously with the pose;
 *   * anything else has a vertex among its closest features: the vertex-face candidates' case.
 * Normal from the object to the hull, point halfway between the surfaces. */
#define HULL_MAXV 256
#define HULL_MARGIN 1e-3       /* rounding of the cube's core against the hull (m) */
#define HULL_FEAT_EPS 1e-6     /* a witness lies on a plane within this (m) */
#define HULL_SIN_PARALLEL 0.0871557427476582  /* sin 5 deg: edges closer to parallel are no edge-edge contact */
#define HULL_SIN_ON_FACE 0.0348994967025010   /* sin 2 deg: an edge closer to a face's plane lies on the face */
#define HULL_CLIP_EPS 1e-9     /* slack of the face clipping (m) */
#define HULL_COS_COPLANAR 0.9999619230641713  /* cos 0.5 deg: planes this close to parallel are one face */
static void hull_support(const real (*hv)[3], int nv, const cvx_shape* B, const real* d, real* w) {
  real best = -1e300;
  int bi = 0;
  for (int v = 0; v < nv; v++) {
    const real s = hv[v][0] * d[0] + hv[v][1] * d[1] + hv[v][2] * d[2];
    if (s > best) { best = s; bi = v; }
  }
  real nd[3] = {-d[0], -d[1], -d[2]}, b[3];
  cvx_support(B, nd, b);
  for (int a = 0; a < 3; a++) w[a] = hv[bi][a] - b[a];
  (void)0;
}
/* the hull-side support point (the vertex) of direction d: GJK / MPR keep it for the witness */
static void hull_vertex_of(const real (*hv)[3], int nv, const real* d, real* o) {
  real best = -1e300;
  int bi = 0;
  for (int v = 0; v < nv; v++) {
    const real s = hv[v][0] * d[0] + hv[v][1] * d[1] + hv[v][2] * d[2];
    if (s > best) { best = s; bi = v; }
  }
  v3cp(o, hv[bi]);
}
/* 2 = farther than cut, 1 = separated (pa, pb: hull / core witnesses, dist), 0 = overlapping */
static int hull_gjk(const real (*hv)[3], int nv, const real* v0, const cvx_shape* B, real cut, real* pa, real* pb,
                    real* dist) {
  real W[4][3], P[4][3], v[3] = {v0[0], v0[1], v0[2]};
  if (dot3(v, v) < 1e-20) { v[0] = 0; v[1] = 0; v[2] = 1; }
  int n = 0;
  real vv = dot3(v, v);
  real lam[4] = {0, 0, 0, 0};
  for (int it = 0; it < 64; it++) {
    real nd[3] = {-v[0], -v[1], -v[2]}, w[3], a[3];
    hull_support(hv, nv, B, nd, w);
    const real vw = dot3(v, w);
    if (vw > 0 && vw * vw > vv * cut * cut) {
      *dist = vw / sqrt(vv);
      return 2;
    }
    if (n > 0 && vv - vw <= 1e-10 * vv + 1e-24) break;
    int dup = 0;
    for (int i = 0; i < n; i++) {
      real dd[3] = {W[i][0] - w[0], W[i][1] - w[1], W[i][2] - w[2]};
      if (dot3(dd, dd) <= 1e-24) dup = 1;
    }
    if (dup) break;
    hull_vertex_of(hv, nv, nd, a);
    for (int k = 0; k < 3; k++) { W[n][k] = w[k]; P[n][k] = a[k]; }
    n++;
    if (cvx_simplex(W, P, &n, v, lam)) return 0;
    const real vn = dot3(v, v);
    if (vn <= 1e-20) return 0;
    const int stall = it > 0 && vn >= vv * (1.0 - 1e-14);
    vv = vn;
    if (stall) break;
  }
  for (int k = 0; k < 3; k++) {
    pa[k] = 0;
    for (int i = 0; i < n; i++) pa[k] += lam[i] * P[i][k];
    pb[k] = pa[k] - v[k];
  }
  *dist = sqrt(vv);
  return 1;
}
/* MPR on hull - core from the interior point v0: x = the boundary point (moving the hull by -x separates),
 * pa = the hull-side witness; 0 if the portal search degenerates */
static void hull_mpr_support(const real (*hv)[3], int nv, const cvx_shape* B, const real* d, real* w, real* a) {
  hull_support(hv, nv, B, d, w);
  hull_vertex_of(hv, nv, d, a);
}
static int hull_mpr(const real (*hv)[3], int nv, const real* v0, const cvx_shape* B, real* x, real* pa) {
  real V[5][3], Pa[5][3], dir[3];
  v3cp(V[0], v0);
  if (dot3(V[0], V[0]) < 1e-20) { V[0][0] = 1e-6; V[0][1] = 0; V[0][2] = 0; }
  for (int k = 0; k < 3; k++) dir[k] = -V[0][k];
  v3unit(dir);
  hull_mpr_support(hv, nv, B, dir, V[1], Pa[1]);
  if (dot3(V[1], dir) <= 0) return 0;
  cross3(V[0], V[1], dir);
  if (dot3(dir, dir) <= 1e-24) {
    v3cp(x, V[1]);
    v3cp(pa, Pa[1]);
    return 1;
  }
  v3unit(dir);
  hull_mpr_support(hv, nv, B, dir, V[2], Pa[2]);
  if (dot3(V[2], dir) <= 0) return 0;
  real va[3], vb[3];
  v3sub(V[1], V[0], va);
  v3sub(V[2], V[0], vb);
  cross3(va, vb, dir);
  v3unit(dir);
  if (dot3(dir, V[0]) > 0) {
    real t[3];
    v3cp(t, V[1]); v3cp(V[1], V[2]); v3cp(V[2], t);
    v3cp(t, Pa[1]); v3cp(Pa[1], Pa[2]); v3cp(Pa[2], t);
    for (int k = 0; k < 3; k++) dir[k] = -dir[k];
  }
  int it;
  for (it = 0; it < 64; it++) {
    hull_mpr_support(hv, nv, B, dir, V[3], Pa[3]);
    if (dot3(V[3], dir) <= 0) return 0;
    real c[3];
    cross3(V[1], V[3], c);
    if (dot3(c, V[0]) < -MPR_EPS) {
      v3cp(V[2], V[3]); v3cp(Pa[2], Pa[3]);
    } else {
      cross3(V[3], V[2], c);
      if (dot3(c, V[0]) < -MPR_EPS) { v3cp(V[1], V[3]); v3cp(Pa[1], Pa[3]); }
      else break;
    }
    v3sub(V[1], V[0], va);
    v3sub(V[2], V[0], vb);
    cross3(va, vb, dir);
    v3unit(dir);
  }
  if (it == 64) return 0;
  for (it = 0;; it++) {
    mpr_portal_dir(V, dir);
    if (it >= 64) return 0;
    if (dot3(V[1], dir) >= 0) break;
    hull_mpr_support(hv, nv, B, dir, V[4], Pa[4]);
    if (dot3(V[4], dir) < 0 || mpr_reached(V, dir)) return 0;
    mpr_expand(V, Pa);
  }
  for (it = 0;; it++) {
    mpr_portal_dir(V, dir);
    hull_mpr_support(hv, nv, B, dir, V[4], Pa[4]);
    if (mpr_reached(V, dir) || it >= 64) break;
    mpr_expand(V, Pa);
  }
  real lam[3];
  cvx_tri(V[1], V[2], V[3], lam);
  for (int k = 0; k < 3; k++) {
    x[k] = lam[0] * V[1][k] + lam[1] * V[2][k] + lam[2] * V[3][k];
    pa[k] = lam[0] * Pa[1][k] + lam[1] * Pa[2][k] + lam[2] * Pa[3][k];
  }
  return 1;
}
/* the pen's segment (p0 + t u, radius rB) over face f: the clipped part's inner ends as contacts */
static int hull_face_clip(const float (*pl)[4], int np, int f, const real* p0, const real* u, real rB, real off,
                          real* out) {
  const real nf[3] = {pl[f][0], pl[f][1], pl[f][2]}, df = pl[f][3];
  const real s0 = dot3(nf, p0) - df, su = dot3(nf, u);
  real q0[3], qu[3];
  for (int a = 0; a < 3; a++) { q0[a] = p0[a] - s0 * nf[a]; qu[a] = u[a] - su * nf[a]; }
  real t0 = 0.0, t1 = 1.0;
  for (int i = 0; i < np; i++) {
    if (i == f) continue;
    const real a = pl[i][0] * q0[0] + pl[i][1] * q0[1] + pl[i][2] * q0[2] - pl[i][3] - HULL_CLIP_EPS;
    const real b = pl[i][0] * qu[0] + pl[i][1] * qu[1] + pl[i][2] * qu[2];
    if (b > 0) t1 = fmin(t1, -a / b); /* a + t b <= 0 */
    else if (b < 0) t0 = fmax(t0, -a / b);
    else if (a > 0) return 0;
  }
  if (!(t0 <= t1)) return 0;
  int n = 0;
  for (int e = 0; e < 2; e++) {
    const real t = e == 0 ? t0 : t1;
    if (!(t > 1e-6 && t < 1.0 - 1e-6) || (e == 1 && t1 - t0 < 1e-9)) continue;
    const real g = s0 + t * su - rB;
    if (!(g < off)) continue;
    real* o = out + 7 * n;
    for (int a = 0; a < 3; a++) {
      o[a] = p0[a] + t * u[a] - nf[a] * (rB + 0.5 * g);
      o[3 + a] = -nf[a];
    }
    o[6] = g;
    n++;
  }
  return n;
}
/* the exact candidates in the hull's geom frame: core B (+ radius rB); up to 2 contacts (point, normal from the
 * object to the hull, gap) written to out[7 * i], their count returned */
static int hull_core_contacts_at(const real (*hv)[3], int nv, const float (*pl)[4], int np, const cvx_shape* B, real rB,
                              real off, real* out) {
  const real FE = HULL_FEAT_EPS * orc_hv.fe, SOF = HULL_SIN_ON_FACE * orc_hv.ang, SPA = HULL_SIN_PARALLEL * orc_hv.ang;
  const real COP = 1.0 - (1.0 - HULL_COS_COPLANAR) * orc_hv.cop;
  real ctr[3] = {0, 0, 0}, cb[3], v0[3], pa[3], pb[3], x[3], dist, nrm[3], pt[3], d;
  for (int v = 0; v < nv; v++)
    for (int a = 0; a < 3; a++) ctr[a] += hv[v][a];
  for (int a = 0; a < 3; a++) ctr[a] /= nv;
  if (B->kind == 0) for (int a = 0; a < 3; a++) cb[a] = 0.5 * (B->p0[a] + B->p1[a]);
  else v3cp(cb, B->c);
  v3sub(ctr, cb, v0);
  const int gk = hull_gjk(hv, nv, v0, B, rB + off, pa, pb, &dist);
  orc_hull_ill = 0;
  if (gk == 2) return 0;
  if (gk == 1) {
    if (!(dist > 1e-9)) return 0;
    orc_hull_ill = dist < NORMAL_ILL;
    for (int a = 0; a < 3; a++) {
      nrm[a] = (pa[a] - pb[a]) / dist;
      pt[a] = 0.5 * (pa[a] + pb[a] + nrm[a] * rB);
    }
    d = dist - rB;
  } else {
    if (!hull_mpr(hv, nv, v0, B, x, pa)) return 0;
    const real l = sqrt(dot3(x, x));
    if (!(l > 1e-9)) return 0;
    for (int a = 0; a < 3; a++) {
      nrm[a] = -x[a] / l;
      pb[a] = pa[a] - x[a];
      pt[a] = pa[a] - 0.5 * x[a] + 0.5 * nrm[a] * rB;
    }
    d = -l - rB;
  }
  if (!cvx_finite(pt, nrm, d)) return 0;
  /* no contact can be made at or beyond the offset: a face-clip gap is at least the distance, and the cube's
   * sharp edge is at most (sqrt2 - 1) of its rounding nearer than the rounded core */
  if (!(d - (B->kind == 1 ? 0.41422 * rB : 0.0) < off)) return 0;
  /* the hull's features at pa: the planes through it (the first two kept).  A plane within 0.5 deg of one already
   * kept is the same face (the one pa lies nearer to is kept): qhull triangulates the curved forearm mesh into
   * facets a fraction of a degree apart, and a witness on such a seam lies on two planes without being on an edge */
  int kA = 0, fa[2] = {0, 0};
  real fd[2] = {0, 0};
  for (int i = 0; i < np; i++) {
    const real di = fabs(pl[i][0] * pa[0] + pl[i][1] * pa[1] + pl[i][2] * pa[2] - pl[i][3]);
    if (di < FE) {
      int same = -1;
      for (int j = 0; j < (kA < 2 ? kA : 2); j++) {
        const real c = pl[i][0] * pl[fa[j]][0] + pl[i][1] * pl[fa[j]][1] + pl[i][2] * pl[fa[j]][2];
        if (same < 0 && c > COP) same = j;
      }
      if (same >= 0) {
        /* the nearer of the two is the face that clips the segment (orc_hv.seam 1 / 2: the later / the earlier
         * plane whatever the distances -- a segment parallel to the seam's facets has its witness on the seam,
         * where fp32 and fp64 GJK can land on either side) */
        const int take = orc_hv.seam == 1 ? 1 : (orc_hv.seam == 2 ? 0 : di < fd[same]);
        if (take) { fa[same] = i; fd[same] = di; }
        continue;
      }
      if (kA < 2) { fa[kA] = i; fd[kA] = di; }
      kA++;
    }
  }
  if (kA == 0 || kA >= 3) return 0; /* a hull vertex (or a witness off the surface) */
  /* the core's feature at pb: the edge direction ub (0 for a box face / vertex or a segment end) */
  real ub[3] = {0, 0, 0}, u[3];
  int kB;
  if (B->kind == 0) {
    v3sub(B->p1, B->p0, u);
    const real uu = dot3(u, u);
    real dp[3];
    v3sub(pb, B->p0, dp);
    const real t = uu > 0 ? dot3(dp, u) / uu : 0.0;
    if (!(t * sqrt(uu) > FE && (1.0 - t) * sqrt(uu) > FE)) return 0; /* an end */
    v3cp(ub, u);
    kB = 2;
  } else {
    real dl[3], l[3];
    v3sub(pb, B->c, dl);
    mattvec3((real(*)[3])B->R, dl, l);
    kB = 0;
    int free_ax = -1;
    for (int k = 0; k < 3; k++) {
      if (fabs(l[k]) > B->h[k] - FE) kB++;
      else free_ax = k;
    }
    if (kB != 2) return 0; /* a face of the box (an edge of the hull lying on it) or a corner */
    for (int a = 0; a < 3; a++) ub[a] = B->R[a][free_ax];
  }
  const real lub = sqrt(dot3(ub, ub));
  /* the pen's interior parallel to a face of the hull at the witness: the face case */
  int face = -1;
  real falign = -2.0;
  for (int i = 0; i < kA; i++) { /* the parallel face best aligned with the contact normal */
    const real nn[3] = {pl[fa[i]][0], pl[fa[i]][1], pl[fa[i]][2]};
    const real al = -dot3(nn, nrm);
    if (fabs(dot3(nn, ub)) < SOF * lub && al > falign) { face = fa[i]; falign = al; }
  }
  if (face >= 0 || kA == 1) {
    if (B->kind != 0) return 0; /* a box edge on a hull face: its ends are vertex-face candidates */
    /* the face that clips: among the planes within the coplanar angle of the witness's face, the one highest at
     * the segment's midpoint (on a convex hull: the facet under it).  A segment lying parallel to near-coplanar
     * facets has its witness anywhere along them -- fp32 and fp64 GJK end on different facets -- and its
     * midpoint does not move with the witness */
    const int f0 = face >= 0 ? face : fa[0];
    real mid[3], bv = -1e30, sv = -1e30;
    int fc = f0;
    for (int a = 0; a < 3; a++) mid[a] = B->p0[a] + 0.5 * u[a];
    for (int i = 0; i < np; i++) {
      if (pl[i][0] * pl[f0][0] + pl[i][1] * pl[f0][1] + pl[i][2] * pl[f0][2] <= COP) continue;
      const real v = pl[i][0] * mid[0] + pl[i][1] * mid[1] + pl[i][2] * mid[2] - pl[i][3];
      if (v > bv) { sv = bv; bv = v; fc = i; }
      else if (v > sv) sv = v;
    }
    orc_hv.face = fc;
    orc_hv.marg = bv - sv;
    return hull_face_clip(pl, np, fc, B->p0, u, rB, off, out);
  }
  /* edge against edge: the hull edge's direction, the core edge not near parallel to it nor to the box's faces */
  const real n1[3] = {pl[fa[0]][0], pl[fa[0]][1], pl[fa[0]][2]}, n2[3] = {pl[fa[1]][0], pl[fa[1]][1], pl[fa[1]][2]};
  real ua[3], cx[3];
  cross3(n1, n2, ua);
  cross3(ua, ub, cx);
  if (!(dot3(cx, cx) > SPA * SPA * dot3(ua, ua) * dot3(ub, ub))) return 0;
  if (B->kind == 1) /* the hull edge lying on a face of the box: the hull edge's ends are vertex candidates */
    for (int k = 0; k < 3; k++) {
      const real col[3] = {B->R[0][k], B->R[1][k], B->R[2][k]};
      if (fabs(dot3(col, ub)) < 0.5 && fabs(dot3(col, ua)) < SOF * sqrt(dot3(ua, ua))) {
        /* col is a face normal of the box adjacent to its witness edge */
        real dl[3], l[3];
        v3sub(pb, B->c, dl);
        mattvec3((real(*)[3])B->R, dl, l);
        if (fabs(l[k]) > B->h[k] - FE) return 0;
      }
    }
  if (B->kind == 1) {
    /* the cube's sharp edge: the core edge moved out by the margin along its two faces' normals; the contact on
     * the common perpendicular of the hull edge's line (pa, ua) and that edge's line (q, ub) */
    real dl[3], l[3], q[3];
    v3sub(pb, B->c, dl);
    mattvec3((real(*)[3])B->R, dl, l);
    v3cp(q, pb);
    for (int k = 0; k < 3; k++) {
      if (!(fabs(l[k]) > B->h[k] - FE)) continue;
      const real sg = l[k] < 0 ? -rB : rB;
      for (int a = 0; a < 3; a++) q[a] += sg * B->R[a][k];
    }
    real np_[3], w0[3];
    cross3(ua, ub, np_);
    v3unit(np_);
    if (dot3(np_, nrm) < 0) for (int a = 0; a < 3; a++) np_[a] = -np_[a];
    v3sub(pa, q, w0);
    const real a_ = dot3(ua, ua), b_ = dot3(ua, ub), c_ = dot3(ub, ub), d_ = dot3(ua, w0), e_ = dot3(ub, w0);
    const real den = a_ * c_ - b_ * b_;
    const real sa = (b_ * e_ - c_ * d_) / den, tb = (a_ * e_ - b_ * d_) / den;
    for (int a = 0; a < 3; a++) {
      pt[a] = 0.5 * ((pa[a] + sa * ua[a]) + (q[a] + tb * ub[a]));
      nrm[a] = np_[a];
    }
    d = dot3(w0, np_);
  }
  if (!(d < off)) return 0;
  v3cp(out, pt);
  v3cp(out + 3, nrm);
  out[6] = d;
  return 1;
}
/* hull_core_contacts_at with the build's thresholds.  Under orc_step_flips it also runs with every decision
 * threshold moved within its band -- HULL_FEAT_EPS x0.5 / x2, the parallel / on-face angles and the coplanar
 * angle x0.98 / x1.02, either facet of a near-coplanar seam -- and marks the pair (orc_amb_pend, bit 16) when any
 * of them changes the contacts, or when the face case's clipping facet is a near tie at the segment's midpoint:
 * the decision is then one fp32 can take either way */
static int hull_core_contacts(const real (*hv)[3], int nv, const float (*pl)[4], int np, const cvx_shape* B, real rB,
                              real off, real* out) {
  orc_hv.face = -1;
  const int nc = hull_core_contacts_at(hv, nv, pl, np, B, rB, off, out);
  if (orc_tie_delta < 0.0) return nc;
  const int ill = orc_hull_ill, f = orc_hv.face;   /* orc_hv.marg: that face's margin (below) */
  /* the face case: the midpoint within HULL_FEAT_EPS of the seam between the two highest facets */
  if (f >= 0 && nc > 0 && orc_hv.marg < HULL_FEAT_EPS) orc_amb_pend = 1;
  static const double var[8][4] = {{0.5, 1, 1, 0}, {2, 1, 1, 0}, {1, 0.98, 1, 0}, {1, 1.02, 1, 0},
                                   {1, 1, 0.98, 0}, {1, 1, 1.02, 0}, {1, 1, 1, 1}, {1, 1, 1, 2}};
  for (int k = 0; k < 8 && !orc_amb_pend; k++) {
    real o2[14];
    orc_hv.fe = var[k][0]; orc_hv.ang = var[k][1]; orc_hv.cop = var[k][2]; orc_hv.seam = (int)var[k][3];
    const int n2 = hull_core_contacts_at(hv, nv, pl, np, B, rB, off, o2);
    int same = n2 == nc;
    for (int i = 0; same && i < 7 * nc; i++) same = fabs(o2[i] - out[i]) <= 1e-12;
    if (!same) orc_amb_pend = 1;
  }
  orc_hv.fe = orc_hv.ang = orc_hv.cop = 1.0;
  orc_hv.seam = 0;
  orc_hull_ill = ill;
  return nc;
}
/* the object's core in the hull's geom frame (centre c, axes R) */
static void hull_object_core(const mg_model* m, const kin* k, const real* c, real R[3][3], cvx_shape* B, real* rB) {
  memset(B, 0, sizeof(*B));
  real dl[3];
  if (m->obj_type == MG_GT_BOX) {
    B->kind = 1;
    for (int a = 0; a < 3; a++) dl[a] = k->op[a] - c[a];
    mattvec3(R, dl, B->c);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) B->R[a][b] = R[0][a] * k->oR[0][b] + R[1][a] * k->oR[1][b] + R[2][a] * k->oR[2][b];
    const real h0 = m->obj_size[0], h1 = m->obj_size[1], h2 = m->obj_size[2];
    const real mg = fmin(HULL_MARGIN, 0.5 * fmin(h0, fmin(h1, h2)));
    B->h[0] = h0 - mg; B->h[1] = h1 - mg; B->h[2] = h2 - mg;
    *rB = mg;
  } else { /* pen: segment along the object's z, half length obj_size[1], radius obj_size[0] */
    B->kind = 0;
    real e0[3], e1[3];
    for (int a = 0; a < 3; a++) {
      e0[a] = k->op[a] - k->oR[a][2] * m->obj_size[1] - c[a];
      e1[a] = k->op[a] + k->oR[a][2] * m->obj_size[1] - c[a];
    }
    mattvec3(R, e0, B->p0);
    mattvec3(R, e1, B->p1);
    *rB = m->obj_size[0];
  }
}
static int hull_object_exact(const mg_model* m, const kin* k, int g, const real* c, real R[3][3], real off,
                             contact* out, int n, int cap) {
  real hv[HULL_MAXV][3], res[14];
  const int nv = m->hull_num_verts < HULL_MAXV ? m->hull_num_verts : HULL_MAXV;
  for (int v = 0; v < nv; v++)
    for (int a = 0; a < 3; a++) hv[v][a] = m->hull_vert[v][a];
  cvx_shape B;
  real rB;
  hull_object_core(m, k, c, R, &B, &rB);
  const int nc = hull_core_contacts((const real(*)[3])hv, nv, m->hull_plane, m->hull_num_planes, &B, rB, off, res);
  for (int i = 0; i < nc; i++) {
    real pw[3], nw[3];
    matvec3(R, res + 7 * i, pw);
    for (int a = 0; a < 3; a++) pw[a] += c[a];
    matvec3(R, res + 7 * i + 3, nw);
    orc_ill_next = orc_hull_ill;
    n = push_contact(out, n, cap, m->geom_node[g], g, OBJ_NODE, -2, pw, nw, res[7 * i + 6]);
  }
  return n;
}

/* number of object-contact candidates of an articulation geom (the HIP kernel enumerates the same) */
static int obj_candidates(int otype, int gtype, int hull_verts) {
  const int round = gtype == MG_GT_SPHERE || gtype == MG_GT_CAPSULE;
  if (gtype == MG_GT_CONVEX) /* block: hull vertices + the box's 8 + exact; pen: hull vertices + its 2 ends + exact;
                                egg: planes */
    return otype == MG_GT_BOX ? hull_verts + 9 : (otype == MG_GT_CAPSULE ? hull_verts + 3 : 1);
  if (!round && gtype != MG_GT_BOX) return 0;
  if (otype == MG_GT_BOX) return round ? 1 : 17; /* box: 8 + 8 vertex-face, 1 edge-edge */
  if (otype == MG_GT_CAPSULE) return round ? 1 : 3;
  return 1; /* ellipsoid */
}

/* hand geom g (A) vs the egg / pen object (B); normal points from the object to the geom */
static int geom_object_convex(const mg_model* m, const kin* k, int g, real off, contact* out, int n, int cap) {
  const int nd = m->geom_node[g], ty = m->geom_type[g], ot = m->obj_type;
  const real os[3] = {m->obj_size[0], m->obj_size[1], m->obj_size[2]};
  real c[3], R[3][3];
  geom_world(m, k, g, c, R);
  const int round = ty == MG_GT_SPHERE || ty == MG_GT_CAPSULE;
  if (!round && ty != MG_GT_BOX && ty != MG_GT_CONVEX) return n;
  real pw[3], nw[3];
  if (ty == MG_GT_CONVEX) {
    const real hg[3] = {m->geom_size[g][0], m->geom_size[g][1], m->geom_size[g][2]};
    const real orad = ot == MG_GT_ELLIPSOID ? fmax(os[0], fmax(os[1], os[2])) : os[0] + os[1];
    if (!hull_box_near(c, R, hg, k->op, orad, off)) return n;
    if (ot == MG_GT_ELLIPSOID) {
      /* egg: the hull's face planes against the ellipsoid's support points (the plane distance of the egg's
       * point farthest along -n_f, largest over the faces): exact where a hull face is the nearest feature,
       * a lower bound near hull edges; normal minus that face's normal, point halfway across the gap */
      real cl[3], dl[3];
      for (int a = 0; a < 3; a++) dl[a] = k->op[a] - c[a];
      mattvec3(R, dl, cl); /* egg centre, geom frame */
      real Rl[3][3]; /* egg axes in the geom frame: R^T oR */
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Rl[a][b] = R[0][a] * k->oR[0][b] + R[1][a] * k->oR[1][b] + R[2][a] * k->oR[2][b];
      real best = -1e300, bs[3] = {0, 0, 0};
      int bf = 0;
      for (int f = 0; f < m->hull_num_planes; f++) {
        const float* q = m->hull_plane[f];
        real ne[3]; /* -n_f in the egg frame */
        for (int b = 0; b < 3; b++) ne[b] = -(Rl[0][b] * q[0] + Rl[1][b] * q[1] + Rl[2][b] * q[2]);
        real se[3], sg[3];
        ell_support(os, ne, se);
        matvec3(Rl, se, sg);
        for (int a = 0; a < 3; a++) sg[a] += cl[a];
        const real sd = q[0] * sg[0] + q[1] * sg[1] + q[2] * sg[2] - q[3];
        if (sd > best) { best = sd; bf = f; bs[0] = sg[0]; bs[1] = sg[1]; bs[2] = sg[2]; }
      }
      if (best < off) {
        const real ng[3] = {m->hull_plane[bf][0], m->hull_plane[bf][1], m->hull_plane[bf][2]};
        real pm[3];
        for (int a = 0; a < 3; a++) pm[a] = bs[a] - 0.5 * best * ng[a];
        matvec3(R, pm, pw);
        for (int a = 0; a < 3; a++) pw[a] += c[a];
        matvec3(R, ng, nw);
        for (int a = 0; a < 3; a++) nw[a] = -nw[a];
        n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, best);
      }
      return n;
    }
    /* pen: the hull's vertices against the pen's segment, then the pen's end spheres against the faces */
    const real ro = os[0];
    real p0[3], p1[3];
    for (int a = 0; a < 3; a++) { p0[a] = k->op[a] - k->oR[a][2] * os[1]; p1[a] = k->op[a] + k->oR[a][2] * os[1]; }
    for (int v = 0; v < m->hull_num_verts; v++) {
      real l[3] = {m->hull_vert[v][0], m->hull_vert[v][1], m->hull_vert[v][2]}, w[3], s, t, q[3], dv[3];
      matvec3(R, l, w);
      for (int a = 0; a < 3; a++) w[a] += c[a];
      closest_seg_seg(w, w, p0, p1, &s, &t);
      for (int a = 0; a < 3; a++) { q[a] = p0[a] + t * (p1[a] - p0[a]); dv[a] = w[a] - q[a]; }
      const real dist = sqrt(dot3(dv, dv)), d = dist - ro;
      if (d < off && dist > 1e-9) {
        for (int a = 0; a < 3; a++) {
          nw[a] = dv[a] / dist;
          pw[a] = 0.5 * (w[a] + (q[a] + nw[a] * ro));
        }
        orc_ill_next = dist < NORMAL_ILL;   /* a hull vertex against the segment: a point */
        n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
      }
    }
    for (int e = 0; e < 2; e++) {
      const real* pe = e == 0 ? p0 : p1;
      real dl[3], pl[3];
      for (int a = 0; a < 3; a++) dl[a] = pe[a] - c[a];
      mattvec3(R, dl, pl);
      int f;
      const real d = point_hull(m, pl, &f) - ro;
      if (d < off) {
        const real ng[3] = {m->hull_plane[f][0], m->hull_plane[f][1], m->hull_plane[f][2]};
        real pm[3];
        for (int a = 0; a < 3; a++) pm[a] = pl[a] - (ro + 0.5 * d) * ng[a];
        matvec3(R, pm, pw);
        for (int a = 0; a < 3; a++) pw[a] += c[a];
        matvec3(R, ng, nw);
        for (int a = 0; a < 3; a++) nw[a] = -nw[a];
        n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
      }
    }
    /* the pen's segment interior across the hull (a ridge, or a face its ends overhang): exact distance */
    return hull_object_exact(m, k, g, c, R, off, out, n, cap);
  }
  if (ot == MG_GT_ELLIPSOID) {
    cvx_shape A;
    memset(&A, 0, sizeof(A));
    real r = 0.0;
    if (round) {
      real hl = ty == MG_GT_CAPSULE ? m->geom_size[g][1] : 0.0, aw[3], bw[3];
      for (int a = 0; a < 3; a++) { aw[a] = c[a] - R[a][2] * hl; bw[a] = c[a] + R[a][2] * hl; }
      A.kind = 0;
      to_obj(k, aw, A.p0);
      to_obj(k, bw, A.p1);
      r = m->geom_size[g][0];
    } else {
      A.kind = 1;
      to_obj(k, c, A.c);
      real Rt[3][3];
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Rt[a][b] = k->oR[b][a];
      matmul3(Rt, R, A.R);
      for (int a = 0; a < 3; a++) A.h[a] = m->geom_size[g][a];
    }
    real pl[3], nl[3], d;
    cvx_contact(&A, r, os, off, pl, nl, &d);
    if (d < off) {
      from_obj_pt(k, pl, pw);
      from_obj_dir(k, nl, nw);
      orc_ill_next = orc_cvx_ill;
      n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
    }
    return n;
  }
  /* pen: capsule of radius os[0] along the object's z, half length os[1] */
  const real ro = os[0];
  real p0[3], p1[3];
  for (int a = 0; a < 3; a++) { p0[a] = k->op[a] - k->oR[a][2] * os[1]; p1[a] = k->op[a] + k->oR[a][2] * os[1]; }
  if (round) {
    real hl = ty == MG_GT_CAPSULE ? m->geom_size[g][1] : 0.0, r = m->geom_size[g][0], a0[3], a1[3];
    for (int a = 0; a < 3; a++) { a0[a] = c[a] - R[a][2] * hl; a1[a] = c[a] + R[a][2] * hl; }
    real s, t, pa[3], pb[3], dv[3];
    closest_seg_seg(a0, a1, p0, p1, &s, &t);
    for (int a = 0; a < 3; a++) {
      pa[a] = a0[a] + s * (a1[a] - a0[a]);
      pb[a] = p0[a] + t * (p1[a] - p0[a]);
      dv[a] = pa[a] - pb[a];
    }
    real dist = sqrt(dot3(dv, dv)), d = dist - r - ro;
    if (d < off && dist > 1e-9) {
      for (int a = 0; a < 3; a++) {
        nw[a] = dv[a] / dist;
        pw[a] = 0.5 * ((pa[a] - nw[a] * r) + (pb[a] + nw[a] * ro));
      }
      orc_ill_next = dist < NORMAL_ILL;
      n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
    }
    return n;
  }
  /* hand box vs the pen: the pen segment's closest point to the box, then its two ends (an end is
   * skipped when the closest point is within 1 % of the segment from it) */
  const real hg[3] = {m->geom_size[g][0], m->geom_size[g][1], m->geom_size[g][2]};
  real d0[3], P0[3], du[3], u[3];
  for (int a = 0; a < 3; a++) { d0[a] = p0[a] - c[a]; du[a] = p1[a] - p0[a]; }
  mattvec3(R, d0, P0);
  mattvec3(R, du, u);
  int inside;
  real ts = seg_box_t(P0, u, hg, &inside);
  /* the core inside the box: every candidate against the face seg_box_sat picks (q = 0 its deepest end, the
   * other end by its own depth behind that face) */
  const int face = inside ? seg_box_sat(P0, u, hg, &ts) : -1;
  for (int q = 0; q < 3; q++) {
    if ((q == 1 && ts < 0.01) || (q == 2 && ts > 0.99)) continue;
    const real t = q == 0 ? ts : (q == 1 ? 0.0 : 1.0);
    real P[3], nb[3], cb[3], pm[3];
    for (int a = 0; a < 3; a++) P[a] = P0[a] + t * u[a];
    const real d = (inside ? box_face_point(P, hg, face, nb, cb) : point_box(P, hg, nb, cb)) - ro;
    if (d < off) {
      for (int a = 0; a < 3; a++) pm[a] = 0.5 * ((P[a] - nb[a] * ro) + cb[a]);
      matvec3(R, pm, pw);
      for (int a = 0; a < 3; a++) pw[a] += c[a];
      matvec3(R, nb, nw);
      for (int a = 0; a < 3; a++) nw[a] = -nw[a];
      orc_ill_next = !inside && orc_pb_ill;
      n = push_contact(out, n, cap, nd, g, OBJ_NODE, -2, pw, nw, d);
    }
  }
  return n;
}

/* contact order (the HIP kernel emits the same list): ground contacts of the articulation's geoms
 * in geom order, the object's box corners on the ground, self-collision pairs in pair order (capsule /
 * sphere pairs; a box against a capsule / sphere; ShadowHand's explicit MJCF pairs are frictionless), then
 * articulation geoms against the object: the convex-mesh geom, then the others in geom order */
static int collide(const mg_model* m, const mg_sim_params* p, const kin* k, contact* out, int cap) {
  int n = 0;
  real off = p->contact_offset;
  for (int g = 0; g < m->num_geoms; g++) {
    if (!(m->geom_filter[g] & MG_COLLIDE_GROUND)) continue;
    int nd = m->geom_node[g], ty = m->geom_type[g];
    real c[3], R[3][3];
    geom_world(m, k, g, c, R);
    if (ty == MG_GT_SPHERE) {
      n = sphere_plane(out, n, cap, nd, g, c, m->geom_size[g][0], off);
    } else if (ty == MG_GT_CAPSULE) {
      real hl = m->geom_size[g][1], r = m->geom_size[g][0], e[3];
      for (int s = -1; s <= 1; s += 2) {
        for (int a = 0; a < 3; a++) e[a] = c[a] + s * R[a][2] * hl;
        n = sphere_plane(out, n, cap, nd, g, e, r, off);
      }
    } else if (ty == MG_GT_CONVEX) { /* the hull's vertices (the box of geom_size culls them in the kernel) */
      for (int v = 0; v < m->hull_num_verts; v++) {
        real l[3] = {m->hull_vert[v][0], m->hull_vert[v][1], m->hull_vert[v][2]}, w[3], e[3];
        matvec3(R, l, w);
        for (int a = 0; a < 3; a++) e[a] = c[a] + w[a];
        n = sphere_plane(out, n, cap, nd, g, e, 0.0, off);
      }
    } else if (ty == MG_GT_BOX) {
      for (int corner = 0; corner < 8; corner++) {
        real l[3] = {(corner & 1 ? 1 : -1) * m->geom_size[g][0], (corner & 2 ? 1 : -1) * m->geom_size[g][1],
                       (corner & 4 ? 1 : -1) * m->geom_size[g][2]};
        real w[3], e[3];
        matvec3(R, l, w);
        for (int a = 0; a < 3; a++) e[a] = c[a] + w[a];
        n = sphere_plane(out, n, cap, nd, g, e, 0.0, off);
      }
    }
  }
  if (m->obj_type == MG_GT_BOX) {
    for (int corner = 0; corner < 8; corner++) {
      real l[3] = {(corner & 1 ? 1 : -1) * m->obj_size[0], (corner & 2 ? 1 : -1) * m->obj_size[1],
                     (corner & 4 ? 1 : -1) * m->obj_size[2]}, e[3];
      from_obj_pt(k, l, e);
      n = sphere_plane(out, n, cap, OBJ_NODE, -2, e, 0.0, off);
    }
  } else if (m->obj_type == MG_GT_CAPSULE) { /* pen: its two end spheres */
    for (int s = -1; s <= 1; s += 2) {
      real l[3] = {0.0, 0.0, s * (real)m->obj_size[1]}, e[3];
      from_obj_pt(k, l, e);
      n = sphere_plane(out, n, cap, OBJ_NODE, -2, e, m->obj_size[0], off);
    }
  } else if (m->obj_type == MG_GT_ELLIPSOID) { /* egg: its support point in -z */
    const real es[3] = {m->obj_size[0], m->obj_size[1], m->obj_size[2]};
    real dl[3] = {-k->oR[2][0], -k->oR[2][1], -k->oR[2][2]}, sl[3], e[3];
    ell_support(es, dl, sl);
    from_obj_pt(k, sl, e);
    n = sphere_plane(out, n, cap, OBJ_NODE, -2, e, 0.0, off);
  }
  /* explicit MJCF pairs: in contact from zero distance (margin 0); orc_step_flips moves that threshold too */
  const real poff = m->pair_mjcf ? orc_pair_offset : off;
  for (int pi = 0; pi < m->num_pairs; pi++) {
    int ga = m->pair[pi][0], gb = m->pair[pi][1];
    real a0[3], a1[3], b0[3], b1[3], ra, rb;
    const int sa = geom_segment(m, k, ga, a0, a1, &ra), sb = geom_segment(m, k, gb, b0, b1, &rb);
    if (sa != sb) { /* a box against a sphere / capsule (the hand's palm vs the thumb, shared.xml:39) */
      const int gx = sa ? gb : ga;
      const real* p0 = sa ? a0 : b0;
      const real* p1 = sa ? a1 : b1;
      const real r = sa ? ra : rb;
      real c[3], R[3][3], d0[3], du[3], al[3], u[3], P[3], nb[3], cb[3], pm[3], pw[3], nw[3];
      geom_world(m, k, gx, c, R);
      const real hg[3] = {m->geom_size[gx][0], m->geom_size[gx][1], m->geom_size[gx][2]};
      for (int a = 0; a < 3; a++) { d0[a] = p0[a] - c[a]; du[a] = p1[a] - p0[a]; }
      mattvec3(R, d0, al);
      mattvec3(R, du, u);
      int inside;
      real t = seg_box_t(al, u, hg, &inside);
      const int face = inside ? seg_box_sat(al, u, hg, &t) : -1;
      for (int a = 0; a < 3; a++) P[a] = al[a] + t * u[a];
      const real d = (inside ? box_face_point(P, hg, face, nb, cb) : point_box(P, hg, nb, cb)) - r;
      if (d < poff) {
        for (int a = 0; a < 3; a++) pm[a] = 0.5 * ((P[a] - nb[a] * r) + cb[a]);
        matvec3(R, pm, pw);
        matvec3(R, nb, nw);
        for (int a = 0; a < 3; a++) { pw[a] += c[a]; nw[a] = sa ? nw[a] : -nw[a]; } /* normal from B to A */
        orc_ill_next = !inside && orc_pb_ill;
        n = push_contact(out, n, cap, m->geom_node[ga], ga, m->geom_node[gb], gb, pw, nw, d);
      }
      continue;
    }
    if (!sa) continue;
    real s, t, pa[3], pb[3], dv[3];
    closest_seg_seg(a0, a1, b0, b1, &s, &t);
    for (int a = 0; a < 3; a++) {
      pa[a] = a0[a] + s * (a1[a] - a0[a]);
      pb[a] = b0[a] + t * (b1[a] - b0[a]);
      dv[a] = pa[a] - pb[a];
    }
    real dist = sqrt(dot3(dv, dv));
    real d = dist - ra - rb;
    if (d < poff && dist > 1e-9) {
      real nrm[3] = {dv[0] / dist, dv[1] / dist, dv[2] / dist}, pt[3];
      for (int a = 0; a < 3; a++) pt[a] = 0.5 * (pa[a] - ra * nrm[a] + pb[a] + rb * nrm[a]);
      orc_ill_next = dist < NORMAL_ILL;
      n = push_contact(out, n, cap, m->geom_node[ga], ga, m->geom_node[gb], gb, pt, nrm, d);
    }
  }
  /* articulation geoms against the object: the convex-mesh geom first, then the others in geom order */
  if (m->obj_type)
    for (int pass = 0; pass < 2; pass++)
      for (int g = 0; g < m->num_geoms; g++)
        if ((m->geom_filter[g] & MG_COLLIDE_OBJECT) && ((m->geom_type[g] == MG_GT_CONVEX) == (pass == 0)))
        {
          /* an ambiguous narrowphase decision marks the contacts of this geom-object pair (bit 16 when the solve
           * uses one of them); one that left the pair without any contact marks the step */
          const int n0 = n;
          orc_amb_pend = 0;
          n = m->obj_type == MG_GT_BOX ? geom_object(m, k, g, off, out, n, cap)
                                       : geom_object_convex(m, k, g, off, out, n, cap);
          if (orc_amb_pend) {
            for (int i = n0; i < n; i++) out[i].amb = 1;
            if (n == n0) orc_amb_hit = 1;
          }
          orc_amb_pend = 0;
        }
  return n;
}

static void tangent_basis(const real* n, real* t1, real* t2) {
  real a[3] = {0, 0, 0};
  if (fabs(n[0]) < 0.57735) a[0] = 1; else a[1] = 1;
  cross3(a, n, t1);
  real l = sqrt(dot3(t1, t1));
  for (int i = 0; i < 3; i++) t1[i] /= l;
  cross3(n, t1, t2);
}

/* generalized Jacobian row of a unit force `dir` at point p on nodeA (minus on nodeB); a side
 * equal to OBJ_NODE acts on the free object's columns [w; v_com] (after the articulation's) */
static void jac_row(const mg_model* m, const kin* k, int nodeA, int nodeB, const real* p, const real* dir,
                    real* J) {
  int nv = nv_of(m), nvt = nvt_of(m);
  memset(J, 0, sizeof(real) * nvt);
  real r[3], w[6];
  for (int a = 0; a < 3; a++) r[a] = p[a] - k->o[a];
  cross3(r, dir, w);
  w[3] = dir[0]; w[4] = dir[1]; w[5] = dir[2];
  for (int side = 0; side < 2; side++) {
    int node = side == 0 ? nodeA : nodeB;
    real sg = side == 0 ? 1.0 : -1.0;
    if (node == OBJ_NODE) {
      real ro[3], rxd[3];
      for (int a = 0; a < 3; a++) ro[a] = p[a] - k->op[a];
      cross3(ro, dir, rxd);
      for (int a = 0; a < 3; a++) { J[nv + a] += sg * rxd[a]; J[nv + 3 + a] += sg * dir[a]; }
      continue;
    }
    if (node < 0) continue;
    if (!m->fixed_base)
      for (int c = 0; c < 6; c++) J[c] += sg * w[c];
    for (int j = node; j > 0; j = m->parent[j]) J[dof_col(m, j)] += sg * dot6(k->S[j], w);
  }
}

/* gym AssetOptions.max_angular_velocity (humanoid.py:154; gym default 64, the object's too): after the
 * solve every link's angular velocity is held to |w| <= W.  The root first: w scaled to W, its COM
 * velocity kept.  Then in tree order (parents first) a hinge's rate qd is clamped to the interval
 * { t : |w_parent + a t| <= W } (a = the unit world axis): a link's w moves only along its own axis in
 * joint space, and that interval holds qd = 0 because the parent is already clamped.  A body made of
 * several hinge nodes is clamped node by node.  Slides carry the parent's w.  The free object: |w| <= W. */
static void clamp_ang_vel(const mg_model* m, const kin* k, real* nu) {
  const real W = m->link_max_ang_vel;
  real om[MAXN][3];
  if (W > 0.0) {
    om[0][0] = om[0][1] = om[0][2] = 0.0;
    if (!m->fixed_base) {
      real w[3] = {nu[0], nu[1], nu[2]};
      real n = sqrt(dot3(w, w));
      if (n > W) {
        real sc = W / n, wn[3], dw[3], cw[3], dv[3];
        real c[3] = {m->body_com[0][0], m->body_com[0][1], m->body_com[0][2]};
        matvec3((real(*)[3])k->R[0], c, cw);
        for (int a = 0; a < 3; a++) { wn[a] = w[a] * sc; dw[a] = w[a] - wn[a]; }
        cross3(dw, cw, dv);
        for (int a = 0; a < 3; a++) { nu[a] = wn[a]; nu[3 + a] += dv[a]; }
      }
      for (int a = 0; a < 3; a++) om[0][a] = nu[a];
    }
    for (int i = 1; i < m->num_nodes; i++) {
      const real* wp = om[m->parent[i]];
      if (m->jtype[i] == MG_JT_HINGE) {
        const real* ax = k->S[i];
        const int ci = dof_col(m, i);
        real q = nu[ci], w[3];
        for (int a = 0; a < 3; a++) w[a] = wp[a] + ax[a] * q;
        if (dot3(w, w) > W * W) {
          real b = dot3(ax, wp), disc = b * b - dot3(wp, wp) + W * W;
          real sq = sqrt(disc > 0.0 ? disc : 0.0), lo = -b - sq, hi = -b + sq;
          if (1.1920929e-7 * W * W > CAP_ILL_TOL * sq) orc_cap_hit = 1;
          q = q < lo ? lo : (q > hi ? hi : q);
          nu[ci] = q;
          for (int a = 0; a < 3; a++) w[a] = wp[a] + ax[a] * q;
        }
        for (int a = 0; a < 3; a++) om[i][a] = w[a];
      } else {
        for (int a = 0; a < 3; a++) om[i][a] = wp[a];
      }
    }
  }
  if (m->obj_type && m->obj_max_ang_vel > 0.0) {
    const int nv = nv_of(m);
    real n = sqrt(nu[nv] * nu[nv] + nu[nv + 1] * nu[nv + 1] + nu[nv + 2] * nu[nv + 2]);
    if (n > m->obj_max_ang_vel) {
      real sc = m->obj_max_ang_vel / n;
      for (int a = 0; a < 3; a++) nu[nv + a] *= sc;
    }
  }
}

/* ---------------------------------------------------------------- one substep */
typedef struct {
  real h;
  contact con[MAXC];
  int ncon;
  real lam[MAXR];
  real lmax[MAXR];    /* the largest |impulse| a row held at any visit of the sweeps */
  int nrows;
  int row_kind[MAXR]; /* 0 normal, 1 friction, 2 limit-lower, 3 limit-upper */
  int row_ref[MAXR];  /* contact index or node */
} substep_out;

/* TGS integration: positions by the accumulated sub-step displacement dq instead of h nu (root: rotation vector
 * dq[0..2] by the exponential map, origin by dq[3..5], the final twist re-expressed at the new origin; joints
 * q += dq; the free object likewise); velocities are the final nu (after the velocity sweeps and the cap) */
static void tgs_rot(const real* th, const real* q, real* out) {
  real tn = sqrt(dot3(th, th)), d[4];
  if (tn > 1e-12) {
    real sn = sin(0.5 * tn) / tn;
    d[0] = th[0] * sn; d[1] = th[1] * sn; d[2] = th[2] * sn; d[3] = cos(0.5 * tn);
  } else {
    d[0] = 0.5 * th[0]; d[1] = 0.5 * th[1]; d[2] = 0.5 * th[2]; d[3] = 1.0;
  }
  real qn[4];
  quat_mul_d(d, q, qn);
  real l = sqrt(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
  for (int a = 0; a < 4; a++) out[a] = qn[a] / l;
}
static void tgs_integrate(const mg_model* m, astate* s, const real* nu, const real* dq) {
  const int nv = nv_of(m), nn = m->num_nodes;
  if (!m->fixed_base) {
    tgs_rot(dq, s->q, s->q);
    real dp[3] = {dq[3], dq[4], dq[5]}, w[3] = {nu[0], nu[1], nu[2]}, wxdp[3];
    cross3(w, dp, wxdp);
    for (int a = 0; a < 3; a++) { s->p[a] += dp[a]; s->nu0[a] = w[a]; s->nu0[3 + a] = nu[3 + a] + wxdp[a]; }
  }
  for (int i = 1; i < nn; i++) {
    s->qd[i] = nu[dof_col(m, i)];
    s->qj[i] += dq[dof_col(m, i)];
  }
  if (m->obj_type) {
    tgs_rot(dq + nv, s->oq, s->oq);
    for (int a = 0; a < 3; a++) {
      s->ow[a] = nu[nv + a];
      s->ov[a] = nu[nv + 3 + a];
      s->op[a] += dq[nv + 3 + a];
    }
  }
}

static void substep(const mg_model* m, const mg_sim_params* p, astate* s, const real* tau_act, substep_out* so) {
  int nv = nv_of(m), nvt = nvt_of(m), nn = m->num_nodes;
  real h = p->dt / p->substeps;
  so->h = h;
  kin k;
  forward_kinematics(m, s, &k);
  static __thread real M[MAXV * MAXV];
  real C[MAXV], diag[MAXN], tadd[MAXN], kk[MAXN], bb[MAXN], ref[MAXN];
  real ga = m->gravity_off ? 0.0 : 1.0;
  real g[3] = {ga * p->gravity[0], ga * p->gravity[1], ga * p->gravity[2]};
  tendon_forces(m, s, s->ttend);
  for (int i = 1; i < nn; i++) {
    dofterm t = dof_term(m, s, i);
    kk[i] = t.k; bb[i] = t.b; ref[i] = t.ref; tadd[i] = t.tadd; s->sat[i] = t.sat;
    diag[i] = m->armature[i] + h * t.b + h * h * t.k;
    /* dry joint friction (MJCF frictionloss, mg_model.frictionloss): tau = -f tanh(qd / v_s), linearly implicit:
     * tau(qd + h qdd) ~ tau(qd) - (f / v_s) sech^2(qd / v_s) h qdd */
    const real fl = m->frictionloss[i];
    if (fl > 0.0) {
      const real th = tanh(s->qd[i] / (real)MG_FRICTIONLOSS_VS);
      tadd[i] -= fl * th;
      diag[i] += h * fl / (real)MG_FRICTIONLOSS_VS * (1.0 - th * th);
    }
  }
  mass_matrix(m, &k, h, M, diag, nvt, h * m->link_ang_damping);
  bias_forces(m, &k, s, g, C, m->link_ang_damping);
  real nu[MAXV], rhs[MAXV];
  for (int c = 0; c < 6 && !m->fixed_base; c++) nu[c] = s->nu0[c];
  for (int i = 1; i < nn; i++) nu[dof_col(m, i)] = s->qd[i];
  for (int c = 0; c < nv; c++) rhs[c] = -C[c];
  for (int i = 1; i < nn; i++) {
    int ci = dof_col(m, i);
    real t = tau_act ? tau_act[i - 1] : 0.0;
    rhs[ci] += t + tadd[i] + s->ttend[i] - bb[i] * s->qd[i] - kk[i] * (s->qj[i] - ref[i] + h * s->qd[i]);
  }
  if (m->obj_type) {
    /* object block: diag(I_world, m 1); bias = [w x I w; -m g] */
    real Iw[3][3], Rt[3][3], T[3][3], Il[3][3] = {{m->obj_inertia[0], 0, 0}, {0, m->obj_inertia[1], 0},
                                                      {0, 0, m->obj_inertia[2]}};
    matmul3(k.oR, Il, T);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) Rt[a][b] = k.oR[b][a];
    matmul3(T, Rt, Iw);
    for (int a = 0; a < 3; a++) {
      for (int b = 0; b < 3; b++) M[(nv + a) * nvt + nv + b] = Iw[a][b];
      M[(nv + 3 + a) * nvt + nv + 3 + a] = m->obj_mass;
    }
    real Iwv[3], gyro[3];
    matvec3(Iw, s->ow, Iwv);
    cross3(s->ow, Iwv, gyro);
    for (int a = 0; a < 3; a++) {
      nu[nv + a] = s->ow[a];
      nu[nv + 3 + a] = s->ov[a];
      rhs[nv + a] = -gyro[a];
      rhs[nv + 3 + a] = m->obj_mass * m->obj_gravity * p->gravity[a];
    }
    real fw[3];
    if (s->of_local) matvec3(k.oR, s->of, fw);
    else for (int a = 0; a < 3; a++) fw[a] = s->of[a];
    for (int a = 0; a < 3; a++) rhs[nv + 3 + a] += fw[a];
  }
  if (cholesky(M, nvt) != 0) return;
  chol_solve(M, nvt, rhs);
  for (int c = 0; c < nvt; c++) nu[c] += h * rhs[c];
  if (m->obj_type) { /* velocity damping of the free body (gym AssetOptions angular/linear_damping) */
    real fa = 1.0 / (1.0 + h * m->obj_ang_damping), fl = 1.0 / (1.0 + h * m->obj_lin_damping);
    for (int a = 0; a < 3; a++) { nu[nv + a] *= fa; nu[nv + 3 + a] *= fl; }
  }

  /* constraint rows */
  int cap = p->max_contacts < MAXC ? p->max_contacts : MAXC;
  so->ncon = collide(m, p, &k, so->con, cap);
  static __thread real J[MAXR][MAXV], Y[MAXR][MAXV];
  real b[MAXR], W[MAXR], e0[MAXR];
  int nr = 0;
  /* TGS (p->solver_type == 1): the position iterations are sub-steps of h / N; a normal / limit row's target is
   * recomputed each sweep from its gap moved by the accumulated displacement, e = e0 + J . dq (e0 = the row's gap
   * at the substep start), with the PGS rule on h / N, and each sub-step moves the positions by (h / N) nu.  Then
   * max(N, vel_iters) velocity sweeps with the bias off (a penetrating row targets 0, a separated one -e / h) take
   * the depenetration velocity back out of nu: the position error is corrected through dq, not carried on as
   * momentum.  Friction rows target 0 throughout, as in PGS */
  const int tgs = p->solver_type == MG_SOLVER_TGS;
  const real hs = h / (p->pos_iters > 0 ? p->pos_iters : 1);
  const int n_sweeps = p->pos_iters + (tgs ? (p->vel_iters > p->pos_iters ? p->vel_iters : p->pos_iters) : 0);
  for (int c = 0; c < so->ncon; c++) {
    contact* ct = &so->con[c];
    real t1[3], t2[3];
    tangent_basis(ct->n, t1, t2);
    real deff = ct->d - p->rest_offset;
    real bn = deff >= 0 ? -deff / h : fmin(-p->baumgarte * deff / h, p->max_depen_vel);
    const real* dirs[3] = {ct->n, t1, t2};
    for (int r = 0; r < 3; r++) {
      jac_row(m, &k, ct->nodeA, ct->nodeB, ct->p, dirs[r], J[nr]);
      b[nr] = r == 0 ? bn : 0.0;
      e0[nr] = r == 0 ? deff : 0.0;
      so->row_kind[nr] = r == 0 ? 0 : 1;
      so->row_ref[nr] = c;
      nr++;
    }
  }
  for (int i = 1; i < nn; i++) {
    if (!m->limited[i]) continue;
    real dl = s->qj[i] - m->lower[i], du = m->upper[i] - s->qj[i];
    for (int side = 0; side < 2; side++) {
      real d = side == 0 ? dl : du;
      if (d >= p->limit_margin) continue;
      memset(J[nr], 0, sizeof(real) * nvt);
      J[nr][dof_col(m, i)] = side == 0 ? 1.0 : -1.0;
      b[nr] = d >= 0 ? -d / h : fmin(-p->baumgarte * d / h, p->max_depen_vel);
      e0[nr] = d;
      so->row_kind[nr] = 2 + side;
      so->row_ref[nr] = i;
      nr++;
    }
  }
  so->nrows = nr;
  for (int r = 0; r < nr; r++) {
    for (int c = 0; c < nvt; c++) Y[r][c] = J[r][c];
    chol_solve(M, nvt, Y[r]);
    real w = 0;
    for (int c = 0; c < nvt; c++) w += J[r][c] * Y[r][c];
    W[r] = w;
    so->lam[r] = 0;
    so->lmax[r] = 0;
  }
  real dq[MAXV];   /* TGS: the accumulated displacement of the sub-steps (generalized coordinates) */
  for (int c = 0; c < nvt; c++) dq[c] = 0.0;
  for (int it = 0; it < n_sweeps; it++) {
    const int vel_sweep = it >= p->pos_iters;
    for (int r = 0; r < nr; r++) {
      if (W[r] <= 1e-12) continue;
      real v = 0;
      for (int c = 0; c < nvt; c++) v += J[r][c] * nu[c];
      real tr = b[r];
      if (tgs && so->row_kind[r] != 1) {
        real ed = 0;
        for (int c = 0; c < nvt; c++) ed += J[r][c] * dq[c];
        const real e = e0[r] + ed;
        if (vel_sweep)
          tr = e >= 0 ? -e / h : 0.0;
        else
          tr = e >= 0 ? -e / hs : fmin(-p->baumgarte * e / hs, p->max_depen_vel);
      }
      real lnew = so->lam[r] + (tr - v) / W[r];
      if (so->row_kind[r] == 1) {
        real mu = p->friction;
        if (s->gmu) { /* DR: mean of the two shapes' friction (ground plane: sim friction) */
          const contact* ct = &so->con[so->row_ref[r]];
          const int g2[2] = {ct->geomA, ct->geomB};
          real sum = 0.0;
          for (int k = 0; k < 2; k++)
            sum += g2[k] >= 0 ? s->gmu[g2[k]] : (g2[k] == -2 ? s->gmu[m->num_geoms] : p->friction);
          mu = 0.5 * sum;
        }
        if (m->pair_mjcf && so->con[so->row_ref[r]].nodeB >= 0) mu = 0.0; /* explicit MJCF pair: condim 1 */
        real lim = mu * so->lam[3 * so->row_ref[r]];  /* normal row of this contact */
        lnew = lnew < -lim ? -lim : (lnew > lim ? lim : lnew);
      } else if (lnew < 0) {
        lnew = 0;
      }
      real dl = lnew - so->lam[r];
      so->lam[r] = lnew;
      if (fabs(lnew) > so->lmax[r]) so->lmax[r] = fabs(lnew);
      for (int c = 0; c < nvt; c++) nu[c] += Y[r][c] * dl;
    }
    /* TGS: the sub-step's displacement */
    if (tgs && !vel_sweep)
      for (int c = 0; c < nvt; c++) dq[c] += hs * nu[c];
  }
  clamp_ang_vel(m, &k, nu);
  if (tgs) {
    tgs_integrate(m, s, nu, dq);
    return;
  }
  /* integrate */
  if (!m->fixed_base) {
    real w[3] = {nu[0], nu[1], nu[2]}, vo[3] = {nu[3], nu[4], nu[5]};
    real pn[3];
    for (int a = 0; a < 3; a++) pn[a] = s->p[a] + h * vo[a];
    real wn = sqrt(dot3(w, w)), dq[4];
    if (wn * h > 1e-12) {
      real ha = 0.5 * wn * h, sn = sin(ha) / wn;
      dq[0] = w[0] * sn; dq[1] = w[1] * sn; dq[2] = w[2] * sn; dq[3] = cos(ha);
    } else {
      dq[0] = 0.5 * h * w[0]; dq[1] = 0.5 * h * w[1]; dq[2] = 0.5 * h * w[2]; dq[3] = 1.0;
    }
    real qn[4];
    quat_mul_d(dq, s->q, qn);
    real l = sqrt(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
    for (int a = 0; a < 4; a++) s->q[a] = qn[a] / l;
    real dp[3] = {pn[0] - s->p[0], pn[1] - s->p[1], pn[2] - s->p[2]}, wxdp[3];
    cross3(w, dp, wxdp);
    for (int a = 0; a < 3; a++) { s->p[a] = pn[a]; s->nu0[a] = w[a]; s->nu0[3 + a] = vo[a] + wxdp[a]; }
  }
  for (int i = 1; i < nn; i++) {
    s->qd[i] = nu[dof_col(m, i)];
    s->qj[i] += h * s->qd[i];
  }
  if (m->obj_type) {
    real w[3] = {nu[nv], nu[nv + 1], nu[nv + 2]}, dq[4], qn[4];
    real wn = sqrt(dot3(w, w));
    if (wn * h > 1e-12) {
      real ha = 0.5 * wn * h, sn = sin(ha) / wn;
      dq[0] = w[0] * sn; dq[1] = w[1] * sn; dq[2] = w[2] * sn; dq[3] = cos(ha);
    } else {
      dq[0] = 0.5 * h * w[0]; dq[1] = 0.5 * h * w[1]; dq[2] = 0.5 * h * w[2]; dq[3] = 1.0;
    }
    quat_mul_d(dq, s->oq, qn);
    real l = sqrt(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
    for (int a = 0; a < 4; a++) s->oq[a] = qn[a] / l;
    for (int a = 0; a < 3; a++) {
      s->ow[a] = w[a];
      s->ov[a] = nu[nv + 3 + a];
      s->op[a] += h * s->ov[a];
    }
  }
}

/* sensor wrench and dof force from the last substep's impulses */
static void sensor_outputs(const mg_model* m, const astate* s, const substep_out* so, const real* tau_act,
                           float* sensors, float* dof_force) {
  if (sensors && m->num_sensors > 0) {
    kin k;
    forward_kinematics(m, s, &k);  /* post-step pose for the body frame */
    for (int si = 0; si < m->num_sensors; si++) {
      int body = m->sensor_body[si], nd = m->body_node[body];
      real Rb[3][3], bq[4] = {m->body_quat[body][0], m->body_quat[body][1], m->body_quat[body][2],
                                 m->body_quat[body][3]}, Rl[3][3];
      quat_to_mat(bq, Rl);
      matmul3(k.R[nd], Rl, Rb);
      real bp[3] = {m->body_pos[body][0], m->body_pos[body][1], m->body_pos[body][2]}, bw[3], xb[3];
      matvec3(k.R[nd], bp, bw);
      for (int a = 0; a < 3; a++) xb[a] = k.x[nd][a] + bw[a];
      real F[3] = {0, 0, 0}, T[3] = {0, 0, 0};
      for (int c = 0; c < so->ncon; c++) {
        const contact* ct = &so->con[c];
        real sg = 0;
        if (ct->geomA >= 0 && m->geom_body[ct->geomA] == body) sg = 1;
        else if (ct->geomB >= 0 && m->geom_body[ct->geomB] == body) sg = -1;
        if (sg == 0) continue;
        real t1[3], t2[3];
        tangent_basis(ct->n, t1, t2);
        real f[3], r[3], rf[3];
        for (int a = 0; a < 3; a++)
          f[a] = sg * (so->lam[3 * c] * ct->n[a] + so->lam[3 * c + 1] * t1[a] + so->lam[3 * c + 2] * t2[a]) / so->h;
        for (int a = 0; a < 3; a++) r[a] = ct->p[a] - xb[a];
        cross3(r, f, rf);
        for (int a = 0; a < 3; a++) { F[a] += f[a]; T[a] += rf[a]; }
      }
      real Fl[3], Tl[3];
      mattvec3(Rb, F, Fl);
      mattvec3(Rb, T, Tl);
      for (int a = 0; a < 3; a++) { sensors[6 * si + a] = (float)Fl[a]; sensors[6 * si + 3 + a] = (float)Tl[a]; }
    }
  }
  if (dof_force) {
    /* drive / passive force at the post-step state (saturated drives report +-effort), tendon force
     * of the last substep, plus the joint-limit impulses / h */
    for (int i = 1; i < m->num_nodes; i++) {
      real t = (tau_act ? tau_act[i - 1] : 0.0) + s->ttend[i];
      if (m->drive_kp[i] > 0.0) {
        real tgt = s->tgt ? s->tgt[i - 1] : 0.0;
        t += s->sat[i] ? (m->drive_kp[i] * (tgt - s->qj[i]) - m->damping[i] * s->qd[i] > 0 ? m->effort_limit[i]
                                                                                                 : -m->effort_limit[i])
                       : m->drive_kp[i] * (tgt - s->qj[i]) - m->damping[i] * s->qd[i];
      } else {
        t += -m->damping[i] * s->qd[i] - m->stiffness[i] * s->qj[i];
      }
      if (m->frictionloss[i] > 0.0f) t -= m->frictionloss[i] * tanh(s->qd[i] / (real)MG_FRICTIONLOSS_VS);
      for (int r = 0; r < so->nrows; r++) {
        if (so->row_ref[r] != i) continue;
        if (so->row_kind[r] == 2) t += so->lam[r] / so->h;
        if (so->row_kind[r] == 3) t -= so->lam[r] / so->h;
      }
      dof_force[i - 1] = (float)t;
    }
  }
}

/* gym net contact forces (acquire_net_contact_force_tensor; franka_reach_MA.py:506, 563): per rigid body (the
 * articulation's bodies, then the object and the goal for hand tasks), the world-frame sum of the last substep's
 * contact impulses / h acting on it -- + on side A, - on side B of each contact (ground: no body) */
static void net_contact_forces(const mg_model* m, const substep_out* so, float* ncf) {
  const int nb = m->num_bodies, nbe = nb + (m->obj_type ? 2 : 0);
  real F[MG_MAX_BODIES + 2][3];
  memset(F, 0, sizeof(F));
  for (int c = 0; c < so->ncon; c++) {
    const contact* ct = &so->con[c];
    const int bA = ct->geomA >= 0 ? m->geom_body[ct->geomA] : (ct->geomA == -2 ? nb : -1);
    const int bB = ct->geomB >= 0 ? m->geom_body[ct->geomB] : (ct->geomB == -2 ? nb : -1);
    real t1[3], t2[3], f[3];
    tangent_basis(ct->n, t1, t2);
    for (int a = 0; a < 3; a++)
      f[a] = (so->lam[3 * c] * ct->n[a] + so->lam[3 * c + 1] * t1[a] + so->lam[3 * c + 2] * t2[a]) / so->h;
    for (int a = 0; a < 3; a++) {
      if (bA >= 0) F[bA][a] += f[a];
      if (bB >= 0) F[bB][a] -= f[a];
    }
  }
  for (int b = 0; b < nbe; b++)
    for (int a = 0; a < 3; a++) ncf[3 * b + a] = (float)F[b][a];
}

static void load_object(astate* s, const float* row) {
  real nq = 0;
  for (int a = 0; a < 3; a++) { s->op[a] = row[a]; s->ov[a] = row[7 + a]; s->ow[a] = row[10 + a]; }
  for (int a = 0; a < 4; a++) { s->oq[a] = row[3 + a]; nq += s->oq[a] * s->oq[a]; }
  nq = sqrt(nq);
  for (int a = 0; a < 4; a++) s->oq[a] /= nq;
}
static void store_object(const astate* s, float* row) {
  for (int a = 0; a < 3; a++) {
    row[a] = (float)s->op[a];
    row[7 + a] = (float)s->ov[a];
    row[10 + a] = (float)s->ow[a];
  }
  for (int a = 0; a < 4; a++) row[3 + a] = (float)s->oq[a];
}

/* gym rigid-body states of the articulation (body origin pose, COM linear velocity, angular velocity) */
static void body_states(const mg_model* m, const astate* s, float* out) {
  kin k;
  forward_kinematics(m, s, &k);
  for (int b = 0; b < m->num_bodies; b++) {
    int nd = m->body_node[b];
    real bq[4] = {m->body_quat[b][0], m->body_quat[b][1], m->body_quat[b][2], m->body_quat[b][3]}, Rl[3][3],
           Rb[3][3];
    quat_to_mat(bq, Rl);
    matmul3(k.R[nd], Rl, Rb);
    real bp[3] = {m->body_pos[b][0], m->body_pos[b][1], m->body_pos[b][2]}, bw[3], xb[3], q[4];
    matvec3(k.R[nd], bp, bw);
    for (int a = 0; a < 3; a++) xb[a] = k.x[nd][a] + bw[a];
    mat_to_quat(Rb, q);
    real cl[3] = {m->body_com[b][0], m->body_com[b][1], m->body_com[b][2]}, cw[3], r[3], wxr[3];
    matvec3(Rb, cl, cw);
    for (int a = 0; a < 3; a++) r[a] = xb[a] + cw[a] - k.o[a];
    cross3(k.V[nd], r, wxr);
    float* o = out + 13 * b;
    for (int a = 0; a < 3; a++) {
      o[a] = (float)xb[a];
      o[7 + a] = (float)(k.V[nd][3 + a] + wxr[a]);
      o[10 + a] = (float)k.V[nd][a];
    }
    for (int a = 0; a < 4; a++) o[3 + a] = (float)q[a];
  }
}

/* one env: root rows [articulation, (object, goal)], dof rows, PD targets, sensors, dof forces,
 * rigid-body rows [articulation bodies, (object, goal)] */
/* domain randomization: the model with one env_props row applied (include/migym.h layout) */
static void apply_env_props(const mg_model* m, const float* row, mg_model* mm, real* gmu) {
  *mm = *m;
  const int nn = m->num_nodes, ng = m->num_geoms, nt = m->num_tendons;
  for (int i = 0; i < nn; i++) {
    const float* r = row + MG_EP_NODE_WIDTH * i;
    const real sc = m->mass[i] > 0.0f ? (real)r[0] / (real)m->mass[i] : 1.0;
    mm->mass[i] = r[0];
    for (int k = 0; k < 6; k++) mm->inertia[i][k] = (float)((real)m->inertia[i][k] * sc);
    mm->armature[i] = r[1]; mm->damping[i] = r[2]; mm->stiffness[i] = r[3];
    mm->lower[i] = r[4]; mm->upper[i] = r[5]; mm->drive_kp[i] = r[6]; mm->effort_limit[i] = r[7];
    mm->frictionloss[i] = r[8];
  }
  const float* g = row + MG_EP_NODE_WIDTH * nn;
  for (int k = 0; k < ng; k++) gmu[k] = g[k];
  const float* t = g + ng;
  for (int q = 0; q < nt; q++) { mm->tendon_limit_stiffness[q] = t[2 * q]; mm->tendon_damping[q] = t[2 * q + 1]; }
  const float* o = t + 2 * nt;
  gmu[ng] = o[1];
  if (m->obj_type) {
    const real sc = (real)o[2], fm = (real)o[0] / (real)m->obj_mass;
    mm->obj_mass = o[0];
    for (int a = 0; a < 3; a++) {
      mm->obj_size[a] = (float)((real)m->obj_size[a] * sc);
      mm->obj_inertia[a] = (float)((real)m->obj_inertia[a] * fm * sc * sc);
    }
  }
}

static void simulate_env(const mg_model* m0, const mg_sim_params* p, float* root, float* dof, const float* act,
                         const float* tgt, float* sensors, float* dof_force, float* rbs, const float* oforce,
                         int oforce_local, const float* props, float* ncf) {
  astate s;
  memset(&s, 0, sizeof(s));
  mg_model* mdr = NULL;
  real gmu[MG_MAX_GEOMS + 1];
  const mg_model* m = m0;
  if (props) {
    mdr = (mg_model*)malloc(sizeof(mg_model));
    apply_env_props(m0, props, mdr, gmu);
    m = mdr;
    s.gmu = gmu;
  }
  load_state(m, root, dof, &s);
  s.tgt = tgt;
  if (m->obj_type) load_object(&s, root + 13);
  if (oforce)
    for (int a = 0; a < 3; a++) s.of[a] = oforce[a];
  s.of_local = oforce_local;
  real tau[MAXN];
  for (int i = 0; i < m->num_dofs; i++) tau[i] = act ? act[i] : 0.0;
  substep_out* so = (substep_out*)malloc(sizeof(substep_out));
  memset(so, 0, sizeof(*so));
  for (int st = 0; st < p->substeps; st++) substep(m, p, &s, tau, so);
  store_state(m, &s, root, dof);
  if (m->obj_type) store_object(&s, root + 13);
  sensor_outputs(m, &s, so, tau, sensors, dof_force);
  if (ncf) net_contact_forces(m, so, ncf);
  if (rbs) {
    body_states(m, &s, rbs);
    if (m->obj_type) {
      memcpy(rbs + 13 * m->num_bodies, root + 13, 13 * sizeof(float));
      memcpy(rbs + 13 * (m->num_bodies + 1), root + 26, 13 * sizeof(float));
    }
  }
  free(so);
  free(mdr);
}

int orc_simulate_views(const mg_model* m, const mg_sim_params* p, int32_t n, const mg_state_views* v,
                       int32_t threads) {
  int nd = m->num_dofs, ns = m->num_sensors;
  int rows = m->obj_type ? 3 : 1, nb = m->num_bodies + (m->obj_type ? 2 : 0);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (int e = 0; e < n; e++) {
    simulate_env(m, p, v->root_states + (size_t)13 * rows * e, v->dof_state + (size_t)2 * nd * e,
                 v->dof_actuation ? v->dof_actuation + (size_t)nd * e : 0,
                 v->dof_targets ? v->dof_targets + (size_t)nd * e : 0, v->sensors ? v->sensors + (size_t)6 * ns * e : 0,
                 v->dof_force ? v->dof_force + (size_t)nd * e : 0,
                 v->rigid_body_states ? v->rigid_body_states + (size_t)13 * nb * e : 0,
                 (m->obj_type && v->rb_forces) ? v->rb_forces + ((size_t)nb * e + m->num_bodies) * 3 : 0,
                 v->rb_force_space == MG_LOCAL_SPACE,
                 v->env_props ? v->env_props + (size_t)v->env_props_stride * e : 0,
                 v->net_contact_forces ? v->net_contact_forces + (size_t)3 * nb * e : 0);
  }
  (void)threads;
  return 0;
}

int orc_simulate(const mg_model* m, const mg_sim_params* p, int32_t n, float* root_states, float* dof_state,
                 const float* dof_actuation, float* sensors, float* dof_force, int32_t threads) {
  mg_state_views v;
  memset(&v, 0, sizeof(v));
  v.root_states = root_states;
  v.dof_state = dof_state;
  v.dof_actuation = dof_actuation;
  v.sensors = sensors;
  v.dof_force = dof_force;
  return orc_simulate_views(m, p, n, &v, threads);
}

/* contacts of one actor with both geoms: (nodeA, geomA, nodeB, geomB, p(3), n(3), d) records of 11 reals (real is
 * float in the fp32 build: diagnostics of fp32-vs-fp64 partings, tools/pair_diag.py) */
int orc_contacts_full(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2, real* out,
                      int32_t cap) {
  astate s;
  kin k;
  memset(&s, 0, sizeof(s));
  load_state(m, root13, dof2, &s);
  if (m->obj_type) load_object(&s, root13 + 13);
  forward_kinematics(m, &s, &k);
  contact con[MAXC];
  int nc = collide(m, p, &k, con, cap < MAXC ? cap : MAXC);
  for (int i = 0; i < nc; i++) {
    real* o = out + 11 * i;
    o[0] = con[i].nodeA; o[1] = con[i].geomA; o[2] = con[i].nodeB; o[3] = con[i].geomB;
    for (int a = 0; a < 3; a++) { o[4 + a] = con[i].p[a]; o[7 + a] = con[i].n[a]; }
    o[10] = con[i].d;
  }
  return nc;
}

#ifndef ORC_FP32 /* fp64 inspection hooks of the checker (KATs); not in the fp32 timing build */
/* The discontinuities of the build's physics that env `e`'s gym.simulate (state views as orc_simulate_views)
 * passes near, substep by substep (tests/parity_stats.py): an fp32 and an fp64 step of the same state may part
 * ways there, and nowhere else.  Each substep is solved once more with the thresholds moved out by `delta` (the
 * contact offset, the MJCF pairs' zero distance, the joint-limit margin), and the state advances by the normal
 * substep.  Bits:
 *   1  a contact within delta of its threshold that the solve uses (its normal impulse leaves 0 at some visit;
 *      a row whose impulse stays 0 changes nothing, so its presence or absence is no discontinuity)
 *   2  a joint-limit row within delta of the margin that the solve uses (the same rule)
 *   4  a PD drive whose explicit force is within df (relative) of its effort limit (implicit <-> saturated)
 *   8  a segment core inside a box whose two least push-out faces are within delta (seg_box_sat's tie)
 *  16  a narrowphase decision near its threshold: a hull witness 0.5-2 um from a plane, a segment end or a box
 *      face (HULL_FEAT_EPS 1 um decides the features), an edge within 2 % of the parallel / on-face angles --
 *      when the solve uses a contact of that geom-object pair, or the decision left the pair without any
 *  32  a contact in use whose normal is ill-conditioned: the direction of a core distance below NORMAL_ILL
 *      (0.5 mm) that the geometry does not pin (an end point, a box edge or corner at the closest point; an
 *      MPR or hull-GJK depth), so that a 1e-7 m difference of the state turns it by ~1e-4 rad
 *  64  the angular-velocity cap clipped a hinge rate to an ill-conditioned interval end (clamp_ang_vel) */
int orc_step_flips(const mg_model* m0, const mg_sim_params* p, const mg_state_views* v, int32_t e, double delta,
                   double df) {
  const mg_model* m = m0;
  int nd = m0->num_dofs, rows = m0->obj_type ? 3 : 1, nb = m0->num_bodies + (m0->obj_type ? 2 : 0);
  (void)nb;
  float* root = v->root_states + (size_t)13 * rows * e;
  float* dof = v->dof_state + (size_t)2 * nd * e;
  const float* act = v->dof_actuation ? v->dof_actuation + (size_t)nd * e : 0;
  const float* tgt = v->dof_targets ? v->dof_targets + (size_t)nd * e : 0;
  const float* of = (m0->obj_type && v->rb_forces) ? v->rb_forces + ((size_t)(m0->num_bodies + 2) * e + m0->num_bodies) * 3 : 0;
  const float* props = v->env_props ? v->env_props + (size_t)v->env_props_stride * e : 0;
  astate s;
  memset(&s, 0, sizeof(s));
  mg_model* mdr = NULL;
  real gmu[MG_MAX_GEOMS + 1];
  if (props) {
    mdr = (mg_model*)malloc(sizeof(mg_model));
    apply_env_props(m0, props, mdr, gmu);
    m = mdr;
    s.gmu = gmu;
  }
  load_state(m, root, dof, &s);
  s.tgt = tgt;
  if (m->obj_type) load_object(&s, root + 13);
  if (of)
    for (int a = 0; a < 3; a++) s.of[a] = of[a];
  s.of_local = v->rb_force_space == MG_LOCAL_SPACE;
  real tau[MAXN];
  for (int i = 0; i < m->num_dofs; i++) tau[i] = act ? act[i] : 0.0;
  substep_out* so = (substep_out*)calloc(1, sizeof(substep_out));
  mg_sim_params pw = *p;
  pw.contact_offset = (float)(p->contact_offset + delta);
  pw.limit_margin = (float)(p->limit_margin + delta);
  int flags = 0;
  for (int st = 0; st < p->substeps; st++) {
    /* drives near saturation at this substep's state */
    for (int i = 1; i < m->num_nodes; i++) {
      if (m->drive_kp[i] <= 0.0) continue;
      const real fe = m->drive_kp[i] * ((tgt ? tgt[i - 1] : 0.0) - s.qj[i]) - m->damping[i] * s.qd[i];
      const real lim = m->effort_limit[i];
      if (fabs(fabs(fe) - lim) < df * (lim > 1e-6 ? lim : 1e-6)) flags |= 4;
    }
    /* the solve with the thresholds moved out (its collide also reports seg_box_sat ties) */
    astate sw = s;
    orc_pair_offset = delta;
    orc_tie_delta = delta;
    orc_tie_hit = 0;
    orc_amb_hit = 0;
    orc_cap_hit = 0;
    substep(m, &pw, &sw, tau, so);
    orc_pair_offset = 0.0;
    orc_tie_delta = -1.0;
    if (orc_tie_hit) flags |= 8;
    if (orc_amb_hit) flags |= 16;
    if (orc_cap_hit) flags |= 64;
    const real eps = 1e-9;
    for (int c = 0; c < so->ncon; c++) {
      const contact* ct = &so->con[c];
      const int pair = m->pair_mjcf && ct->nodeB >= 0;
      const real thr = pair ? 0.0 : p->contact_offset;
      if (fabs(ct->d - thr) < delta && so->lmax[3 * c] > eps) flags |= 1;
      if (ct->ill && so->lmax[3 * c] > eps) flags |= 32;
      if (ct->amb && so->lmax[3 * c] > eps) flags |= 16;
    }
    for (int r = 3 * so->ncon; r < so->nrows; r++) {
      const int i = so->row_ref[r];
      const real d = so->row_kind[r] == 2 ? s.qj[i] - m->lower[i] : m->upper[i] - s.qj[i];
      if (fabs(d - p->limit_margin) < delta && so->lmax[r] > eps) flags |= 2;
    }
    substep(m, p, &s, tau, so);
  }
  free(so);
  free(mdr);
  return flags;
}

int orc_mass_matrix(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2,
                    real* M_out) {
  astate s;
  kin k;
  load_state(m, root13, dof2, &s);
  forward_kinematics(m, &s, &k);
  mass_matrix(m, &k, p->dt / p->substeps, M_out, 0, nv_of(m), 0.0);
  return nv_of(m);
}

int orc_free_acceleration(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2,
                          const float* tau, real* qacc_out) {
  astate s;
  kin k;
  load_state(m, root13, dof2, &s);
  forward_kinematics(m, &s, &k);
  int nv = nv_of(m);
  real h = p->dt / p->substeps, M[MAXV * MAXV], C[MAXV], g[3] = {p->gravity[0], p->gravity[1], p->gravity[2]};
  mass_matrix(m, &k, h, M, 0, nv, h * m->link_ang_damping);
  bias_forces(m, &k, &s, g, C, m->link_ang_damping);
  if (cholesky(M, nv) != 0) return -1;
  for (int c = 0; c < nv; c++) qacc_out[c] = -C[c];
  for (int i = 1; i < m->num_nodes; i++)
    qacc_out[dof_col(m, i)] += (tau ? tau[i - 1] : 0.0) - m->damping[i] * s.qd[i] -
                               m->stiffness[i] * (s.qj[i] + h * s.qd[i]);
  chol_solve(M, nv, qacc_out);
  return nv;
}

int orc_contacts(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2, real* out,
                 int32_t cap) {
  astate s;
  kin k;
  memset(&s, 0, sizeof(s));
  load_state(m, root13, dof2, &s);
  if (m->obj_type) load_object(&s, root13 + 13); /* env root rows [articulation, object, goal] */
  forward_kinematics(m, &s, &k);
  contact con[MAXC];
  int c = cap < MAXC ? cap : MAXC;
  int nc = collide(m, p, &k, con, c);
  for (int i = 0; i < nc; i++) {
    real* o = out + 9 * i;
    o[0] = con[i].nodeA;
    o[1] = con[i].p[0]; o[2] = con[i].p[1]; o[3] = con[i].p[2];
    o[4] = con[i].n[0]; o[5] = con[i].n[1]; o[6] = con[i].n[2];
    o[7] = con[i].d;
    o[8] = con[i].nodeB;
  }
  return nc;
}

#endif

int orc_rigid_body_states(const mg_model* m, const float* root13, const float* dof2, float* out) {
  astate s;
  memset(&s, 0, sizeof(s));
  load_state(m, root13, dof2, &s);
  body_states(m, &s, out);
  return m->num_bodies;
}

#ifndef ORC_FP32
/* KAT hook: the egg narrowphase (cvx_contact) for core A against the origin-centred ellipsoid e.
 * kind 0: shape = segment p0, p1 (6 doubles); kind 1: shape = box centre (3), axes R row-major (9),
 * half extents (3).  out = contact point (3), normal from the ellipsoid to A (3), signed distance. */
int orc_ellipsoid_contact(int32_t kind, const real* shape, real radius, const real* e, real* out) {
  cvx_shape A;
  memset(&A, 0, sizeof(A));
  A.kind = kind;
  if (kind == 0) {
    for (int a = 0; a < 3; a++) { A.p0[a] = shape[a]; A.p1[a] = shape[3 + a]; }
  } else {
    for (int a = 0; a < 3; a++) {
      A.c[a] = shape[a];
      A.h[a] = shape[12 + a];
      for (int b = 0; b < 3; b++) A.R[a][b] = shape[3 + 3 * a + b];
    }
  }
  cvx_contact(&A, radius, e, 1e300, out, out + 3, out + 6);
  return MG_OK;
}

/* KAT hook: box-box edge-edge contact (box_box_edge) in the object box's frame: shape = hand box centre (3),
 * axes R row-major (9), half extents (3); hb = object half extents.  out = point (3), normal from the object
 * to the hand box (3), separation; returns 1 when an edge-edge contact is generated. */
int orc_box_box_edge(const real* shape, const real* hb, real off, real* out) {
  real c[3], R[3][3], hg[3];
  for (int a = 0; a < 3; a++) {
    c[a] = shape[a];
    hg[a] = shape[12 + a];
    for (int b = 0; b < 3; b++) R[a][b] = shape[3 + 3 * a + b];
  }
  return box_box_edge(c, R, hg, hb, off, out, out + 3, out + 6);
}

/* KAT hook: the hull's plane distance (point_hull) of points pl (n x 3, geom frame); out = distance, face */
int orc_hull_distance(const mg_model* m, const real* pl, int32_t n, real* out) {
  for (int i = 0; i < n; i++) {
    int f;
    out[2 * i] = point_hull(m, pl + 3 * i, &f);
    out[2 * i + 1] = f;
  }
  return MG_OK;
}
#endif

/* KAT hook: the exact hull candidates (hull_core_contacts) of the model's hull against a core given in the hull's
 * geom frame: shape = [kind, p0 (3), p1 (3)] (segment) or [kind, c (3), R (9, row-major), h (3)] (box);
 * out = up to 2 x [point (3), normal (3), gap].  Returns the number of contacts. */
int orc_hull_core_contact(const mg_model* m, const double* shape, double rB, double off, double* out) {
  real hv[HULL_MAXV][3];
  const int nv = m->hull_num_verts < HULL_MAXV ? m->hull_num_verts : HULL_MAXV;
  for (int v = 0; v < nv; v++)
    for (int a = 0; a < 3; a++) hv[v][a] = m->hull_vert[v][a];
  cvx_shape B;
  memset(&B, 0, sizeof(B));
  B.kind = (int)shape[0];
  if (B.kind == 0) {
    for (int a = 0; a < 3; a++) { B.p0[a] = shape[1 + a]; B.p1[a] = shape[4 + a]; }
  } else {
    for (int a = 0; a < 3; a++) B.c[a] = shape[1 + a];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) B.R[a][b] = shape[4 + 3 * a + b];
    for (int a = 0; a < 3; a++) B.h[a] = shape[13 + a];
  }
  real res[14];
  const int nc = hull_core_contacts((const real(*)[3])hv, nv, m->hull_plane, m->hull_num_planes, &B, rB, off, res);
  for (int i = 0; i < 7 * nc; i++) out[i] = res[i];
  return nc;
}

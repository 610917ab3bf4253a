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
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXN MG_MAX_NODES
#define MAXV (MG_MAX_NODES + 6)
#define MAXC 64
#define MAXR (3 * MAXC + 2 * MG_MAX_NODES)

typedef double v3[3];

/* ---------------------------------------------------------------- small math */
static void cross3(const double* a, const double* b, double* o) {
  double x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void quat_to_mat(const double* q, double R[3][3]) {
  double x = q[0], y = q[1], z = q[2], w = q[3];
  R[0][0] = 1 - 2 * (y * y + z * z); R[0][1] = 2 * (x * y - z * w); R[0][2] = 2 * (x * z + y * w);
  R[1][0] = 2 * (x * y + z * w); R[1][1] = 1 - 2 * (x * x + z * z); R[1][2] = 2 * (y * z - x * w);
  R[2][0] = 2 * (x * z - y * w); R[2][1] = 2 * (y * z + x * w); R[2][2] = 1 - 2 * (x * x + y * y);
}
static void mat_to_quat(double R[3][3], double* q) {
  double tr = R[0][0] + R[1][1] + R[2][2];
  if (tr > 0) {
    double s = sqrt(tr + 1.0) * 2;
    q[3] = 0.25 * s; q[0] = (R[2][1] - R[1][2]) / s; q[1] = (R[0][2] - R[2][0]) / s; q[2] = (R[1][0] - R[0][1]) / s;
  } else if (R[0][0] > R[1][1] && R[0][0] > R[2][2]) {
    double s = sqrt(1.0 + R[0][0] - R[1][1] - R[2][2]) * 2;
    q[3] = (R[2][1] - R[1][2]) / s; q[0] = 0.25 * s; q[1] = (R[0][1] + R[1][0]) / s; q[2] = (R[0][2] + R[2][0]) / s;
  } else if (R[1][1] > R[2][2]) {
    double s = sqrt(1.0 + R[1][1] - R[0][0] - R[2][2]) * 2;
    q[3] = (R[0][2] - R[2][0]) / s; q[0] = (R[0][1] + R[1][0]) / s; q[1] = 0.25 * s; q[2] = (R[1][2] + R[2][1]) / s;
  } else {
    double s = sqrt(1.0 + R[2][2] - R[0][0] - R[1][1]) * 2;
    q[3] = (R[1][0] - R[0][1]) / s; q[0] = (R[0][2] + R[2][0]) / s; q[1] = (R[1][2] + R[2][1]) / s; q[2] = 0.25 * s;
  }
}
static void matmul3(double A[3][3], double B[3][3], double C[3][3]) {
  double T[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) T[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
  memcpy(C, T, sizeof(T));
}
static void matvec3(double A[3][3], const double* v, double* o) {
  double x = A[0][0] * v[0] + A[0][1] * v[1] + A[0][2] * v[2];
  double y = A[1][0] * v[0] + A[1][1] * v[1] + A[1][2] * v[2];
  double z = A[2][0] * v[0] + A[2][1] * v[1] + A[2][2] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
static void mattvec3(double A[3][3], const double* v, double* o) {
  double x = A[0][0] * v[0] + A[1][0] * v[1] + A[2][0] * v[2];
  double y = A[0][1] * v[0] + A[1][1] * v[1] + A[2][1] * v[2];
  double z = A[0][2] * v[0] + A[1][2] * v[1] + A[2][2] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
static void axis_angle_mat(const double* a, double ang, double R[3][3]) {
  double c = cos(ang), s = sin(ang), t = 1 - c, x = a[0], y = a[1], z = a[2];
  R[0][0] = t * x * x + c; R[0][1] = t * x * y - s * z; R[0][2] = t * x * z + s * y;
  R[1][0] = t * x * y + s * z; R[1][1] = t * y * y + c; R[1][2] = t * y * z - s * x;
  R[2][0] = t * x * z - s * y; R[2][1] = t * y * z + s * x; R[2][2] = t * z * z + c;
}
static void quat_mul_d(const double* a, const double* b, double* o) {
  double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  double y = a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0];
  double z = a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3];
  double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}

/* spatial algebra (6-vectors: angular first) */
static void crm(const double* v, const double* m, double* o) { /* v x m (motion) */
  double a[3], b[3], c[3];
  cross3(v, m, a);
  cross3(v, m + 3, b);
  cross3(v + 3, m, c);
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2];
  o[3] = b[0] + c[0]; o[4] = b[1] + c[1]; o[5] = b[2] + c[2];
}
static void crf(const double* v, const double* f, double* o) { /* v x* f (force) */
  double a[3], b[3], c[3];
  cross3(v, f, a);
  cross3(v + 3, f + 3, b);
  cross3(v, f + 3, c);
  o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2];
  o[3] = c[0]; o[4] = c[1]; o[5] = c[2];
}
static double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
static void mat6vec(double I[6][6], const double* v, double* o) {
  for (int i = 0; i < 6; i++) {
    double s = 0;
    for (int j = 0; j < 6; j++) s += I[i][j] * v[j];
    o[i] = s;
  }
}

/* ---------------------------------------------------------------- per-actor state */
typedef struct {
  double p[3], q[4];     /* root pose */
  double nu0[6];         /* root spatial velocity at root origin [w; v_o] */
  double qj[MAXN], qd[MAXN];
} astate;

typedef struct {
  double R[MAXN][3][3], x[MAXN][3];
  double S[MAXN][6];
  double I[MAXN][6][6];
  double V[MAXN][6];
  double o[3];
} kin;

typedef struct {
  int nodeA, nodeB, geomA, geomB;
  double p[3], n[3], d;
} contact;

static int nv_of(const mg_model* m) { return (m->fixed_base ? 0 : 6) + m->num_dofs; }
static int dof_col(const mg_model* m, int node) { return (m->fixed_base ? 0 : 6) + node - 1; }

static void load_state(const mg_model* m, const float* root, const float* dof, astate* s) {
  for (int k = 0; k < 3; k++) s->p[k] = root[k];
  double nq = 0;
  for (int k = 0; k < 4; k++) { s->q[k] = root[3 + k]; nq += s->q[k] * s->q[k]; }
  nq = sqrt(nq);
  for (int k = 0; k < 4; k++) s->q[k] /= nq;
  memset(s->nu0, 0, sizeof(s->nu0));
  if (!m->fixed_base) {
    double R[3][3], cw[3], wxc[3];
    quat_to_mat(s->q, R);
    double c[3] = {m->body_com[0][0], m->body_com[0][1], m->body_com[0][2]};
    matvec3(R, c, cw);
    double w[3] = {root[10], root[11], root[12]};
    cross3(w, cw, wxc);
    for (int k = 0; k < 3; k++) { s->nu0[k] = w[k]; s->nu0[3 + k] = root[7 + k] - wxc[k]; }
  }
  for (int i = 1; i < m->num_nodes; i++) { s->qj[i] = dof[2 * (i - 1)]; s->qd[i] = dof[2 * (i - 1) + 1]; }
}

static void store_state(const mg_model* m, const astate* s, float* root, float* dof) {
  if (!m->fixed_base) {
    double R[3][3], cw[3], wxc[3];
    quat_to_mat(s->q, R);
    double c[3] = {m->body_com[0][0], m->body_com[0][1], m->body_com[0][2]};
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
    double r0[4] = {m->r0[i][0], m->r0[i][1], m->r0[i][2], m->r0[i][3]};
    double R0[3][3], Rp0[3][3], tp[3];
    quat_to_mat(r0, R0);
    matmul3(k->R[par], R0, Rp0);
    double t[3] = {m->t[i][0], m->t[i][1], m->t[i][2]};
    matvec3(k->R[par], t, tp);
    double ax[3] = {m->axis[i][0], m->axis[i][1], m->axis[i][2]};
    if (m->jtype[i] == MG_JT_HINGE) {
      double Rj[3][3];
      axis_angle_mat(ax, s->qj[i], Rj);
      matmul3(Rp0, Rj, k->R[i]);
      for (int c = 0; c < 3; c++) k->x[i][c] = k->x[par][c] + tp[c];
    } else {
      double sw[3];
      memcpy(k->R[i], Rp0, sizeof(Rp0));
      matvec3(Rp0, ax, sw);
      for (int c = 0; c < 3; c++) k->x[i][c] = k->x[par][c] + tp[c] + sw[c] * s->qj[i];
    }
  }
  /* motion subspaces at o */
  for (int i = 1; i < m->num_nodes; i++) {
    double ax[3] = {m->axis[i][0], m->axis[i][1], m->axis[i][2]}, sw[3], r[3], rxs[3];
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
    double mass = m->mass[i];
    double cl[3] = {m->com[i][0], m->com[i][1], m->com[i][2]}, cw[3], c[3];
    matvec3(k->R[i], cl, cw);
    for (int a = 0; a < 3; a++) c[a] = k->x[i][a] + cw[a] - k->o[a];
    const float* in = m->inertia[i];
    double Il[3][3] = {{in[0], in[3], in[4]}, {in[3], in[1], in[5]}, {in[4], in[5], in[2]}};
    double T[3][3], Iw[3][3], Rt[3][3];
    matmul3(k->R[i], Il, T);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) Rt[a][b] = k->R[i][b][a];
    matmul3(T, Rt, Iw);
    double cc = dot3(c, c);
    double cx[3][3] = {{0, -c[2], c[1]}, {c[2], 0, -c[0]}, {-c[1], c[0], 0}};
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        k->I[i][a][b] = Iw[a][b] + mass * ((a == b ? cc : 0.0) - c[a] * c[b]);
        k->I[i][a][3 + b] = mass * cx[a][b];
        k->I[i][3 + a][b] = mass * cx[b][a];
        k->I[i][3 + a][3 + b] = (a == b) ? mass : 0.0;
      }
  }
  /* velocities */
  for (int c = 0; c < 6; c++) k->V[0][c] = m->fixed_base ? 0.0 : s->nu0[c];
  for (int i = 1; i < m->num_nodes; i++)
    for (int c = 0; c < 6; c++) k->V[i][c] = k->V[m->parent[i]][c] + k->S[i][c] * s->qd[i];
}

/* joint-space inertia (CRBA) incl. implicit diagonal, h = substep */
static void mass_matrix(const mg_model* m, const kin* k, double h, double* M) {
  int nv = nv_of(m), nn = m->num_nodes;
  double Ic[MAXN][6][6];
  memcpy(Ic, k->I, sizeof(double) * 36 * nn);
  for (int i = nn - 1; i >= 1; i--) {
    int p = m->parent[i];
    for (int a = 0; a < 6; a++)
      for (int b = 0; b < 6; b++) Ic[p][a][b] += Ic[i][a][b];
  }
  memset(M, 0, sizeof(double) * nv * nv);
  if (!m->fixed_base)
    for (int a = 0; a < 6; a++)
      for (int b = 0; b < 6; b++) M[a * nv + b] = Ic[0][a][b];
  for (int i = 1; i < nn; i++) {
    double F[6];
    mat6vec(Ic[i], k->S[i], F);
    int ci = dof_col(m, i);
    M[ci * nv + ci] = dot6(k->S[i], F) + m->armature[i] + h * m->damping[i] + h * h * m->stiffness[i];
    int j = m->parent[i];
    while (j > 0) {
      int cj = dof_col(m, j);
      double v = dot6(k->S[j], F);
      M[ci * nv + cj] = v;
      M[cj * nv + ci] = v;
      j = m->parent[j];
    }
    if (!m->fixed_base)
      for (int a = 0; a < 6; a++) { M[ci * nv + a] = F[a]; M[a * nv + ci] = F[a]; }
  }
}

/* bias forces C(q,v) incl. gravity (RNEA with qdd = 0) */
static void bias_forces(const mg_model* m, const kin* k, const astate* s, const double* g, double* C) {
  int nn = m->num_nodes, nv = nv_of(m);
  double A[MAXN][6], f[MAXN][6];
  for (int c = 0; c < 6; c++) A[0][c] = 0;
  for (int i = 1; i < nn; i++) {
    double sq[6], t[6];
    for (int c = 0; c < 6; c++) sq[c] = k->S[i][c] * s->qd[i];
    crm(k->V[i], sq, t);
    for (int c = 0; c < 6; c++) A[i][c] = A[m->parent[i]][c] + t[c];
  }
  for (int i = 0; i < nn; i++) {
    double IA[6], IV[6], vIV[6];
    mat6vec((double(*)[6])k->I[i], A[i], IA);
    mat6vec((double(*)[6])k->I[i], k->V[i], IV);
    crf(k->V[i], IV, vIV);
    /* gravity: force m g at COM; moment about o = c x m g */
    double mass = m->mass[i];
    double cl[3] = {m->com[i][0], m->com[i][1], m->com[i][2]}, cw[3], c[3], mg[3], n[3];
    matvec3((double(*)[3])k->R[i], cl, cw);
    for (int a = 0; a < 3; a++) { c[a] = k->x[i][a] + cw[a] - k->o[a]; mg[a] = mass * g[a]; }
    cross3(c, mg, n);
    for (int a = 0; a < 3; a++) { f[i][a] = IA[a] + vIV[a] - n[a]; f[i][3 + a] = IA[3 + a] + vIV[3 + a] - mg[a]; }
  }
  for (int i = nn - 1; i >= 1; i--)
    for (int c = 0; c < 6; c++) f[m->parent[i]][c] += f[i][c];
  memset(C, 0, sizeof(double) * nv);
  if (!m->fixed_base)
    for (int c = 0; c < 6; c++) C[c] = f[0][c];
  for (int i = 1; i < nn; i++) C[dof_col(m, i)] = dot6(k->S[i], f[i]);
}

static int cholesky(double* A, int n) {
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    if (s <= 0) return -1;
    double d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  return 0;
}
static void chol_solve(const double* L, int n, double* b) {
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * b[k];
    b[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = b[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * b[k];
    b[i] = s / L[i * n + i];
  }
}

/* ---------------------------------------------------------------- collision */
static void geom_world(const mg_model* m, const kin* k, int g, double* c, double R[3][3]) {
  int nd = m->geom_node[g];
  double pl[3] = {m->geom_pos[g][0], m->geom_pos[g][1], m->geom_pos[g][2]}, pw[3];
  matvec3((double(*)[3])k->R[nd], pl, pw);
  for (int a = 0; a < 3; a++) c[a] = k->x[nd][a] + pw[a];
  double gq[4] = {m->geom_quat[g][0], m->geom_quat[g][1], m->geom_quat[g][2], m->geom_quat[g][3]}, Rg[3][3];
  quat_to_mat(gq, Rg);
  matmul3((double(*)[3])k->R[nd], Rg, R);
}

static int push_contact(contact* out, int n, int cap, int nodeA, int gA, int nodeB, int gB, const double* p,
                        const double* nrm, double d) {
  if (n >= cap) return n;
  contact* c = &out[n];
  c->nodeA = nodeA; c->geomA = gA; c->nodeB = nodeB; c->geomB = gB;
  for (int a = 0; a < 3; a++) { c->p[a] = p[a]; c->n[a] = nrm[a]; }
  c->d = d;
  return n + 1;
}

/* sphere (center c, radius r) vs ground plane z = 0 */
static int sphere_plane(contact* out, int n, int cap, int node, int g, const double* c, double r, double off) {
  double d = c[2] - r;
  if (d < off) {
    double p[3] = {c[0], c[1], c[2] - r}, nz[3] = {0, 0, 1};
    n = push_contact(out, n, cap, node, g, -1, -1, p, nz, d);
  }
  return n;
}

static void closest_seg_seg(const double* p1, const double* q1, const double* p2, const double* q2, double* s_out,
                            double* t_out) {
  double d1[3], d2[3], r[3];
  for (int a = 0; a < 3; a++) { d1[a] = q1[a] - p1[a]; d2[a] = q2[a] - p2[a]; r[a] = p1[a] - p2[a]; }
  double a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  double s, t;
  double eps = 1e-12;
  if (a <= eps && e <= eps) { s = t = 0; }
  else if (a <= eps) { s = 0; t = f / e; t = t < 0 ? 0 : (t > 1 ? 1 : t); }
  else {
    double c = dot3(d1, r);
    if (e <= eps) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
    else {
      double b = dot3(d1, d2), den = a * e - b * b;
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
static int geom_segment(const mg_model* m, const kin* k, int g, double* a, double* b, double* r) {
  double c[3], R[3][3];
  geom_world(m, k, g, c, R);
  int ty = m->geom_type[g];
  if (ty == MG_GT_SPHERE) {
    for (int i = 0; i < 3; i++) a[i] = b[i] = c[i];
    *r = m->geom_size[g][0];
    return 1;
  }
  if (ty == MG_GT_CAPSULE) {
    double hl = m->geom_size[g][1];
    for (int i = 0; i < 3; i++) { a[i] = c[i] - R[i][2] * hl; b[i] = c[i] + R[i][2] * hl; }
    *r = m->geom_size[g][0];
    return 1;
  }
  return 0;
}

static int collide(const mg_model* m, const mg_sim_params* p, const kin* k, contact* out, int cap) {
  int n = 0;
  double off = p->contact_offset;
  for (int g = 0; g < m->num_geoms; g++) {
    int nd = m->geom_node[g], ty = m->geom_type[g];
    double c[3], R[3][3];
    geom_world(m, k, g, c, R);
    if (ty == MG_GT_SPHERE) {
      n = sphere_plane(out, n, cap, nd, g, c, m->geom_size[g][0], off);
    } else if (ty == MG_GT_CAPSULE) {
      double hl = m->geom_size[g][1], r = m->geom_size[g][0], e[3];
      for (int s = -1; s <= 1; s += 2) {
        for (int a = 0; a < 3; a++) e[a] = c[a] + s * R[a][2] * hl;
        n = sphere_plane(out, n, cap, nd, g, e, r, off);
      }
    } else if (ty == MG_GT_BOX) {
      for (int corner = 0; corner < 8; corner++) {
        double l[3] = {(corner & 1 ? 1 : -1) * m->geom_size[g][0], (corner & 2 ? 1 : -1) * m->geom_size[g][1],
                       (corner & 4 ? 1 : -1) * m->geom_size[g][2]};
        double w[3], e[3];
        matvec3(R, l, w);
        for (int a = 0; a < 3; a++) e[a] = c[a] + w[a];
        n = sphere_plane(out, n, cap, nd, g, e, 0.0, off);
      }
    }
  }
  for (int pi = 0; pi < m->num_pairs; pi++) {
    int ga = m->pair[pi][0], gb = m->pair[pi][1];
    double a0[3], a1[3], b0[3], b1[3], ra, rb;
    if (!geom_segment(m, k, ga, a0, a1, &ra) || !geom_segment(m, k, gb, b0, b1, &rb)) continue;
    double s, t, pa[3], pb[3], dv[3];
    closest_seg_seg(a0, a1, b0, b1, &s, &t);
    for (int a = 0; a < 3; a++) {
      pa[a] = a0[a] + s * (a1[a] - a0[a]);
      pb[a] = b0[a] + t * (b1[a] - b0[a]);
      dv[a] = pa[a] - pb[a];
    }
    double dist = sqrt(dot3(dv, dv));
    double d = dist - ra - rb;
    if (d < off && dist > 1e-9) {
      double nrm[3] = {dv[0] / dist, dv[1] / dist, dv[2] / dist}, pt[3];
      for (int a = 0; a < 3; a++) pt[a] = 0.5 * (pa[a] - ra * nrm[a] + pb[a] + rb * nrm[a]);
      n = push_contact(out, n, cap, m->geom_node[ga], ga, m->geom_node[gb], gb, pt, nrm, d);
    }
  }
  return n;
}

static void tangent_basis(const double* n, double* t1, double* t2) {
  double a[3] = {0, 0, 0};
  if (fabs(n[0]) < 0.57735) a[0] = 1; else a[1] = 1;
  cross3(a, n, t1);
  double l = sqrt(dot3(t1, t1));
  for (int i = 0; i < 3; i++) t1[i] /= l;
  cross3(n, t1, t2);
}

/* generalized Jacobian row of a unit force `dir` at point p on nodeA (minus on nodeB) */
static void jac_row(const mg_model* m, const kin* k, int nodeA, int nodeB, const double* p, const double* dir,
                    double* J) {
  int nv = nv_of(m);
  memset(J, 0, sizeof(double) * nv);
  double r[3], w[6];
  for (int a = 0; a < 3; a++) r[a] = p[a] - k->o[a];
  cross3(r, dir, w);
  w[3] = dir[0]; w[4] = dir[1]; w[5] = dir[2];
  for (int side = 0; side < 2; side++) {
    int node = side == 0 ? nodeA : nodeB;
    double sg = side == 0 ? 1.0 : -1.0;
    if (node < 0) continue;
    if (!m->fixed_base)
      for (int c = 0; c < 6; c++) J[c] += sg * w[c];
    for (int j = node; j > 0; j = m->parent[j]) J[dof_col(m, j)] += sg * dot6(k->S[j], w);
  }
}

/* ---------------------------------------------------------------- one substep */
typedef struct {
  double h;
  contact con[MAXC];
  int ncon;
  double lam[MAXR];
  int nrows;
  int row_kind[MAXR]; /* 0 normal, 1 friction, 2 limit-lower, 3 limit-upper */
  int row_ref[MAXR];  /* contact index or node */
} substep_out;

static void substep(const mg_model* m, const mg_sim_params* p, astate* s, const double* tau_act, substep_out* so) {
  int nv = nv_of(m), nn = m->num_nodes;
  double h = p->dt / p->substeps;
  so->h = h;
  kin k;
  forward_kinematics(m, s, &k);
  double M[MAXV * MAXV], C[MAXV], g[3] = {p->gravity[0], p->gravity[1], p->gravity[2]};
  mass_matrix(m, &k, h, M);
  bias_forces(m, &k, s, g, C);
  if (cholesky(M, nv) != 0) return;
  double nu[MAXV], rhs[MAXV];
  for (int c = 0; c < 6 && !m->fixed_base; c++) nu[c] = s->nu0[c];
  for (int i = 1; i < nn; i++) nu[dof_col(m, i)] = s->qd[i];
  for (int c = 0; c < nv; c++) rhs[c] = -C[c];
  for (int i = 1; i < nn; i++) {
    int ci = dof_col(m, i);
    double t = tau_act ? tau_act[i - 1] : 0.0;
    rhs[ci] += t - m->damping[i] * s->qd[i] - m->stiffness[i] * (s->qj[i] + h * s->qd[i]);
  }
  chol_solve(M, nv, rhs);
  for (int c = 0; c < nv; c++) nu[c] += h * rhs[c];

  /* constraint rows */
  int cap = p->max_contacts < MAXC ? p->max_contacts : MAXC;
  so->ncon = collide(m, p, &k, so->con, cap);
  static __thread double J[MAXR][MAXV], Y[MAXR][MAXV];
  double b[MAXR], W[MAXR];
  int nr = 0;
  for (int c = 0; c < so->ncon; c++) {
    contact* ct = &so->con[c];
    double t1[3], t2[3];
    tangent_basis(ct->n, t1, t2);
    double deff = ct->d - p->rest_offset;
    double bn = deff >= 0 ? -deff / h : fmin(-p->baumgarte * deff / h, p->max_depen_vel);
    const double* dirs[3] = {ct->n, t1, t2};
    for (int r = 0; r < 3; r++) {
      jac_row(m, &k, ct->nodeA, ct->nodeB, ct->p, dirs[r], J[nr]);
      b[nr] = r == 0 ? bn : 0.0;
      so->row_kind[nr] = r == 0 ? 0 : 1;
      so->row_ref[nr] = c;
      nr++;
    }
  }
  for (int i = 1; i < nn; i++) {
    if (!m->limited[i]) continue;
    double dl = s->qj[i] - m->lower[i], du = m->upper[i] - s->qj[i];
    for (int side = 0; side < 2; side++) {
      double d = side == 0 ? dl : du;
      if (d >= p->limit_margin) continue;
      memset(J[nr], 0, sizeof(double) * nv);
      J[nr][dof_col(m, i)] = side == 0 ? 1.0 : -1.0;
      b[nr] = d >= 0 ? -d / h : fmin(-p->baumgarte * d / h, p->max_depen_vel);
      so->row_kind[nr] = 2 + side;
      so->row_ref[nr] = i;
      nr++;
    }
  }
  so->nrows = nr;
  for (int r = 0; r < nr; r++) {
    for (int c = 0; c < nv; c++) Y[r][c] = J[r][c];
    chol_solve(M, nv, Y[r]);
    double w = 0;
    for (int c = 0; c < nv; c++) w += J[r][c] * Y[r][c];
    W[r] = w;
    so->lam[r] = 0;
  }
  for (int it = 0; it < p->pos_iters; it++) {
    for (int r = 0; r < nr; r++) {
      if (W[r] <= 1e-12) continue;
      double v = 0;
      for (int c = 0; c < nv; c++) v += J[r][c] * nu[c];
      double lnew = so->lam[r] + (b[r] - v) / W[r];
      if (so->row_kind[r] == 1) {
        double lim = p->friction * so->lam[3 * so->row_ref[r]];  /* normal row of this contact */
        lnew = lnew < -lim ? -lim : (lnew > lim ? lim : lnew);
      } else if (lnew < 0) {
        lnew = 0;
      }
      double dl = lnew - so->lam[r];
      so->lam[r] = lnew;
      for (int c = 0; c < nv; c++) nu[c] += Y[r][c] * dl;
    }
  }
  /* integrate */
  if (!m->fixed_base) {
    double w[3] = {nu[0], nu[1], nu[2]}, vo[3] = {nu[3], nu[4], nu[5]};
    double pn[3];
    for (int a = 0; a < 3; a++) pn[a] = s->p[a] + h * vo[a];
    double wn = sqrt(dot3(w, w)), dq[4];
    if (wn * h > 1e-12) {
      double ha = 0.5 * wn * h, sn = sin(ha) / wn;
      dq[0] = w[0] * sn; dq[1] = w[1] * sn; dq[2] = w[2] * sn; dq[3] = cos(ha);
    } else {
      dq[0] = 0.5 * h * w[0]; dq[1] = 0.5 * h * w[1]; dq[2] = 0.5 * h * w[2]; dq[3] = 1.0;
    }
    double qn[4];
    quat_mul_d(dq, s->q, qn);
    double l = sqrt(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
    for (int a = 0; a < 4; a++) s->q[a] = qn[a] / l;
    double dp[3] = {pn[0] - s->p[0], pn[1] - s->p[1], pn[2] - s->p[2]}, wxdp[3];
    cross3(w, dp, wxdp);
    for (int a = 0; a < 3; a++) { s->p[a] = pn[a]; s->nu0[a] = w[a]; s->nu0[3 + a] = vo[a] + wxdp[a]; }
  }
  for (int i = 1; i < nn; i++) {
    s->qd[i] = nu[dof_col(m, i)];
    s->qj[i] += h * s->qd[i];
  }
}

/* sensor wrench and dof force from the last substep's impulses */
static void sensor_outputs(const mg_model* m, const astate* s, const substep_out* so, const double* tau_act,
                           float* sensors, float* dof_force) {
  if (sensors && m->num_sensors > 0) {
    kin k;
    forward_kinematics(m, s, &k);  /* post-step pose for the body frame */
    for (int si = 0; si < m->num_sensors; si++) {
      int body = m->sensor_body[si], nd = m->body_node[body];
      double Rb[3][3], bq[4] = {m->body_quat[body][0], m->body_quat[body][1], m->body_quat[body][2],
                                 m->body_quat[body][3]}, Rl[3][3];
      quat_to_mat(bq, Rl);
      matmul3(k.R[nd], Rl, Rb);
      double bp[3] = {m->body_pos[body][0], m->body_pos[body][1], m->body_pos[body][2]}, bw[3], xb[3];
      matvec3(k.R[nd], bp, bw);
      for (int a = 0; a < 3; a++) xb[a] = k.x[nd][a] + bw[a];
      double F[3] = {0, 0, 0}, T[3] = {0, 0, 0};
      for (int c = 0; c < so->ncon; c++) {
        const contact* ct = &so->con[c];
        double sg = 0;
        if (m->geom_body[ct->geomA] == body) sg = 1;
        else if (ct->geomB >= 0 && m->geom_body[ct->geomB] == body) sg = -1;
        if (sg == 0) continue;
        double t1[3], t2[3];
        tangent_basis(ct->n, t1, t2);
        double f[3], r[3], rf[3];
        for (int a = 0; a < 3; a++)
          f[a] = sg * (so->lam[3 * c] * ct->n[a] + so->lam[3 * c + 1] * t1[a] + so->lam[3 * c + 2] * t2[a]) / so->h;
        for (int a = 0; a < 3; a++) r[a] = ct->p[a] - xb[a];
        cross3(r, f, rf);
        for (int a = 0; a < 3; a++) { F[a] += f[a]; T[a] += rf[a]; }
      }
      double Fl[3], Tl[3];
      mattvec3(Rb, F, Fl);
      mattvec3(Rb, T, Tl);
      for (int a = 0; a < 3; a++) { sensors[6 * si + a] = (float)Fl[a]; sensors[6 * si + 3 + a] = (float)Tl[a]; }
    }
  }
  if (dof_force) {
    for (int i = 1; i < m->num_nodes; i++) {
      double t = (tau_act ? tau_act[i - 1] : 0.0) - m->damping[i] * s->qd[i] - m->stiffness[i] * s->qj[i];
      for (int r = 0; r < so->nrows; r++) {
        if (so->row_ref[r] != i) continue;
        if (so->row_kind[r] == 2) t += so->lam[r] / so->h;
        if (so->row_kind[r] == 3) t -= so->lam[r] / so->h;
      }
      dof_force[i - 1] = (float)t;
    }
  }
}

static void simulate_actor(const mg_model* m, const mg_sim_params* p, float* root, float* dof, const float* act,
                           float* sensors, float* dof_force) {
  astate s;
  load_state(m, root, dof, &s);
  double tau[MAXN];
  for (int i = 0; i < m->num_dofs; i++) tau[i] = act ? act[i] : 0.0;
  substep_out* so = (substep_out*)malloc(sizeof(substep_out));
  memset(so, 0, sizeof(*so));
  for (int st = 0; st < p->substeps; st++) substep(m, p, &s, tau, so);
  store_state(m, &s, root, dof);
  sensor_outputs(m, &s, so, tau, sensors, dof_force);
  free(so);
}

int orc_simulate(const mg_model* m, const mg_sim_params* p, int32_t n, float* root_states, float* dof_state,
                 const float* dof_actuation, float* sensors, float* dof_force, int32_t threads) {
  int nd = m->num_dofs, ns = m->num_sensors;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (int e = 0; e < n; e++) {
    simulate_actor(m, p, root_states + 13 * e, dof_state + 2 * nd * e, dof_actuation ? dof_actuation + nd * e : 0,
                   sensors ? sensors + 6 * ns * e : 0, dof_force ? dof_force + nd * e : 0);
  }
  (void)threads;
  return 0;
}

int orc_mass_matrix(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2,
                    double* M_out) {
  astate s;
  kin k;
  load_state(m, root13, dof2, &s);
  forward_kinematics(m, &s, &k);
  mass_matrix(m, &k, p->dt / p->substeps, M_out);
  return nv_of(m);
}

int orc_free_acceleration(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2,
                          const float* tau, double* qacc_out) {
  astate s;
  kin k;
  load_state(m, root13, dof2, &s);
  forward_kinematics(m, &s, &k);
  int nv = nv_of(m);
  double h = p->dt / p->substeps, M[MAXV * MAXV], C[MAXV], g[3] = {p->gravity[0], p->gravity[1], p->gravity[2]};
  mass_matrix(m, &k, h, M);
  bias_forces(m, &k, &s, g, C);
  if (cholesky(M, nv) != 0) return -1;
  for (int c = 0; c < nv; c++) qacc_out[c] = -C[c];
  for (int i = 1; i < m->num_nodes; i++)
    qacc_out[dof_col(m, i)] += (tau ? tau[i - 1] : 0.0) - m->damping[i] * s.qd[i] -
                               m->stiffness[i] * (s.qj[i] + h * s.qd[i]);
  chol_solve(M, nv, qacc_out);
  return nv;
}

int orc_contacts(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2, double* out,
                 int32_t cap) {
  astate s;
  kin k;
  load_state(m, root13, dof2, &s);
  forward_kinematics(m, &s, &k);
  contact con[MAXC];
  int c = cap < MAXC ? cap : MAXC;
  int nc = collide(m, p, &k, con, c);
  for (int i = 0; i < nc; i++) {
    double* o = out + 9 * i;
    o[0] = con[i].nodeA;
    o[1] = con[i].p[0]; o[2] = con[i].p[1]; o[3] = con[i].p[2];
    o[4] = con[i].n[0]; o[5] = con[i].n[1]; o[6] = con[i].n[2];
    o[7] = con[i].d;
    o[8] = con[i].nodeB;
  }
  return nc;
}

int orc_rigid_body_states(const mg_model* m, const float* root13, const float* dof2, float* out) {
  astate s;
  kin k;
  load_state(m, root13, dof2, &s);
  forward_kinematics(m, &s, &k);
  for (int b = 0; b < m->num_bodies; b++) {
    int nd = m->body_node[b];
    double bq[4] = {m->body_quat[b][0], m->body_quat[b][1], m->body_quat[b][2], m->body_quat[b][3]}, Rl[3][3],
           Rb[3][3];
    quat_to_mat(bq, Rl);
    matmul3(k.R[nd], Rl, Rb);
    double bp[3] = {m->body_pos[b][0], m->body_pos[b][1], m->body_pos[b][2]}, bw[3], xb[3], q[4];
    matvec3(k.R[nd], bp, bw);
    for (int a = 0; a < 3; a++) xb[a] = k.x[nd][a] + bw[a];
    mat_to_quat(Rb, q);
    double cl[3] = {m->body_com[b][0], m->body_com[b][1], m->body_com[b][2]}, cw[3], r[3], wxr[3];
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
  return m->num_bodies;
}

// physics.hpp — per-actor articulated-body step on gfx950 (gym.simulate
// counterpart).  One lane owns one actor.
//
// Per substep h = dt / substeps (Ant.yaml:43-44):
//   1. forward kinematics of the node tree (world-aligned frames; spatial
//      quantities expressed at the root origin o)
//   2. Featherstone articulated-body algorithm (ABA): backward pass builds the
//      articulated inertias I^A, U = I^A S, D = S.U + armature + h b + h^2 k,
//      forward pass gives the unconstrained accelerations; nu* = nu + h a
//   3. contact generation (sphere/capsule/box vs ground plane; sphere/capsule
//      self pairs) under a speculative contact offset
//   4. constraint rows [normal, t1, t2] per contact, then joint limits; the
//      response columns Y = M~^-1 J^T come from ABA "test force" solves that
//      reuse the factorisation of step 2 (no mass matrix is ever formed)
//   5. projected Gauss-Seidel, pos_iters sweeps, box friction |l_t| <= mu l_n
//   6. semi-implicit Euler; root orientation by the exact exponential map
// The fp64 CPU oracle (oracle/oracle_physics.c) restates the same algorithm
// with a dense mass matrix (CRBA + Cholesky) instead of the ABA; parity tests
// compare the two (tests/test_gpu_parity.py).
#pragma once
#include "../../include/migym.h"
#include "device_math.hpp"

namespace mg {

template <int MN, int MC>
struct ActorWork {
  static constexpr int MV = MN - 1 + 6;
  static constexpr int MR = 3 * MC + 2 * (MN - 1);
  // state
  V3 p;
  float q[4];
  SV nu0;
  float qj[MN], qd[MN];
  // kinematics (valid after fk())
  M3 R[MN];
  V3 x[MN];
  SV S[MN];
  SV V[MN];
  V3 o;
  // ABA factorisation (valid after aba())
  SV U[MN];
  float Dinv[MN];
  float L0[21];
  // contacts + rows of the last substep
  int ncon, nrows;
  int cA[MC], cB[MC], cgA[MC], cgB[MC];
  V3 cp[MC], cn[MC];
  float cd[MC];
  float J[MR][MV];
  float Y[MR][MV];
  float lam[MR], bb[MR], W[MR];
  int rkind[MR], rref[MR];
  float h;
};

__device__ __forceinline__ int nv_of(const mg_model* m) { return (m->fixed_base ? 0 : 6) + m->num_dofs; }
__device__ __forceinline__ int dof_col(const mg_model* m, int node) { return (m->fixed_base ? 0 : 6) + node - 1; }

template <int MN, int MC>
__device__ void load_state(const mg_model* m, const float* root, const float* dof, ActorWork<MN, MC>& w) {
  w.p = ld3(root);
  float n = sqrtf(root[3] * root[3] + root[4] * root[4] + root[5] * root[5] + root[6] * root[6]);
  for (int k = 0; k < 4; k++) w.q[k] = root[3 + k] / n;
  w.nu0 = szero();
  if (!m->fixed_base) {
    M3 R = quat_to_mat(w.q[0], w.q[1], w.q[2], w.q[3]);
    V3 cw = mul(R, ld3(m->body_com[0]));
    V3 om = ld3(root + 10);
    w.nu0 = sv(om, ld3(root + 7) - cross(om, cw));
  }
  for (int i = 1; i < m->num_nodes; i++) {
    w.qj[i] = dof[2 * (i - 1)];
    w.qd[i] = dof[2 * (i - 1) + 1];
  }
}

template <int MN, int MC>
__device__ void store_state(const mg_model* m, const ActorWork<MN, MC>& w, float* root, float* dof) {
  if (!m->fixed_base) {
    M3 R = quat_to_mat(w.q[0], w.q[1], w.q[2], w.q[3]);
    V3 cw = mul(R, ld3(m->body_com[0]));
    V3 vc = w.nu0.l + cross(w.nu0.a, cw);
    root[0] = w.p.x; root[1] = w.p.y; root[2] = w.p.z;
    for (int k = 0; k < 4; k++) root[3 + k] = w.q[k];
    root[7] = vc.x; root[8] = vc.y; root[9] = vc.z;
    root[10] = w.nu0.a.x; root[11] = w.nu0.a.y; root[12] = w.nu0.a.z;
  }
  for (int i = 1; i < m->num_nodes; i++) {
    dof[2 * (i - 1)] = w.qj[i];
    dof[2 * (i - 1) + 1] = w.qd[i];
  }
}

template <int MN, int MC>
__device__ void fk(const mg_model* m, ActorWork<MN, MC>& w) {
  const int nn = m->num_nodes;
  w.R[0] = quat_to_mat(w.q[0], w.q[1], w.q[2], w.q[3]);
  w.x[0] = w.p;
  w.o = w.p;
  for (int i = 1; i < nn; i++) {
    const int par = m->parent[i];
    M3 Rp0 = mul(w.R[par], quat_to_mat(m->r0[i][0], m->r0[i][1], m->r0[i][2], m->r0[i][3]));
    V3 tp = mul(w.R[par], ld3(m->t[i]));
    V3 ax = ld3(m->axis[i]);
    if (m->jtype[i] == MG_JT_HINGE) {
      w.R[i] = mul(Rp0, axis_angle(ax, w.qj[i]));
      w.x[i] = w.x[par] + tp;
      V3 s = mul(w.R[i], ax);
      w.S[i] = sv(s, cross(w.x[i] - w.o, s));
    } else {
      w.R[i] = Rp0;
      V3 s = mul(Rp0, ax);
      w.x[i] = w.x[par] + tp + s * w.qj[i];
      w.S[i] = sv(v3(0, 0, 0), s);
    }
  }
  w.V[0] = m->fixed_base ? szero() : w.nu0;
  for (int i = 1; i < nn; i++) w.V[i] = w.V[m->parent[i]] + w.S[i] * w.qd[i];
}

template <int MN, int MC>
__device__ __forceinline__ Sym6 node_inertia(const mg_model* m, const ActorWork<MN, MC>& w, int i, V3* c_out) {
  const M3& R = w.R[i];
  V3 c = w.x[i] + mul(R, ld3(m->com[i])) - w.o;
  const float* in = m->inertia[i];
  // Iw = R Il R^T (Il sym: xx yy zz xy xz yz)
  float Il[3][3] = {{in[0], in[3], in[4]}, {in[3], in[1], in[5]}, {in[4], in[5], in[2]}};
  float T[3][3], Iw[6];
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) T[a][b] = R.m[a][0] * Il[0][b] + R.m[a][1] * Il[1][b] + R.m[a][2] * Il[2][b];
  const int idx[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
  for (int k = 0; k < 6; k++) {
    int a = idx[k][0], b = idx[k][1];
    Iw[k] = T[a][0] * R.m[b][0] + T[a][1] * R.m[b][1] + T[a][2] * R.m[b][2];
  }
  *c_out = c;
  return body_inertia(m->mass[i], c, Iw);
}

// ABA: factorises (stores U, Dinv, L0) and returns unconstrained accelerations in acc[MV]
template <int MN, int MC>
__device__ void aba(const mg_model* m, const mg_sim_params* p, ActorWork<MN, MC>& w, const float* tau_act,
                    float* acc) {
  const int nn = m->num_nodes;
  const float h = w.h;
  const V3 g = ld3(p->gravity);
  Sym6 IA[MN];
  SV pA[MN], cb[MN];
  float u[MN];
  for (int i = 0; i < nn; i++) {
    V3 c;
    IA[i] = node_inertia(m, w, i, &c);
    SV IV = mul(IA[i], w.V[i]);
    V3 mg = g * m->mass[i];
    pA[i] = crf(w.V[i], IV) - sv(cross(c, mg), mg);
    cb[i] = i == 0 ? szero() : crm(w.V[i], w.S[i] * w.qd[i]);
  }
  for (int i = nn - 1; i >= 1; i--) {
    SV Ui = mul(IA[i], w.S[i]);
    float D = dot(w.S[i], Ui) + m->armature[i] + h * m->damping[i] + h * h * m->stiffness[i];
    float Di = 1.0f / D;
    float t = (tau_act ? tau_act[i - 1] : 0.0f) - m->damping[i] * w.qd[i] - m->stiffness[i] * (w.qj[i] + h * w.qd[i]);
    u[i] = t - dot(w.S[i], pA[i]);
    w.U[i] = Ui;
    w.Dinv[i] = Di;
    Sym6 Ia = IA[i];
    rank1_sub(Ia, Ui, Di);
    SV pa = pA[i] + mul(Ia, cb[i]) + Ui * (u[i] * Di);
    const int par = m->parent[i];
    add_to(IA[par], Ia);
    pA[par] = pA[par] + pa;
  }
  SV a[MN];
  if (!m->fixed_base) {
    chol6(IA[0], w.L0);
    a[0] = chol6_solve(w.L0, pA[0] * -1.0f);
    acc[0] = a[0].a.x; acc[1] = a[0].a.y; acc[2] = a[0].a.z;
    acc[3] = a[0].l.x; acc[4] = a[0].l.y; acc[5] = a[0].l.z;
  } else {
    a[0] = szero();
  }
  for (int i = 1; i < nn; i++) {
    SV ap = a[m->parent[i]] + cb[i];
    float qdd = (u[i] - dot(w.U[i], ap)) * w.Dinv[i];
    a[i] = ap + w.S[i] * qdd;
    acc[dof_col(m, i)] = qdd;
  }
}

// y = M~^-1 (J^T) for a generalized force given as: spatial force fw on nodeA (and -fw on nodeB),
// plus a unit joint force on node `jn` with sign js (jn = 0: none).  Reuses the ABA factorisation.
template <int MN, int MC>
__device__ void test_solve(const mg_model* m, ActorWork<MN, MC>& w, int nodeA, int nodeB, SV fw, int jn, float js,
                          float* y) {
  const int nn = m->num_nodes;
  SV pA[MN];
  float u[MN];
  for (int i = 0; i < nn; i++) pA[i] = szero();
  if (nodeA >= 0) pA[nodeA] = pA[nodeA] - fw;
  if (nodeB >= 0) pA[nodeB] = pA[nodeB] + fw;
  for (int i = nn - 1; i >= 1; i--) {
    float t = (i == jn) ? js : 0.0f;
    u[i] = t - dot(w.S[i], pA[i]);
    const int par = m->parent[i];
    pA[par] = pA[par] + pA[i] + w.U[i] * (u[i] * w.Dinv[i]);
  }
  SV a[MN];
  if (!m->fixed_base) {
    a[0] = chol6_solve(w.L0, pA[0] * -1.0f);
    y[0] = a[0].a.x; y[1] = a[0].a.y; y[2] = a[0].a.z;
    y[3] = a[0].l.x; y[4] = a[0].l.y; y[5] = a[0].l.z;
  } else {
    a[0] = szero();
  }
  for (int i = 1; i < nn; i++) {
    SV ap = a[m->parent[i]];
    float qdd = (u[i] - dot(w.U[i], ap)) * w.Dinv[i];
    a[i] = ap + w.S[i] * qdd;
    y[dof_col(m, i)] = qdd;
  }
}

// ---------------------------------------------------------------- collision
template <int MN, int MC>
__device__ __forceinline__ void geom_world(const mg_model* m, const ActorWork<MN, MC>& w, int g, V3* c, M3* R) {
  const int nd = m->geom_node[g];
  *c = w.x[nd] + mul(w.R[nd], ld3(m->geom_pos[g]));
  *R = mul(w.R[nd], quat_to_mat(m->geom_quat[g][0], m->geom_quat[g][1], m->geom_quat[g][2], m->geom_quat[g][3]));
}

template <int MN, int MC>
__device__ __forceinline__ void push_contact(ActorWork<MN, MC>& w, int cap, int nA, int gA, int nB, int gB, V3 pt,
                                             V3 nrm, float d) {
  if (w.ncon >= cap) return;
  int k = w.ncon++;
  w.cA[k] = nA; w.cgA[k] = gA; w.cB[k] = nB; w.cgB[k] = gB;
  w.cp[k] = pt; w.cn[k] = nrm; w.cd[k] = d;
}

template <int MN, int MC>
__device__ __forceinline__ void sphere_plane(ActorWork<MN, MC>& w, int cap, int nd, int g, V3 c, float r, float off) {
  float d = c.z - r;
  if (d < off) push_contact(w, cap, nd, g, -1, -1, v3(c.x, c.y, c.z - r), v3(0, 0, 1), d);
}

__device__ __forceinline__ void closest_seg_seg(V3 p1, V3 q1, V3 p2, V3 q2, float* s_out, float* t_out) {
  V3 d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
  float a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r);
  float s, t;
  const float eps = 1e-12f;
  if (a <= eps && e <= eps) {
    s = t = 0;
  } else if (a <= eps) {
    s = 0;
    t = fminf(fmaxf(f / e, 0.0f), 1.0f);
  } else {
    float c = dot(d1, r);
    if (e <= eps) {
      t = 0;
      s = fminf(fmaxf(-c / a, 0.0f), 1.0f);
    } else {
      float b = dot(d1, d2), den = a * e - b * b;
      s = den > eps ? (b * f - c * e) / den : 0.0f;
      s = fminf(fmaxf(s, 0.0f), 1.0f);
      t = (b * s + f) / e;
      if (t < 0) {
        t = 0;
        s = fminf(fmaxf(-c / a, 0.0f), 1.0f);
      } else if (t > 1) {
        t = 1;
        s = fminf(fmaxf((b - c) / a, 0.0f), 1.0f);
      }
    }
  }
  *s_out = s;
  *t_out = t;
}

template <int MN, int MC>
__device__ __forceinline__ bool geom_segment(const mg_model* m, const ActorWork<MN, MC>& w, int g, V3* a, V3* b,
                                             float* r) {
  V3 c;
  M3 R;
  geom_world(m, w, g, &c, &R);
  int ty = m->geom_type[g];
  if (ty == MG_GT_SPHERE) {
    *a = c; *b = c; *r = m->geom_size[g][0];
    return true;
  }
  if (ty == MG_GT_CAPSULE) {
    V3 ax = v3(R.m[0][2], R.m[1][2], R.m[2][2]) * m->geom_size[g][1];
    *a = c - ax; *b = c + ax; *r = m->geom_size[g][0];
    return true;
  }
  return false;
}

template <int MN, int MC>
__device__ void collide(const mg_model* m, const mg_sim_params* p, ActorWork<MN, MC>& w) {
  w.ncon = 0;
  const int cap = p->max_contacts < MC ? p->max_contacts : MC;
  const float off = p->contact_offset;
  for (int g = 0; g < m->num_geoms; g++) {
    const int nd = m->geom_node[g], ty = m->geom_type[g];
    V3 c;
    M3 R;
    geom_world(m, w, g, &c, &R);
    if (ty == MG_GT_SPHERE) {
      sphere_plane(w, cap, nd, g, c, m->geom_size[g][0], off);
    } else if (ty == MG_GT_CAPSULE) {
      V3 ax = v3(R.m[0][2], R.m[1][2], R.m[2][2]) * m->geom_size[g][1];
      sphere_plane(w, cap, nd, g, c - ax, m->geom_size[g][0], off);
      sphere_plane(w, cap, nd, g, c + ax, m->geom_size[g][0], off);
    } else if (ty == MG_GT_BOX) {
      for (int corner = 0; corner < 8; corner++) {
        V3 l = v3((corner & 1 ? 1.f : -1.f) * m->geom_size[g][0], (corner & 2 ? 1.f : -1.f) * m->geom_size[g][1],
                  (corner & 4 ? 1.f : -1.f) * m->geom_size[g][2]);
        sphere_plane(w, cap, nd, g, c + mul(R, l), 0.0f, off);
      }
    }
  }
  for (int pi = 0; pi < m->num_pairs; pi++) {
    const int ga = m->pair[pi][0], gb = m->pair[pi][1];
    V3 a0, a1, b0, b1;
    float ra, rb;
    if (!geom_segment(m, w, ga, &a0, &a1, &ra) || !geom_segment(m, w, gb, &b0, &b1, &rb)) continue;
    // broadphase: bounding spheres of the two segments
    V3 ca = (a0 + a1) * 0.5f, cb = (b0 + b1) * 0.5f;
    V3 dc = ca - cb;
    float ha = sqrtf(dot(a1 - a0, a1 - a0)) * 0.5f, hb = sqrtf(dot(b1 - b0, b1 - b0)) * 0.5f;
    float reach = ha + hb + ra + rb + off;
    if (dot(dc, dc) > reach * reach) continue;
    float s, t;
    closest_seg_seg(a0, a1, b0, b1, &s, &t);
    V3 pa = a0 + (a1 - a0) * s, pb = b0 + (b1 - b0) * t, dv = pa - pb;
    float dist = sqrtf(dot(dv, dv));
    float d = dist - ra - rb;
    if (d < off && dist > 1e-9f) {
      V3 nrm = dv * (1.0f / dist);
      V3 pt = ((pa - nrm * ra) + (pb + nrm * rb)) * 0.5f;
      push_contact(w, cap, m->geom_node[ga], ga, m->geom_node[gb], gb, pt, nrm, d);
    }
  }
}

__device__ __forceinline__ void tangent_basis(V3 n, V3* t1, V3* t2) {
  V3 a = fabsf(n.x) < 0.57735f ? v3(1, 0, 0) : v3(0, 1, 0);
  V3 t = cross(a, n);
  t = t * (1.0f / sqrtf(dot(t, t)));
  *t1 = t;
  *t2 = cross(n, t);
}

template <int MN, int MC>
__device__ void jac_row(const mg_model* m, const ActorWork<MN, MC>& w, int nA, int nB, V3 pt, V3 dir, float* J) {
  const int nv = nv_of(m);
  for (int c = 0; c < nv; c++) J[c] = 0.0f;
  SV fw = sv(cross(pt - w.o, dir), dir);
  for (int side = 0; side < 2; side++) {
    int node = side == 0 ? nA : nB;
    float sg = side == 0 ? 1.0f : -1.0f;
    if (node < 0) continue;
    if (!m->fixed_base) {
      J[0] += sg * fw.a.x; J[1] += sg * fw.a.y; J[2] += sg * fw.a.z;
      J[3] += sg * fw.l.x; J[4] += sg * fw.l.y; J[5] += sg * fw.l.z;
    }
    for (int j = node; j > 0; j = m->parent[j]) J[dof_col(m, j)] += sg * dot(w.S[j], fw);
  }
}

// ---------------------------------------------------------------- substep
template <int MN, int MC>
__device__ void substep(const mg_model* m, const mg_sim_params* p, ActorWork<MN, MC>& w, const float* tau) {
  const int nv = nv_of(m), nn = m->num_nodes;
  const float h = w.h;
  fk(m, w);
  float nu[ActorWork<MN, MC>::MV], acc[ActorWork<MN, MC>::MV];
  aba(m, p, w, tau, acc);
  if (!m->fixed_base) {
    nu[0] = w.nu0.a.x; nu[1] = w.nu0.a.y; nu[2] = w.nu0.a.z;
    nu[3] = w.nu0.l.x; nu[4] = w.nu0.l.y; nu[5] = w.nu0.l.z;
  }
  for (int i = 1; i < nn; i++) nu[dof_col(m, i)] = w.qd[i];
  for (int c = 0; c < nv; c++) nu[c] += h * acc[c];

  collide(m, p, w);
  int nr = 0;
  for (int c = 0; c < w.ncon; c++) {
    V3 t1, t2;
    tangent_basis(w.cn[c], &t1, &t2);
    float deff = w.cd[c] - p->rest_offset;
    float bn = deff >= 0.0f ? -deff / h : fminf(-p->baumgarte * deff / h, p->max_depen_vel);
    V3 dirs[3] = {w.cn[c], t1, t2};
    for (int r = 0; r < 3; r++) {
      jac_row(m, w, w.cA[c], w.cB[c], w.cp[c], dirs[r], w.J[nr]);
      SV fw = sv(cross(w.cp[c] - w.o, dirs[r]), dirs[r]);
      test_solve(m, w, w.cA[c], w.cB[c], fw, 0, 0.0f, w.Y[nr]);
      w.bb[nr] = r == 0 ? bn : 0.0f;
      w.rkind[nr] = r == 0 ? 0 : 1;
      w.rref[nr] = c;
      nr++;
    }
  }
  for (int i = 1; i < nn; i++) {
    if (!m->limited[i]) continue;
    float dl = w.qj[i] - m->lower[i], du = m->upper[i] - w.qj[i];
    for (int side = 0; side < 2; side++) {
      float d = side == 0 ? dl : du;
      if (d >= p->limit_margin) continue;
      float sg = side == 0 ? 1.0f : -1.0f;
      for (int c = 0; c < nv; c++) w.J[nr][c] = 0.0f;
      w.J[nr][dof_col(m, i)] = sg;
      test_solve(m, w, -1, -1, szero(), i, sg, w.Y[nr]);
      w.bb[nr] = d >= 0.0f ? -d / h : fminf(-p->baumgarte * d / h, p->max_depen_vel);
      w.rkind[nr] = 2 + side;
      w.rref[nr] = i;
      nr++;
    }
  }
  w.nrows = nr;
  for (int r = 0; r < nr; r++) {
    float s = 0.0f;
    for (int c = 0; c < nv; c++) s += w.J[r][c] * w.Y[r][c];
    w.W[r] = s;
    w.lam[r] = 0.0f;
  }
  for (int it = 0; it < p->pos_iters; it++) {
    for (int r = 0; r < nr; r++) {
      if (w.W[r] <= 1e-12f) continue;
      float v = 0.0f;
      for (int c = 0; c < nv; c++) v += w.J[r][c] * nu[c];
      float lnew = w.lam[r] + (w.bb[r] - v) / w.W[r];
      if (w.rkind[r] == 1) {
        float lim = p->friction * w.lam[3 * w.rref[r]];
        lnew = fminf(fmaxf(lnew, -lim), lim);
      } else {
        lnew = fmaxf(lnew, 0.0f);
      }
      float dl = lnew - w.lam[r];
      w.lam[r] = lnew;
      for (int c = 0; c < nv; c++) nu[c] += w.Y[r][c] * dl;
    }
  }
  // integrate
  if (!m->fixed_base) {
    V3 om = v3(nu[0], nu[1], nu[2]), vo = v3(nu[3], nu[4], nu[5]);
    V3 pn = w.p + vo * h;
    float wn = sqrtf(dot(om, om));
    float dq[4];
    if (wn * h > 1e-12f) {
      float ha = 0.5f * wn * h, sn = sinf(ha) / wn;
      dq[0] = om.x * sn; dq[1] = om.y * sn; dq[2] = om.z * sn; dq[3] = cosf(ha);
    } else {
      dq[0] = 0.5f * h * om.x; dq[1] = 0.5f * h * om.y; dq[2] = 0.5f * h * om.z; dq[3] = 1.0f;
    }
    const float* a = dq;
    const float* b = w.q;
    float qn[4] = {a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1],
                   a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0],
                   a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3],
                   a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]};
    float l = 1.0f / sqrtf(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
    for (int k = 0; k < 4; k++) w.q[k] = qn[k] * l;
    V3 dp = pn - w.p;
    w.p = pn;
    w.nu0 = sv(om, vo + cross(om, dp));
  }
  for (int i = 1; i < nn; i++) {
    w.qd[i] = nu[dof_col(m, i)];
    w.qj[i] += h * w.qd[i];
  }
}

template <int MN, int MC>
__device__ void sensor_outputs(const mg_model* m, ActorWork<MN, MC>& w, const float* tau, float* sensors,
                               float* dof_force) {
  if (sensors && m->num_sensors > 0) {
    fk(m, w);
    for (int si = 0; si < m->num_sensors; si++) {
      const int body = m->sensor_body[si], nd = m->body_node[body];
      M3 Rb = mul(w.R[nd], quat_to_mat(m->body_quat[body][0], m->body_quat[body][1], m->body_quat[body][2],
                                        m->body_quat[body][3]));
      V3 xb = w.x[nd] + mul(w.R[nd], ld3(m->body_pos[body]));
      V3 F = v3(0, 0, 0), T = v3(0, 0, 0);
      for (int c = 0; c < w.ncon; c++) {
        float sg = 0.0f;
        if (m->geom_body[w.cgA[c]] == body) sg = 1.0f;
        else if (w.cgB[c] >= 0 && m->geom_body[w.cgB[c]] == body) sg = -1.0f;
        if (sg == 0.0f) continue;
        V3 t1, t2;
        tangent_basis(w.cn[c], &t1, &t2);
        V3 f = (w.cn[c] * w.lam[3 * c] + t1 * w.lam[3 * c + 1] + t2 * w.lam[3 * c + 2]) * (sg / w.h);
        F = F + f;
        T = T + cross(w.cp[c] - xb, f);
      }
      V3 Fl = mulT(Rb, F), Tl = mulT(Rb, T);
      float* s = sensors + 6 * si;
      s[0] = Fl.x; s[1] = Fl.y; s[2] = Fl.z; s[3] = Tl.x; s[4] = Tl.y; s[5] = Tl.z;
    }
  }
  if (dof_force) {
    for (int i = 1; i < m->num_nodes; i++) {
      float t = (tau ? tau[i - 1] : 0.0f) - m->damping[i] * w.qd[i] - m->stiffness[i] * w.qj[i];
      for (int r = 0; r < w.nrows; r++) {
        if (w.rref[r] != i) continue;
        if (w.rkind[r] == 2) t += w.lam[r] / w.h;
        if (w.rkind[r] == 3) t -= w.lam[r] / w.h;
      }
      dof_force[i - 1] = t;
    }
  }
}

// Whole gym.simulate for one actor: substeps x substep(), then sensors.
template <int MN, int MC>
__device__ void simulate_actor(const mg_model* m, const mg_sim_params* p, float* root, float* dof, const float* tau,
                               float* sensors, float* dof_force) {
  ActorWork<MN, MC> w;
  w.h = p->dt / (float)p->substeps;
  w.ncon = 0;
  w.nrows = 0;
  load_state(m, root, dof, w);
  for (int st = 0; st < p->substeps; st++) substep(m, p, w, tau);
  store_state(m, w, root, dof);
  sensor_outputs(m, w, tau, sensors, dof_force);
}

}  // namespace mg

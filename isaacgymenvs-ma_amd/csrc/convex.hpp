// convex.hpp — narrowphase of articulation geoms against the egg (ellipsoid) object of ShadowHand's
// objectType egg (shadow_hand.py:86-100; open_ai_assets/hand/egg.xml), fp32, one lane per candidate.
// Same algorithm and constants as the oracle's cvx_* functions (oracle/oracle_physics.c), which run it in fp64:
//
//   * everything in the object frame (ellipsoid of semi-axes e centred at the origin);
//   * shape A is a hand geom's core: a segment (sphere / capsule, radius added afterwards) or a box;
//   * GJK distance on A - B: closest point of the simplex by Voronoi-region tests (Ericson 5.1.2,
//     5.1.5, 5.1.6), stop on |v|^2 - v.w <= GJK_REL |v|^2 + 1e-24 (kernel 0.1, oracle 1e-8: the polish below
//     makes the result independent of it; the kernel's GJK only has to find the feature), a repeated support point, no progress
//     or 64 iterations; exit early once a separating plane is farther than the contact offset (such a
//     candidate is no contact, so most broadphase survivors cost one or two support calls);
//   * GJK's witnesses polished to the exact closest pair (cvx_polish): GJK converges linearly against the curved
//     surface and its fp32 stop rule leaves ~1e-3 of direction error in the witnesses (what kept rounds 1-2 in
//     fp64).  The polish solves the optimality conditions on the feature of A that holds the witness -- Newton on
//     the egg point's Lagrange multiplier for a vertex, (t, multiplier) Newton for an edge or the segment, the
//     closed form for a box face -- with an active set over the box's clamped axes, CVX_NEWTON iterations a solve;
//   * box cores are rounded by a 1 mm margin, so penetrations shallower than that (resting contacts)
//     stay with GJK;
//   * overlapping cores -> MPR (Minkowski portal refinement) in fp64 (namespace mpr64): a fixed five-point state
//     (interior point, portal triangle, candidate), so nothing grows per lane the way an EPA polytope would;
//     the penetration vector is the refined portal's point nearest the origin.
//
// Rounds 1-2 ran this in fp64 without the polish: the fp64 working set spilled 186 VGPRs in the egg kernels
// (23x the algorithmic HBM traffic) and cost a quarter of their throughput.  The simplex lives in small fixed
// arrays that the unrolled loops index with constants; the code runs only in the egg instance (OBJ template).
#pragma once
#include "device_math.hpp"

namespace mg {

// GJK stop / no-progress thresholds relative to |v|^2 (fp32)
constexpr float GJK_REL = 1e-1f;  // loose on purpose: the polish resolves the pair
constexpr float GJK_STALL = 1e-7f;
constexpr int CVX_NEWTON = 6;  // Newton iterations per polish solve
constexpr float CVX_MARGIN = 1e-3f;  // rounding of box cores against the egg (m)

struct CvxShape {
  int kind;      // 0 segment [p0, p1], 1 box (centre c, axes = columns of R, half extents h)
  V3 p0, p1;
  V3 c, h;
  float R[3][3];
};

__device__ __forceinline__ V3 cvx_support(const CvxShape& A, V3 d) {
  if (A.kind == 0) return dot(A.p0, d) >= dot(A.p1, d) ? A.p0 : A.p1;
  V3 o = A.c;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const V3 col = v3(A.R[0][k], A.R[1][k], A.R[2][k]);
    const float hk = k == 0 ? A.h.x : (k == 1 ? A.h.y : A.h.z);
    o = o + col * (dot(col, d) >= 0.0f ? hk : -hk);
  }
  return o;
}

// support point of the ellipsoid with semi-axes e in direction d
__device__ __forceinline__ V3 ell_support(V3 e, V3 d) {
  const V3 q = v3(e.x * e.x * d.x, e.y * e.y * d.y, e.z * e.z * d.z);
  const float n = sqrtf(q.x * d.x + q.y * d.y + q.z * d.z);
  if (n < 1e-30f) return v3(0, 0, 0);
  return q * prcp(n);
}

__device__ __forceinline__ void cvx_seg(V3 a, V3 b, float* lam) {
  const V3 ab = b - a;
  const float den = dot(ab, ab);
  float t = den > 0.0f ? -dot(a, ab) * prcp(den) : 0.0f;
  t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
  lam[0] = 1.0f - t;
  lam[1] = t;
}

__device__ __forceinline__ void cvx_tri(V3 a, V3 b, V3 c, float* lam) {
  const V3 ab = b - a, ac = c - a;
  lam[0] = lam[1] = lam[2] = 0.0f;
  const float d1 = -dot(ab, a), d2 = -dot(ac, a);
  if (d1 <= 0.0f && d2 <= 0.0f) { lam[0] = 1.0f; return; }
  const float e3 = -dot(ab, b), d4 = -dot(ac, b);
  if (e3 >= 0.0f && d4 <= e3) { lam[1] = 1.0f; return; }
  const float vc = d1 * d4 - e3 * d2;
  // the edge cases divide by a length that is 0 only for coincident vertices (an MPR portal whose support
  // points repeat): the vertex itself is then the answer, not 0 / 0 (the oracle's cvx_tri likewise)
  if (vc <= 0.0f && d1 >= 0.0f && e3 <= 0.0f) {
    const float v = (d1 - e3) > 0.0f ? d1 * prcp(d1 - e3) : 0.0f;
    lam[0] = 1.0f - v; lam[1] = v; return;
  }
  const float d5 = -dot(ab, c), d6 = -dot(ac, c);
  if (d6 >= 0.0f && d5 <= d6) { lam[2] = 1.0f; return; }
  const float vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0f && d2 >= 0.0f && d6 <= 0.0f) {
    const float w = (d2 - d6) > 0.0f ? d2 * prcp(d2 - d6) : 0.0f;
    lam[0] = 1.0f - w; lam[2] = w; return;
  }
  const float va = e3 * d6 - d5 * d4;
  if (va <= 0.0f && (d4 - e3) >= 0.0f && (d5 - d6) >= 0.0f) {
    const float den2 = (d4 - e3) + (d5 - d6);
    const float w = den2 > 0.0f ? (d4 - e3) * prcp(den2) : 0.0f;
    lam[1] = 1.0f - w;
    lam[2] = w;
    return;
  }
  const float den = va + vb + vc;
  if (!(den > 0.0f)) { cvx_seg(a, b, lam); lam[2] = 0.0f; return; }
  const float iden = prcp(den);
  const float v = vb * iden, w = vc * iden;
  lam[0] = 1.0f - v - w;
  lam[1] = v;
  lam[2] = w;
}

// closest point of the simplex W[0..n-1] to the origin; keeps the supporting vertices in order,
// their weights in lk; returns true if the origin is inside a (non-degenerate) tetrahedron
__device__ __forceinline__ bool cvx_simplex(V3* W, V3* P, int& n, V3& v, float* lk) {
  float lam[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (n == 1) {
    lam[0] = 1.0f;
  } else if (n == 2) {
    cvx_seg(W[0], W[1], lam);
  } else if (n == 3) {
    cvx_tri(W[0], W[1], W[2], lam);
  } else {
    constexpr int F[4][4] = {{0, 1, 2, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {1, 3, 2, 0}};  // face + opposite
    float best = 3.0e38f;
    bool any = false;
#pragma unroll
    for (int f = 0; f < 4; f++) {
      const V3 a = W[F[f][0]], b = W[F[f][1]], c = W[F[f][2]], d = W[F[f][3]];
      const V3 ab = b - a, ac = c - a, ad = d - a;
      const V3 nf = cross(ab, ac);
      const float sp = -dot(nf, a), sd = dot(nf, ad);
      const float sc = dot(ab, ab) + dot(ac, ac) + dot(ad, ad);
      const bool degenerate = sd * sd <= 1e-12f * sc * sc * sc;
      if (!(sp * sd < 0.0f) && !degenerate) continue;
      any = true;
      float l3[3];
      cvx_tri(a, b, c, l3);
      const V3 q = a * l3[0] + b * l3[1] + c * l3[2];
      const float dq = dot(q, q);
      if (dq < best) {
        best = dq;
#pragma unroll
        for (int i = 0; i < 4; i++) lam[i] = 0.0f;
        lam[F[f][0]] = l3[0];
        lam[F[f][1]] = l3[1];
        lam[F[f][2]] = l3[2];
      }
    }
    if (!any) return true;
  }
  // compact in place (a kept vertex only moves down: slot m <= i), no second copy of the simplex
  int m = 0;
  v = v3(0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i < n && lam[i] > 0.0f) {
      v = v + W[i] * lam[i];
#pragma unroll
      for (int j = 0; j <= i; j++)
        if (j == m) { W[j] = W[i]; P[j] = P[i]; lk[j] = lam[i]; }
      m++;
    }
  }
  n = m;
  return false;
}

// GJK distance between core A and the origin-centred ellipsoid e: true when separated (closest
// points pa on A, pb on the ellipsoid, distance), false when the cores overlap
// the core's point nearest the egg's centre in the egg-scaled metric (x / e): the segment's exact
// minimiser of |p(t) / e|^2, or the box centre; true when it lies inside the egg (the cores certainly
// overlap: exact for a segment, sufficient for a box)
__device__ __forceinline__ bool cvx_core_point(const CvxShape& A, V3 e, V3& sp) {
  if (A.kind == 0) {
    const V3 q0 = v3(A.p0.x / e.x, A.p0.y / e.y, A.p0.z / e.z);
    const V3 du = A.p1 - A.p0, qu = v3(du.x / e.x, du.y / e.y, du.z / e.z);
    const float den = dot(qu, qu);
    float t = den > 0.0f ? -dot(q0, qu) / den : 0.0f;
    t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
    sp = A.p0 + du * t;
  } else {
    sp = A.c;
  }
  const float x = sp.x / e.x, y = sp.y / e.y, z = sp.z / e.z;
  return x * x + y * y + z * z < 1.0f;
}

__device__ __forceinline__ int cvx_gjk(const CvxShape& A, V3 e, float cut, V3& pa, V3& pb, float& dist) {
  V3 W[4];
  V3 P[4];  // A-side support points (the witness on A)
  V3 v;
  if (A.kind == 0) {  // start from the segment point nearest the egg in its metric, towards the egg
    V3 sp;
    cvx_core_point(A, e, sp);
    v = sp - ell_support(e, v3(sp.x / (e.x * e.x), sp.y / (e.y * e.y), sp.z / (e.z * e.z)));
  } else {
    v = A.c;
  }
  if (dot(v, v) < 1e-20f) v = v3(0, 0, 1);
  int n = 0;
  float vv = dot(v, v);
  float lam[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int it = 0; it < 64; it++) {
    const V3 a = cvx_support(A, -v), b = ell_support(e, v), w = a - b;
    const float vw = dot(v, w);
    if (vw > 0.0f && vw * vw > vv * cut * cut) {  // separating plane farther than cut: no contact
      dist = vw / sqrtf(vv);
      return 2;
    }
    if (n > 0 && vv - vw <= GJK_REL * vv + 1e-24f) break;
    bool dup = false;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const V3 dd = W[i] - w;
      if (i < n && dot(dd, dd) <= 1e-24f) dup = true;
    }
    if (dup) break;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (i == n) { W[i] = w; P[i] = (a); }
    n++;
    if (cvx_simplex(W, P, n, v, lam)) return 0;
    const float vn = dot(v, v);
    if (vn <= 1e-20f) return 0;
    const bool stall = it > 0 && vn >= vv * (1.0f - GJK_STALL);
    vv = vn;
    if (stall) break;
  }
  pa = v3(0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (i < n) pa = pa + P[i] * lam[i];
  pb = pa - v;
  dist = sqrtf(vv);
  return 1;
}

// Exact closest points from GJK's witnesses (oracle cvx_polish, whose comment has the derivation): Newton on the egg
// point's multiplier lam (b_i = e_i^2 a_i q_i, q_i = 1 / (e_i^2 + lam); a - b = lam a_i q_i) for a vertex of A
// (unknown lam) or an edge a0 + t u (unknowns t, lam), the closed form for a box face, and an active set over the
// box's clamped axes.  CVX_NEWTON iterations per solve from GJK's start (quadratic convergence from the ~0.3 rad of
// direction error its loose stop leaves).
__device__ __forceinline__ float vtx_newton(V3 e2, V3 a, float lam) {
  const V3 t0 = v3(e2.x * a.x * a.x, e2.y * a.y * a.y, e2.z * a.z * a.z);
  for (int it = 0; it < CVX_NEWTON; it++) {
    const float qx = prcp(e2.x + lam), qy = prcp(e2.y + lam), qz = prcp(e2.z + lam);
    const float tx = t0.x * qx * qx, ty = t0.y * qy * qy, tz = t0.z * qz * qz;
    const float F = (tx + ty + tz) - 1.0f, dF = -2.0f * (tx * qx + ty * qy + tz * qz);
    const float ln = dF < 0.0f ? lam - F * prcp(dF) : lam;
    lam = ln > 0.0f ? ln : 0.0f;
  }
  return lam;
}
__device__ __forceinline__ void edge_newton(V3 e2, V3 a0, V3 u, float& t, float& lam) {
  for (int it = 0; it < CVX_NEWTON; it++) {
    const V3 a = a0 + u * t;
    const V3 q = v3(prcp(e2.x + lam), prcp(e2.y + lam), prcp(e2.z + lam));
    const V3 w = v3(e2.x * a.x * q.x * q.x, e2.y * a.y * q.y * q.y, e2.z * a.z * q.z * q.z);  // b_i q_i
    const float F1 = (a.x * w.x + a.y * w.y + a.z * w.z) - 1.0f;
    const float F1l = -2.0f * (a.x * w.x * q.x + a.y * w.y * q.y + a.z * w.z * q.z);
    const float F1t = 2.0f * dot(w, u);
    const float F2 = lam * (q.x * a.x * u.x + q.y * a.y * u.y + q.z * a.z * u.z);
    const float F2l = dot(u, w);
    const float F2t = lam * (u.x * u.x * q.x + u.y * u.y * q.y + u.z * u.z * q.z);
    const float det = F1t * F2l - F1l * F2t;
    if (!(det > 0.0f)) break;
    const float id = prcp(det);
    t += (F1l * F2 - F1 * F2l) * id;
    const float ln = lam + (F2t * F1 - F1t * F2) * id;
    lam = ln > 0.0f ? ln : 0.0f;
  }
}
__device__ __forceinline__ float box_coord(const CvxShape& A, int k, V3 p) {
  return A.R[0][k] * (p.x - A.c.x) + A.R[1][k] * (p.y - A.c.y) + A.R[2][k] * (p.z - A.c.z);
}
__device__ __forceinline__ float hcomp(V3 h, int k) { return k == 0 ? h.x : (k == 1 ? h.y : h.z); }

// polishes (pa, pb) in place and returns the distance (GJK's dist if the polish cannot run)
__device__ __forceinline__ float cvx_polish(const CvxShape& A, V3 e, V3& pa, V3& pb, float dist) {
  const V3 e2 = v3(e.x * e.x, e.y * e.y, e.z * e.z);
  const V3 g = v3(pb.x / e2.x, pb.y / e2.y, pb.z / e2.z);
  const float gg = dot(g, g);
  float lam = gg > 0.0f ? dot(pa - pb, g) / gg : 0.0f;
  lam = lam > 0.0f ? lam : 0.0f;
  V3 a = pa, b = pb;
  bool face = false, ok = true;
  float fd = 0.0f;
  if (A.kind == 0) {  // segment: its interior, else the end on the side the interior solution left by
    const V3 u = A.p1 - A.p0;
    const float uu = dot(u, u);
    float t = uu > 0.0f ? dot(pa - A.p0, u) / uu : 0.0f;
    t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
    const float t0 = t;
    float l = lam;
    if (uu > 0.0f) edge_newton(e2, A.p0, u, t, l);
    if (uu > 0.0f && t > 0.0f && t < 1.0f && isfinite(t) && isfinite(l)) {
      lam = l;
    } else {
      t = (isfinite(t) ? t : t0) < 0.5f ? 0.0f : 1.0f;
      lam = vtx_newton(e2, A.p0 + u * t, lam);
    }
    a = A.p0 + u * t;
  } else {  // box: active set over the axes clamped at +-h
    const float tol = 1e-5f * fmaxf(A.h.x, fmaxf(A.h.y, A.h.z));
    float lc[3];
    int sg[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      lc[k] = box_coord(A, k, pa);
      const float hk = hcomp(A.h, k);
      sg[k] = lc[k] >= hk - tol ? 1 : (lc[k] <= -hk + tol ? -1 : 0);
    }
    bool done = false;
    for (int pass = 0; pass < 6 && !done && ok; pass++) {
      const int m = (sg[0] == 0) + (sg[1] == 0) + (sg[2] == 0);
      if (m == 3) {  // GJK's witness inside the box (an early stop on a simplex across it): start from the face
                     // whose outward normal is nearest the direction to the egg's witness (oracle, the same)
        const V3 dv = pb - pa;
        int kb = 0;
        float best = -1.0f, dkb = 0.0f;
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const float dk = A.R[0][k] * dv.x + A.R[1][k] * dv.y + A.R[2][k] * dv.z;
          if (fabsf(dk) > best) { best = fabsf(dk); kb = k; dkb = dk; }
        }
#pragma unroll
        for (int k = 0; k < 3; k++)
          if (k == kb) sg[k] = dkb >= 0.0f ? 1 : -1;
        continue;
      }
      if (m == 2) {  // face
        const int k = sg[0] ? 0 : (sg[1] ? 1 : 2);
        const float s = (float)sg[k];
        const V3 nf = v3(A.R[0][k], A.R[1][k], A.R[2][k]) * s;
        b = ell_support(e, -nf);
        fd = dot(nf, b - A.c) - hcomp(A.h, k);
        a = b - nf * fd;
        bool moved = false;
#pragma unroll
        for (int j = 0; j < 3; j++) {
          const float lj = box_coord(A, j, a), hj = hcomp(A.h, j);
          if (j != k && (lj > hj || lj < -hj)) { sg[j] = lj > 0.0f ? 1 : -1; moved = true; }
        }
        if (!moved) { face = true; done = true; }
        continue;
      }
      V3 a0 = A.c;
      int jf = 0;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        if (sg[k] == 0) jf = k;
        else a0 = a0 + v3(A.R[0][k], A.R[1][k], A.R[2][k]) * ((float)sg[k] * hcomp(A.h, k));
      }
      if (m == 1) {  // edge along axis jf
        const V3 u = v3(A.R[0][jf], A.R[1][jf], A.R[2][jf]);
        float t = jf == 0 ? lc[0] : (jf == 1 ? lc[1] : lc[2]), l = lam;
        edge_newton(e2, a0, u, t, l);
        const float hj = hcomp(A.h, jf);
        if (!(isfinite(t) && isfinite(l))) { ok = false; break; }
        if (t > hj || t < -hj) {
#pragma unroll
          for (int k = 0; k < 3; k++)
            if (k == jf) sg[k] = t > 0.0f ? 1 : -1;
          continue;
        }
        lam = l;
        a = a0 + u * t;
      } else {  // vertex
        a = a0;
        lam = vtx_newton(e2, a, lam);
      }
      // optimal only if b - a (along -a_i q_i) leaves A through every clamped face: an axis it does not is freed
      const V3 sv = v3(-a.x / (e2.x + lam), -a.y / (e2.y + lam), -a.z / (e2.z + lam));
      const float sl = sqrtf(dot(sv, sv));
      bool freed = false;
#pragma unroll
      for (int k = 0; k < 3; k++)
        if (sg[k] != 0 && (float)sg[k] * box_coord(A, k, A.c + sv) < -1e-6f * sl) { sg[k] = 0; freed = true; }
      if (freed) {
#pragma unroll
        for (int k = 0; k < 3; k++) lc[k] = box_coord(A, k, a);  // the free coordinates restart from here
        continue;
      }
      done = true;
    }
    ok = ok && done;
  }
  if (!ok) return dist;
  float d = fd;
  if (!face) {
    const V3 q = v3(prcp(e2.x + lam), prcp(e2.y + lam), prcp(e2.z + lam));
    b = v3(e2.x * a.x * q.x, e2.y * a.y * q.y, e2.z * a.z * q.z);
    const V3 sv = v3(a.x * q.x, a.y * q.y, a.z * q.z) * lam;
    d = sqrtf(dot(sv, sv));
  }
  if (!(isfinite(a.x) && isfinite(a.y) && isfinite(a.z) && isfinite(b.x) && isfinite(b.y) && isfinite(b.z) && isfinite(d)))
    return dist;
  pa = a;
  pb = b;
  return d;
}

// MPR in fp64 (namespace mpr64): overlapping cores are rare (a box core more than its 1 mm margin deep, a capsule
// core inside the egg), and the portal sequence is a chain of sign decisions on nearly coplanar points, which an
// fp32 run resolves differently from the oracle's fp64 one in a few % of deep states (whose depenetration impulses
// then differ).  Its fp64 state is live only inside this branch.
namespace mpr64 {
typedef double creal;
struct D3 {
  creal x, y, z;
};
__device__ __forceinline__ D3 d3(creal x, creal y, creal z) { return D3{x, y, z}; }
__device__ __forceinline__ D3 d3(V3 a) { return D3{a.x, a.y, a.z}; }
__device__ __forceinline__ V3 f3(D3 a) { return v3((float)a.x, (float)a.y, (float)a.z); }
__device__ __forceinline__ D3 operator+(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ D3 operator-(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ D3 operator*(D3 a, creal s) { return d3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ D3 operator-(D3 a) { return d3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ creal dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ D3 cross(D3 a, D3 b) {
  return d3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

struct CvxShape {
  int kind;      // 0 segment [p0, p1], 1 box (centre c, axes = columns of R, half extents h)
  D3 p0, p1;
  D3 c, h;
  creal R[3][3];
};

__device__ __forceinline__ D3 cvx_support(const CvxShape& A, D3 d) {
  if (A.kind == 0) return dot(A.p0, d) >= dot(A.p1, d) ? A.p0 : A.p1;
  D3 o = A.c;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const D3 col = d3(A.R[0][k], A.R[1][k], A.R[2][k]);
    const creal hk = k == 0 ? A.h.x : (k == 1 ? A.h.y : A.h.z);
    o = o + col * (dot(col, d) >= 0.0 ? hk : -hk);
  }
  return o;
}

// support point of the ellipsoid with semi-axes e in direction d
__device__ __forceinline__ D3 ell_support(D3 e, D3 d) {
  const D3 q = d3(e.x * e.x * d.x, e.y * e.y * d.y, e.z * e.z * d.z);
  const creal n = sqrt(q.x * d.x + q.y * d.y + q.z * d.z);
  if (n < 1e-30) return d3(0, 0, 0);
  return q * (1.0 / n);
}

__device__ __forceinline__ void cvx_seg(D3 a, D3 b, creal* lam) {
  const D3 ab = b - a;
  const creal den = dot(ab, ab);
  creal t = den > 0.0 ? -dot(a, ab) / den : 0.0;
  t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
  lam[0] = 1.0 - t;
  lam[1] = t;
}

__device__ __forceinline__ void cvx_tri(D3 a, D3 b, D3 c, creal* lam) {
  const D3 ab = b - a, ac = c - a;
  lam[0] = lam[1] = lam[2] = 0.0;
  const creal d1 = -dot(ab, a), d2 = -dot(ac, a);
  if (d1 <= 0.0 && d2 <= 0.0) { lam[0] = 1.0; return; }
  const creal e3 = -dot(ab, b), d4 = -dot(ac, b);
  if (e3 >= 0.0 && d4 <= e3) { lam[1] = 1.0; return; }
  const creal vc = d1 * d4 - e3 * d2;
  // the edge cases divide by a length that is 0 only for coincident vertices (an MPR portal whose support
  // points repeat): the vertex itself is then the answer, not 0 / 0 (the oracle's cvx_tri likewise)
  if (vc <= 0.0 && d1 >= 0.0 && e3 <= 0.0) {
    const creal v = (d1 - e3) > 0.0 ? d1 / (d1 - e3) : 0.0;
    lam[0] = 1.0 - v; lam[1] = v; return;
  }
  const creal d5 = -dot(ab, c), d6 = -dot(ac, c);
  if (d6 >= 0.0 && d5 <= d6) { lam[2] = 1.0; return; }
  const creal vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {
    const creal w = (d2 - d6) > 0.0 ? d2 / (d2 - d6) : 0.0;
    lam[0] = 1.0 - w; lam[2] = w; return;
  }
  const creal va = e3 * d6 - d5 * d4;
  if (va <= 0.0 && (d4 - e3) >= 0.0 && (d5 - d6) >= 0.0) {
    const creal den2 = (d4 - e3) + (d5 - d6);
    const creal w = den2 > 0.0 ? (d4 - e3) / den2 : 0.0;
    lam[1] = 1.0 - w;
    lam[2] = w;
    return;
  }
  const creal den = va + vb + vc;
  if (!(den > 0.0)) { cvx_seg(a, b, lam); lam[2] = 0.0; return; }
  const creal v = vb / den, w = vc / den;
  lam[0] = 1.0 - v - w;
  lam[1] = v;
  lam[2] = w;
}

constexpr creal MPR_TOL = 1e-7;   // portal reached the boundary (m)
constexpr creal MPR_EPS = 1e-12;  // origin-side tests

__device__ __forceinline__ D3 unit3(D3 a) {
  const creal l = sqrt(dot(a, a));
  return l > 0.0 ? a * (1.0 / l) : a;
}

// MPR penetration for overlapping cores: the boundary point x of A - B (moving A by -x separates
// them) and the A-side witness pa; false if the portal search degenerates
__device__ __forceinline__ bool cvx_mpr(const CvxShape& A, D3 e, D3& x, D3& pa) {
  D3 v0 = A.kind == 0 ? (A.p0 + A.p1) * 0.5 : A.c;
  if (dot(v0, v0) < 1e-20) v0 = d3(1e-6, 0, 0);
  D3 dir = unit3(-v0);
  const D3 s1 = cvx_support(A, dir);
  D3 v1 = s1 - ell_support(e, -dir);
  V3 a1 = f3(s1);  // A-side points in fp32: only the final witness reads them
  if (dot(v1, dir) <= 0.0) return false;
  dir = cross(v0, v1);
  if (dot(dir, dir) <= 1e-24) { x = v1; pa = d3(a1); return true; }
  dir = unit3(dir);
  const D3 s2 = cvx_support(A, dir);
  D3 v2 = s2 - ell_support(e, -dir);
  V3 a2 = f3(s2);
  if (dot(v2, dir) <= 0.0) return false;
  dir = unit3(cross(v1 - v0, v2 - v0));
  if (dot(dir, v0) > 0.0) {
    const D3 t = v1; v1 = v2; v2 = t;
    const V3 ta = a1; a1 = a2; a2 = ta;
    dir = -dir;
  }
  D3 v3p;
  V3 a3;
  int it;
  for (it = 0; it < 64; it++) {  // a portal the origin ray passes through
    const D3 s3 = cvx_support(A, dir);
    v3p = s3 - ell_support(e, -dir);
    a3 = f3(s3);
    if (dot(v3p, dir) <= 0.0) return false;
    if (dot(cross(v1, v3p), v0) < -MPR_EPS) {
      v2 = v3p; a2 = a3;
    } else if (dot(cross(v3p, v2), v0) < -MPR_EPS) {
      v1 = v3p; a1 = a3;
    } else {
      break;
    }
    dir = unit3(cross(v1 - v0, v2 - v0));
  }
  if (it == 64) return false;
  // expand: replace one portal vertex by v4 so that the portal keeps facing the origin ray
  auto expand = [&](D3 v4, V3 a4) {
    const D3 c = cross(v4, v0);
    int k;
    if (dot(v1, c) > 0.0) k = dot(v2, c) > 0.0 ? 1 : 3;
    else k = dot(v3p, c) > 0.0 ? 2 : 1;
    if (k == 1) { v1 = v4; a1 = a4; }
    else if (k == 2) { v2 = v4; a2 = a4; }
    else { v3p = v4; a3 = a4; }
  };
  auto reached = [&](D3 v4, D3 d) {
    const creal d4 = dot(v4, d);
    const creal mm = fmin(d4 - dot(v1, d), fmin(d4 - dot(v2, d), d4 - dot(v3p, d)));
    return mm <= MPR_TOL;
  };
  for (it = 0; it < 64; it++) {  // refine until the portal encloses the origin
    dir = unit3(cross(v2 - v1, v3p - v1));
    if (dot(v1, dir) >= 0.0) break;
    const D3 s4 = cvx_support(A, dir), v4 = s4 - ell_support(e, -dir);
    if (dot(v4, dir) < 0.0 || reached(v4, dir)) return false;
    expand(v4, f3(s4));
  }
  if (it == 64) return false;
  for (it = 0;; it++) {  // push the portal onto the boundary
    dir = unit3(cross(v2 - v1, v3p - v1));
    const D3 s4 = cvx_support(A, dir), v4 = s4 - ell_support(e, -dir);
    if (reached(v4, dir) || it >= 64) break;
    expand(v4, f3(s4));
  }
  creal lam[3];
  cvx_tri(v1, v2, v3p, lam);
  x = v1 * lam[0] + v2 * lam[1] + v3p * lam[2];
  pa = d3(a1) * lam[0] + d3(a2) * lam[1] + d3(a3) * lam[2];
  return true;
}

}  // namespace mpr64

// Exact penetration of a segment core overlapping the ellipsoid (the minimum translation), as the oracle's
// seg_mtd, in fp32: the vertex solutions (an end inside: its distance to the surface, valid when the other end is
// not deeper along that normal; the first valid one is the minimum) or the edge one (the shadow point's distance to
// the shadow ellipse's boundary in the plane normal to u), each the nearest-boundary-point root lam in (-min s, 0]
// by Newton's method from 0.  A smooth function of the state (no portal decisions, unlike MPR), so fp32 suffices;
// fp64 raised the egg kernel's spills (14 -> 29) and its traffic (309 -> 350 MB per launch).
__device__ __forceinline__ float ell_root(int k, const float* s2, const float* q) {
  float smin = s2[0];
  for (int i = 1; i < k; i++) smin = fminf(smin, s2[i]);
  float lam = 0.0f;
  for (int it = 0; it < 32; it++) {
    float f = -1.0f, fp = 0.0f;
    for (int i = 0; i < k; i++) {
      const float den = s2[i] + lam, r = s2[i] * q[i] * q[i] / (den * den);
      f += r;
      fp -= 2.0f * r / den;
    }
    if (!(fp < 0.0f)) break;
    float nl = lam - f / fp;
    if (!(nl > -smin)) nl = 0.5f * (lam - smin);
    if (nl > 0.0f) nl = 0.0f;
    const float dl = fabsf(nl - lam);
    lam = nl;
    if (dl <= 1e-7f * smin) break;
  }
  return lam;
}
__device__ __forceinline__ bool mtd_vertex(V3 e, V3 p, V3& n, float& depth) {
  const float s2[3] = {e.x * e.x, e.y * e.y, e.z * e.z};
  if (!(p.x * p.x / s2[0] + p.y * p.y / s2[1] + p.z * p.z / s2[2] < 1.0f)) return false;
  const float q[3] = {p.x, p.y, p.z};
  const float lam = ell_root(3, s2, q);
  const V3 g = v3(p.x / (s2[0] + lam), p.y / (s2[1] + lam), p.z / (s2[2] + lam));
  const float gl = sqrtf(dot(g, g));
  if (!(gl > 0.0f) || !isfinite(gl)) return false;
  n = g * (1.0f / gl);
  depth = -lam * gl;
  return true;
}
__device__ __forceinline__ bool seg_mtd(const CvxShape& A, V3 e, V3& n, float& depth, V3& pa) {
  const V3 u = A.p1 - A.p0;
  const float uu = dot(u, u);
  if (mtd_vertex(e, A.p0, n, depth) && (uu == 0.0f || dot(n, u) >= 0.0f)) { pa = A.p0; return true; }
  if (!(uu > 0.0f)) return false;
  if (mtd_vertex(e, A.p1, n, depth) && dot(n, u) <= 0.0f) { pa = A.p1; return true; }
  const V3 uh = u * (1.0f / sqrtf(uu));
  const int ax = fabsf(uh.x) <= fabsf(uh.y) ? (fabsf(uh.x) <= fabsf(uh.z) ? 0 : 2) : (fabsf(uh.y) <= fabsf(uh.z) ? 1 : 2);
  V3 w1 = cross(uh, v3(ax == 0 ? 1.0f : 0.0f, ax == 1 ? 1.0f : 0.0f, ax == 2 ? 1.0f : 0.0f));
  w1 = w1 * (1.0f / sqrtf(dot(w1, w1)));
  const V3 w2 = cross(uh, w1);
  const float sx = e.x * e.x, sy = e.y * e.y, sz = e.z * e.z;
  const float S00 = w1.x * w1.x * sx + w1.y * w1.y * sy + w1.z * w1.z * sz;
  const float S01 = w1.x * w2.x * sx + w1.y * w2.y * sy + w1.z * w2.z * sz;
  const float S11 = w2.x * w2.x * sx + w2.y * w2.y * sy + w2.z * w2.z * sz;
  const float tr = 0.5f * (S00 + S11), df = 0.5f * (S00 - S11), rad = sqrtf(df * df + S01 * S01);
  const float l2[2] = {tr + rad, tr - rad};
  float c0 = 1.0f, c1 = 0.0f;  // eigenvector of l2[0] from the row without cancellation (the oracle's note)
  if (rad > 1e-30f) {
    const float x = df >= 0.0f ? df + rad : S01, y = df >= 0.0f ? S01 : rad - df, yl = sqrtf(x * x + y * y);
    if (yl > 1e-30f) { c0 = x / yl; c1 = y / yl; }
  } else if (df < 0.0f) { c0 = 0.0f; c1 = 1.0f; }
  const float q0 = dot(w1, A.p0), q1 = dot(w2, A.p0);
  const float q[2] = {c0 * q0 + c1 * q1, -c1 * q0 + c0 * q1};
  if (!(l2[1] > 0.0f) || !(q[0] * q[0] / l2[0] + q[1] * q[1] / l2[1] < 1.0f)) return false;
  const float lam = ell_root(2, l2, q);
  const float g0 = q[0] / (l2[0] + lam), g1 = q[1] / (l2[1] + lam), gl = sqrtf(g0 * g0 + g1 * g1);
  if (!(gl > 0.0f) || !isfinite(gl)) return false;
  const float m0 = (c0 * g0 - c1 * g1) / gl, m1 = (c1 * g0 + c0 * g1) / gl;
  n = w1 * m0 + w2 * m1;
  depth = -lam * gl;
  const V3 b = ell_support(e, n);
  float t = dot(b - A.p0, u) / uu;
  t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
  pa = A.p0 + u * t;
  return true;
}

__device__ __forceinline__ bool cvx_finite(V3 p, V3 n, float d) {
  return isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && isfinite(n.x) && isfinite(n.y) && isfinite(n.z) &&
         isfinite(d);
}

// the narrowphase result: contact point, normal from the object to A, signed distance
struct CvxHit {
  V3 pt, nrm;
  float d;
};

// one contact between core A (+ radius rA) and the ellipsoid e (object frame): GJK when apart; when overlapping
// the exact penetration for a segment core, MPR for a box core; the centre direction if those degenerate.  Normal
// from the object to A.
__device__ __forceinline__ CvxHit cvx_contact_body(CvxShape A, float rA, V3 e, float cut) {
  CvxHit o;
  V3 pa, pb;
  float dist;
  if (A.kind == 1) {  // box cores rounded by CVX_MARGIN (see the oracle): resting contacts stay with GJK
    const float mg = fminf(CVX_MARGIN, 0.5f * fminf(A.h.x, fminf(A.h.y, A.h.z)));
    A.h = A.h - v3(mg, mg, mg);
    rA += mg;
  }
  V3 sp;
  const int g = cvx_core_point(A, e, sp) ? 0 : cvx_gjk(A, e, rA + cut, pa, pb, dist);  // overlap: MPR
  if (g == 2) {  // farther than rA + cut: only the (lower-bound) distance is meaningful
    o.d = dist - rA;
    o.nrm = v3(0, 0, 1);
    o.pt = v3(0, 0, 0);
    return o;
  }
  if (g && dist > 1e-9f) {
    dist = cvx_polish(A, e, pa, pb, dist);
    // the egg's surface normal at its witness point (gradient of the implicit function): better
    // conditioned than (pa - pb) / dist when the gap is small
    const V3 gr = v3(pb.x / (e.x * e.x), pb.y / (e.y * e.y), pb.z / (e.z * e.z));
    const float gl = dot(gr, gr);
    o.nrm = gl > 1e-30f ? gr * (1.0f / sqrtf(gl)) : (pa - pb) * (1.0f / dist);
    o.pt = ((pa - o.nrm * rA) + pb) * 0.5f;
    o.d = dist - rA;
    if (cvx_finite(o.pt, o.nrm, o.d)) return o;
  } else if (A.kind == 0) {  // a segment core: the exact penetration
    V3 nd, pa2;
    float dep;
    if (seg_mtd(A, e, nd, dep, pa2)) {
      o.nrm = nd;
      o.pt = pa2 + nd * (0.5f * dep) - nd * (0.5f * rA);
      o.d = -dep - rA;
      if (cvx_finite(o.pt, o.nrm, o.d)) return o;
    }
  } else {
    mpr64::CvxShape A64;
    A64.kind = A.kind;
    A64.p0 = mpr64::d3(A.p0);
    A64.p1 = mpr64::d3(A.p1);
    A64.c = mpr64::d3(A.c);
    A64.h = mpr64::d3(A.h);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int k = 0; k < 3; k++) A64.R[i][k] = A.R[i][k];
    mpr64::D3 x, pa;
    if (mpr64::cvx_mpr(A64, mpr64::d3(e), x, pa)) {
      const double l = sqrt(mpr64::dot(x, x));
      if (l > 1e-9) {
        const mpr64::D3 nd = x * (-1.0 / l);
        o.nrm = mpr64::f3(nd);
        o.pt = mpr64::f3((pa - x * 0.5) - nd * (rA * 0.5));
        o.d = (float)(-l - rA);
        if (cvx_finite(o.pt, o.nrm, o.d)) return o;
      }
    }
  }
  // MPR degenerate, or a non-finite result of a degenerate simplex: the centre direction
  const V3 ca = A.kind == 0 ? (A.p0 + A.p1) * 0.5f : A.c;
  const float l = sqrtf(dot(ca, ca));
  o.nrm = l > 1e-12f ? ca * (1.0f / l) : v3(0, 0, 1);
  o.pt = ca * 0.5f;
  o.d = -rA;
  return o;
}

// The narrowphase entry: the core as five 3-vectors (segment: p0, p1; box: centre, half extents, the three
// axis columns), the result by value.  Force-inlined into collide().
//
// A real call (noinline) was tried in round 3 (the fp64 version) and found unsafe with this toolchain (ROCm 7.2
// LLVM): wrong object states with interprocedural register allocation on, and two later miscompiles with it off
// (profiles/r03/egg_call_ab.txt).  The fp32 narrowphase is inlined like every other phase.
__device__ __forceinline__ CvxHit cvx_contact_v(int kind, V3 a0, V3 a1, V3 a2, V3 a3, V3 a4, float rA, V3 e,
                                              float cut) {
  CvxShape A;
  A.kind = kind;
  if (kind == 0) {
    A.p0 = a0;
    A.p1 = a1;
  } else {
    A.c = a0;
    A.h = a1;
    const V3 col[3] = {a2, a3, a4};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      A.R[0][k] = col[k].x;
      A.R[1][k] = col[k].y;
      A.R[2][k] = col[k].z;
    }
  }
  return cvx_contact_body(A, rA, e, cut);
}

}  // namespace mg

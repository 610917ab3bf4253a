// convex.hpp — narrowphase of articulation geoms against the egg (ellipsoid) object of ShadowHand's
// objectType egg (shadow_hand.py:86-100; open_ai_assets/hand/egg.xml), fp64, one lane per candidate.
// Same algorithm and constants as the oracle's cvx_* functions (oracle/oracle_physics.c):
//
//   * everything in the object frame (ellipsoid of semi-axes e centred at the origin);
//   * shape A is a hand geom's core: a segment (sphere / capsule, radius added afterwards) or a box;
//   * GJK distance on A - B: closest point of the simplex by Voronoi-region tests (Ericson 5.1.2,
//     5.1.5, 5.1.6), stop on |v|^2 - v.w <= 1e-8 |v|^2 + 1e-24, a repeated support point, no progress
//     or 64 iterations; exit early once a separating plane is farther than the contact offset (such a
//     candidate is no contact, so most broadphase survivors cost one or two support calls);
//   * box cores are rounded by a 1 mm margin, so penetrations shallower than that (resting contacts)
//     stay with GJK;
//   * overlapping cores -> MPR (Minkowski portal refinement): a fixed five-point state (interior
//     point, portal triangle, candidate), so nothing grows per lane the way an EPA polytope would;
//     the penetration vector is the refined portal's point nearest the origin.
//
// The narrowphase runs in fp64 (the CDNA4 VALU's fp64 rate is ample for a few candidates per env):
// GJK against a curved surface converges linearly, and an fp32 stop criterion leaves ~1e-3 of
// direction error in the contact normal; in fp64 the normal is resolved to ~1e-5 and the kernel
// follows the fp64 oracle.  The simplex lives in small fixed arrays that the unrolled loops index
// with constants; the code runs only for the egg, behind a wave-uniform branch on the object type.
#pragma once
#include "device_math.hpp"

namespace mg {

// the narrowphase scalar type (fp64, see the header note)
typedef double creal;
struct D3 {
  creal x, y, z;
};
__device__ __forceinline__ D3 d3(creal x, creal y, creal z) { return D3{x, y, z}; }
__device__ __forceinline__ D3 d3(V3 a) { return D3{a.x, a.y, a.z}; }
// GJK stop / no-progress thresholds: relative to |v|^2, within reach of the scalar's precision
constexpr creal GJK_REL = sizeof(creal) == 4 ? (creal)1e-6 : (creal)1e-8;
constexpr creal GJK_STALL = sizeof(creal) == 4 ? (creal)1e-7 : (creal)1e-14;
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

// closest point of the simplex W[0..n-1] to the origin; keeps the supporting vertices in order,
// their weights in lk; returns true if the origin is inside a (non-degenerate) tetrahedron
__device__ __forceinline__ bool cvx_simplex(D3* W, V3* P, int& n, D3& v, creal* lk) {
  creal lam[4] = {0.0, 0.0, 0.0, 0.0};
  if (n == 1) {
    lam[0] = 1.0;
  } else if (n == 2) {
    cvx_seg(W[0], W[1], lam);
  } else if (n == 3) {
    cvx_tri(W[0], W[1], W[2], lam);
  } else {
    constexpr int F[4][4] = {{0, 1, 2, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {1, 3, 2, 0}};  // face + opposite
    creal best = (creal)3.0e38;
    bool any = false;
#pragma unroll
    for (int f = 0; f < 4; f++) {
      const D3 a = W[F[f][0]], b = W[F[f][1]], c = W[F[f][2]], d = W[F[f][3]];
      const D3 ab = b - a, ac = c - a, ad = d - a;
      const D3 nf = cross(ab, ac);
      const creal sp = -dot(nf, a), sd = dot(nf, ad);
      const creal sc = dot(ab, ab) + dot(ac, ac) + dot(ad, ad);
      const bool degenerate = sd * sd <= 1e-12 * sc * sc * sc;
      if (!(sp * sd < 0.0) && !degenerate) continue;
      any = true;
      creal l3[3];
      cvx_tri(a, b, c, l3);
      const D3 q = a * l3[0] + b * l3[1] + c * l3[2];
      const creal dq = dot(q, q);
      if (dq < best) {
        best = dq;
#pragma unroll
        for (int i = 0; i < 4; i++) lam[i] = 0.0;
        lam[F[f][0]] = l3[0];
        lam[F[f][1]] = l3[1];
        lam[F[f][2]] = l3[2];
      }
    }
    if (!any) return true;
  }
  // compact in place (a kept vertex only moves down: slot m <= i), no second copy of the simplex
  int m = 0;
  v = d3(0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i < n && lam[i] > 0.0) {
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
__device__ __forceinline__ bool cvx_core_point(const CvxShape& A, D3 e, D3& sp) {
  if (A.kind == 0) {
    const D3 q0 = d3(A.p0.x / e.x, A.p0.y / e.y, A.p0.z / e.z);
    const D3 du = A.p1 - A.p0, qu = d3(du.x / e.x, du.y / e.y, du.z / e.z);
    const creal den = dot(qu, qu);
    creal t = den > 0.0 ? -dot(q0, qu) / den : 0.0;
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    sp = A.p0 + du * t;
  } else {
    sp = A.c;
  }
  const creal x = sp.x / e.x, y = sp.y / e.y, z = sp.z / e.z;
  return x * x + y * y + z * z < 1.0;
}

__device__ __forceinline__ int cvx_gjk(const CvxShape& A, D3 e, creal cut, D3& pa, D3& pb, creal& dist) {
  D3 W[4];
  V3 P[4];  // A-side support points: only the final witness reads them, fp32 is enough (halves their registers)
  D3 v;
  if (A.kind == 0) {  // start from the segment point nearest the egg in its metric, towards the egg
    D3 sp;
    cvx_core_point(A, e, sp);
    v = sp - ell_support(e, d3(sp.x / (e.x * e.x), sp.y / (e.y * e.y), sp.z / (e.z * e.z)));
  } else {
    v = A.c;
  }
  if (dot(v, v) < 1e-20) v = d3(0, 0, 1);
  int n = 0;
  creal vv = dot(v, v);
  creal lam[4] = {0.0, 0.0, 0.0, 0.0};
  for (int it = 0; it < 64; it++) {
    const D3 a = cvx_support(A, -v), b = ell_support(e, v), w = a - b;
    const creal vw = dot(v, w);
    if (vw > 0.0 && vw * vw > vv * cut * cut) {  // separating plane farther than cut: no contact
      dist = vw / sqrt(vv);
      return 2;
    }
    if (n > 0 && vv - vw <= GJK_REL * vv + (creal)1e-24) break;
    bool dup = false;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const D3 dd = W[i] - w;
      if (i < n && dot(dd, dd) <= 1e-24) dup = true;
    }
    if (dup) break;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (i == n) { W[i] = w; P[i] = f3(a); }
    n++;
    if (cvx_simplex(W, P, n, v, lam)) return 0;
    const creal vn = dot(v, v);
    if (vn <= 1e-20) return 0;
    const bool stall = it > 0 && vn >= vv * ((creal)1.0 - GJK_STALL);
    vv = vn;
    if (stall) break;
  }
  pa = d3(0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (i < n) pa = pa + d3(P[i]) * lam[i];
  pb = pa - v;
  dist = sqrt(vv);
  return 1;
}

constexpr creal MPR_TOL = 1e-7;   // portal reached the boundary (m)
constexpr creal CVX_MARGIN = 1e-3;  // rounding of box cores against the egg (m)
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

__device__ __forceinline__ bool cvx_finite(D3 p, D3 n, creal d) {
  return isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && isfinite(n.x) && isfinite(n.y) && isfinite(n.z) &&
         isfinite(d);
}

// the narrowphase result: contact point, normal from the object to A, signed distance
struct CvxHit {
  D3 pt, nrm;
  creal d;
};

// one contact between core A (+ radius rA) and the ellipsoid e (object frame): GJK when apart, MPR
// when overlapping, the centre direction if MPR degenerates.  Normal from the object to A.
__device__ __forceinline__ CvxHit cvx_contact_body(CvxShape A, creal rA, D3 e, creal cut) {
  CvxHit o;
  D3 pa, pb, x;
  creal dist;
  if (A.kind == 1) {  // box cores rounded by CVX_MARGIN (see the oracle): resting contacts stay with GJK
    const creal mg = fmin(CVX_MARGIN, 0.5 * fmin(A.h.x, fmin(A.h.y, A.h.z)));
    A.h = A.h - d3(mg, mg, mg);
    rA += mg;
  }
  D3 sp;
  const int g = cvx_core_point(A, e, sp) ? 0 : cvx_gjk(A, e, rA + cut, pa, pb, dist);  // overlap: MPR
  if (g == 2) {  // farther than rA + cut: only the (lower-bound) distance is meaningful
    o.d = dist - rA;
    o.nrm = d3(0, 0, 1);
    o.pt = d3(0, 0, 0);
    return o;
  }
  if (g && dist > 1e-9) {
    // the egg's surface normal at its witness point (gradient of the implicit function): better
    // conditioned than (pa - pb) / dist when the gap is small
    const D3 gr = d3(pb.x / (e.x * e.x), pb.y / (e.y * e.y), pb.z / (e.z * e.z));
    const creal gl = dot(gr, gr);
    o.nrm = gl > 1e-30 ? gr * (1.0 / sqrt(gl)) : (pa - pb) * (1.0 / dist);
    o.pt = ((pa - o.nrm * rA) + pb) * 0.5;
    o.d = dist - rA;
    if (cvx_finite(o.pt, o.nrm, o.d)) return o;
  } else if (cvx_mpr(A, e, x, pa)) {
    const creal l = sqrt(dot(x, x));
    if (l > 1e-9) {
      o.nrm = x * (-1.0 / l);
      o.pt = (pa - x * 0.5) - o.nrm * (rA * 0.5);
      o.d = -l - rA;
      if (cvx_finite(o.pt, o.nrm, o.d)) return o;
    }
  }
  // MPR degenerate, or a non-finite result of a degenerate simplex: the centre direction
  const D3 ca = A.kind == 0 ? (A.p0 + A.p1) * 0.5 : A.c;
  const creal l = sqrt(dot(ca, ca));
  o.nrm = l > 1e-12 ? ca * (1.0 / l) : d3(0, 0, 1);
  o.pt = ca * 0.5;
  o.d = -rA;
  return o;
}

// The narrowphase entry: the core as five 3-vectors (segment: p0, p1; box: centre, half extents, the three
// axis columns), the result by value.  Force-inlined into collide().
//
// A real call (noinline) was tried in round 3 and is not safe with this toolchain (ROCm 7.2 LLVM): with
// interprocedural register allocation on, k_simulate's egg step was wrong in 222 of 256 envs; with it off
// (-mllvm -enable-ipra=false, still passed for the instance TUs) the call passed every egg test, but two
// unrelated edits of the calling kernel then broke it again -- the narrowphase staged after fk() as a call
// faulted (illegal address), and a prefetching rewrite of fk()'s ancestor walk left the DR egg test 93 %
// in agreement -- while the same sources with the narrowphase inlined passed (profiles/r03/egg_call_ab.txt).
// A static check of that build's code object found the callee's saves and the caller's restores in order,
// so the miscompile is not pinned down; inlining costs 0.6 % of egg throughput against the call.
__device__ __forceinline__ CvxHit cvx_contact_v(int kind, D3 a0, D3 a1, D3 a2, D3 a3, D3 a4, creal rA, D3 e,
                                              creal cut) {
  CvxShape A;
  A.kind = kind;
  if (kind == 0) {
    A.p0 = a0;
    A.p1 = a1;
  } else {
    A.c = a0;
    A.h = a1;
    const D3 col[3] = {a2, a3, a4};
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

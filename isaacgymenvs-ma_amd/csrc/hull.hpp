// hull.hpp — the convex-mesh hull (ShadowHand's forearm, robot.xml:8 / shared_asset.xml:15) against the
// object's core, exactly: SURVEY.md §8(a) A6.  Same algorithm and constants as the oracle's hull_core_contacts
// (oracle/oracle_physics.c, whose header comment states the rules):
//
//   * GJK on the Minkowski difference hull - core in the hull's geom frame: A = the hull (support: its
//     vertices, ties to the lowest index), B = the cube's core shrunk by HULL_MARGIN and rounded by it, or the
//     pen's segment with the pen's radius; overlapping cores: MPR from the interior point (hull vertex
//     centroid - core centre);
//   * the features at the witnesses decide: edge against edge (not near parallel, neither edge lying on a face
//     of the other shape) gives one contact (the cube's on its sharp edge: the rounded core finds the features); the pen's interior over a hull face gives the
//     ends of the segment's part over that face (clipped by every other plane), strictly inside the segment,
//     with the face's normal and their own plane gaps; anything with a vertex among its closest features is
//     the vertex-face candidates' case.
//
// fp32, unlike the egg's narrowphase (convex.hpp): GJK on two polytopes ends on the exact closest features
// after finitely many steps (no curved surface whose linear convergence would need fp64 to resolve the
// normal), and the fp64 state of the same code cost the block / pen kernels 11-36 % of their throughput in
// register pressure (same-box A/B, round 3) although it runs only with the object at the forearm.  The oracle
// runs it in fp64.
//
// Team-cooperative: every lane of the team runs the same simplex arithmetic on the same values (control flow
// is uniform within the team); the loops over the hull's vertices and planes are spread over the team's lanes
// (a support is one team argmax; the planes through a witness one ballot per T planes; the face clipping a
// team max / min).  Called once per substep before the tree phases (Team::hull_stage), where little else is
// live: the forearm is on the hand's fixed root, so its pose and the object's are those collide() sees.
#pragma once
#include "../../include/migym.h"
#include "device_math.hpp"

namespace mg {

static_assert(offsetof(mg_model, hull_plane) % 16 == 0, "the hull's planes are read as float4");

#ifndef MG_HULL_SUP_UNROLL
#define MG_HULL_SUP_UNROLL 2  // hull_support: the lane's vertex reads issued together
#endif

constexpr float HULL_MARGIN = 1e-3f;                      // rounding of the cube's core against the hull (m)
constexpr float HULL_FEAT_EPS = 1e-6f;                    // a witness lies on a plane within this (m)
constexpr float HULL_SIN_PARALLEL = 0.0871557427f;        // sin 5 deg
constexpr float HULL_SIN_ON_FACE = 0.0348994967f;         // sin 2 deg
constexpr float HULL_COS_COPLANAR = 0.99996192306f;       // cos 0.5 deg: planes this close to parallel are one face
constexpr float HULL_CLIP_EPS = 1e-9f;                    // slack of the face clipping (m)
constexpr float HULL_MPR_TOL = 1e-7f, HULL_MPR_EPS = 1e-12f;

// the object's core in the hull's geom frame: a segment [p0, p1] or a box (centre c, axes = columns of R,
// half extents h)
struct HullCore {
  int kind;  // 0 segment, 1 box
  V3 p0, p1, c, h;
  M3 R;
};

__device__ __forceinline__ V3 hcore_support(const HullCore& B, V3 d) {
  if (B.kind == 0) return dot(B.p0, d) >= dot(B.p1, d) ? B.p0 : B.p1;
  V3 o = B.c;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const V3 col = v3(B.R.m[0][k], B.R.m[1][k], B.R.m[2][k]);
    const float hk = k == 0 ? B.h.x : (k == 1 ? B.h.y : B.h.z);
    o = o + col * (dot(col, d) >= 0.0f ? hk : -hk);
  }
  return o;
}

__device__ __forceinline__ V3 hunit(V3 a) {
  const float l = sqrtf(dot(a, a));
  return l > 0.0f ? a * prcp(l) : a;
}

// closest point of segment / triangle to the origin as barycentric weights (Ericson 5.1.2 / 5.1.5), as convex.hpp
__device__ __forceinline__ void hseg(V3 a, V3 b, float* lam) {
  const V3 ab = b - a;
  const float den = dot(ab, ab);
  float t = den > 0.0f ? -dot(a, ab) * prcp(den) : 0.0f;
  t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
  lam[0] = 1.0f - t;
  lam[1] = t;
}
__device__ __forceinline__ void htri(V3 a, V3 b, V3 c, float* lam) {
  const V3 ab = b - a, ac = c - a;
  lam[0] = lam[1] = lam[2] = 0.0f;
  const float d1 = -dot(ab, a), d2 = -dot(ac, a);
  if (d1 <= 0.0f && d2 <= 0.0f) { lam[0] = 1.0f; return; }
  const float e3 = -dot(ab, b), d4 = -dot(ac, b);
  if (e3 >= 0.0f && d4 <= e3) { lam[1] = 1.0f; return; }
  const float vc = d1 * d4 - e3 * d2;
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
    lam[1] = 1.0f - w; lam[2] = w; return;
  }
  const float den = va + vb + vc;
  if (!(den > 0.0f)) { hseg(a, b, lam); lam[2] = 0.0f; return; }
  const float iden = prcp(den);
  const float v = vb * iden, w = vc * iden;
  lam[0] = 1.0f - v - w; lam[1] = v; lam[2] = w;
}
// closest point of the simplex W[0..n-1] to the origin, compacted in place (W and the hull points P); true if
// the origin is inside a non-degenerate tetrahedron
__device__ __forceinline__ bool hsimplex(V3* W, V3* P, int& n, V3& v, float* lk) {
  float lam[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (n == 1) {
    lam[0] = 1.0f;
  } else if (n == 2) {
    hseg(W[0], W[1], lam);
  } else if (n == 3) {
    htri(W[0], W[1], W[2], lam);
  } else {
    constexpr int F[4][4] = {{0, 1, 2, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {1, 3, 2, 0}};
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
      htri(a, b, c, l3);
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

// team max / min over the T lanes with DPP row operations (quad xor 1 / 2, row_half_mirror, row_mirror) and
// v_permlane16_swap (xor 16), as team_sum in team_physics.hpp: every lane ends with the result, in a few cycles
// per step instead of an LDS round trip per __shfl_xor
template <int T>
__device__ __forceinline__ float team_max_dpp(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
  if (T >= 8) v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
  if (T >= 16) v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));
  if (T >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(v, __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]));
  }
  if (T >= 64) v = fmaxf(v, __shfl_xor(v, 32));
  return v;
}
template <int T>
__device__ __forceinline__ float team_min_dpp(float v) { return -team_max_dpp<T>(-v); }
template <int T>
__device__ __forceinline__ int team_min_dpp_i(int v) {
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));
  if (T >= 8) v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));
  if (T >= 16) v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));
  if (T >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    v = min(v, (int)((threadIdx.x & 16) ? r[0] : r[1]));
  }
  if (T >= 64) v = min(v, __shfl_xor(v, 32));
  return v;
}

struct HullQ {
  const float (*hv)[3];
  const float (*pl)[4];
  int nv, np, tl, tb;
#ifdef MG_PHASE_TIMING
  mutable unsigned nsup = 0;  // profiling build: support evaluations
  mutable unsigned tsup = 0, tsimp = 0;  // profiling build: GJK's cycles in the supports and in the simplex solver
#endif
};

// the hull's support vertex in direction d (team argmax, ties to the lowest index)
template <int T>
__device__ __forceinline__ V3 hull_support(const HullQ& H, V3 d) {
  float best = -3.0e38f;
  int bi = 0x7fffffff;
  // the lane's vertices in ascending order (a strict compare keeps the first maximum), their LDS reads issued together
#pragma unroll MG_HULL_SUP_UNROLL
  for (int k = 0; k < (MG_MAX_HULL_VERTS + T - 1) / T; k++) {
    const int v = H.tl + k * T;
    if (v < H.nv) {
      const float s = H.hv[v][0] * d.x + H.hv[v][1] * d.y + H.hv[v][2] * d.z;
      if (s > best) { best = s; bi = v; }
    }
  }
  // the largest value, then the lowest vertex index holding it (a serial loop's first maximum)
  const float m = team_max_dpp<T>(best);
  bi = team_min_dpp_i<T>(best == m ? bi : 0x7fffffff);
#ifdef MG_PHASE_TIMING
  H.nsup++;
#endif
  return ld3(H.hv[bi]);
}

// 2 = farther than cut, 1 = separated (pa, pb, dist), 0 = overlapping
template <int T>
__device__ __forceinline__ int hull_gjk(const HullQ& H, V3 v0, const HullCore& B, float cut, V3& pa, V3& pb,
                                        float& dist) {
  V3 W[4], P[4];
  V3 v = v0;
  if (dot(v, v) < 1e-20f) v = v3(0, 0, 1);
  int n = 0;
  float vv = dot(v, v);
  float lam[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int it = 0; it < 64; it++) {
#ifdef MG_PHASE_TIMING
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
#endif
    const V3 a = hull_support<T>(H, -v), w = a - hcore_support(B, v);
#ifdef MG_PHASE_TIMING
    H.tsup += (unsigned)(__builtin_amdgcn_s_memtime() - ts0);
#endif
    const float vw = dot(v, w);
    if (vw > 0.0f && vw * vw > vv * cut * cut) {
      dist = vw / sqrtf(vv);
      return 2;
    }
    if (n > 0 && vv - vw <= 1e-6f * vv + 1e-20f) break;
    bool dup = false;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const V3 dd = W[i] - w;
      if (i < n && dot(dd, dd) <= 1e-20f) dup = true;
    }
    if (dup) break;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (i == n) { W[i] = w; P[i] = a; }
    n++;
#ifdef MG_PHASE_TIMING
    const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
    const bool inside = hsimplex(W, P, n, v, lam);
    H.tsimp += (unsigned)(__builtin_amdgcn_s_memtime() - ts1);
    if (inside) return 0;
#else
    if (hsimplex(W, P, n, v, lam)) return 0;
#endif
    const float vn = dot(v, v);
    if (vn <= 1e-20f) return 0;
    const bool stall = it > 0 && vn >= vv * (1.0f - 1e-7f);
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

// MPR on hull - core from the interior point v0: x = the boundary point (moving the hull by -x separates),
// pa = the hull-side witness; false if the portal search degenerates
template <int T>
__device__ __forceinline__ bool hull_mpr(const HullQ& H, V3 v0, const HullCore& B, V3& x, V3& pa) {
  if (dot(v0, v0) < 1e-20f) v0 = v3(1e-6f, 0, 0);
  V3 dir = hunit(-v0);
  auto sup = [&](V3 d, V3& a) {
    a = hull_support<T>(H, d);
    return a - hcore_support(B, -d);
  };
  V3 a1, a2, a3, a4;
  V3 v1 = sup(dir, a1);
  if (dot(v1, dir) <= 0.0f) return false;
  dir = cross(v0, v1);
  if (dot(dir, dir) <= 1e-24f) {
    x = v1;
    pa = a1;
    return true;
  }
  dir = hunit(dir);
  V3 v2 = sup(dir, a2);
  if (dot(v2, dir) <= 0.0f) return false;
  dir = hunit(cross(v1 - v0, v2 - v0));
  if (dot(dir, v0) > 0.0f) {
    V3 t = v1; v1 = v2; v2 = t;
    t = a1; a1 = a2; a2 = t;
    dir = -dir;
  }
  V3 v3p;
  int it;
  for (it = 0; it < 64; it++) {  // a portal the origin ray passes through
    v3p = sup(dir, a3);
    if (dot(v3p, dir) <= 0.0f) return false;
    if (dot(cross(v1, v3p), v0) < -HULL_MPR_EPS) {
      v2 = v3p; a2 = a3;
    } else if (dot(cross(v3p, v2), v0) < -HULL_MPR_EPS) {
      v1 = v3p; a1 = a3;
    } else {
      break;
    }
    dir = hunit(cross(v1 - v0, v2 - v0));
  }
  if (it == 64) return false;
  auto expand = [&](V3 v4) {
    const V3 c = cross(v4, v0);
    int k;
    if (dot(v1, c) > 0.0f) k = dot(v2, c) > 0.0f ? 1 : 3;
    else k = dot(v3p, c) > 0.0f ? 2 : 1;
    if (k == 1) { v1 = v4; a1 = a4; }
    else if (k == 2) { v2 = v4; a2 = a4; }
    else { v3p = v4; a3 = a4; }
  };
  auto reached = [&](V3 v4, V3 d) {
    const float d4 = dot(v4, d);
    const float mm = fminf(d4 - dot(v1, d), fminf(d4 - dot(v2, d), d4 - dot(v3p, d)));
    return mm <= HULL_MPR_TOL;
  };
  for (it = 0;; it++) {  // refine until the portal encloses the origin
    dir = hunit(cross(v2 - v1, v3p - v1));
    if (it >= 64) return false;
    if (dot(v1, dir) >= 0.0f) break;
    const V3 v4 = sup(dir, a4);
    if (dot(v4, dir) < 0.0f || reached(v4, dir)) return false;
    expand(v4);
  }
  for (it = 0;; it++) {  // push the portal onto the boundary
    dir = hunit(cross(v2 - v1, v3p - v1));
    const V3 v4 = sup(dir, a4);
    if (reached(v4, dir) || it >= 64) break;
    expand(v4);
  }
  float lam[3];
  htri(v1, v2, v3p, lam);
  x = v1 * lam[0] + v2 * lam[1] + v3p * lam[2];
  pa = a1 * lam[0] + a2 * lam[1] + a3 * lam[2];
  return true;
}

// the segment p0 + t u (radius rB) over face f: the clipped part's inner ends as contacts (out[7 * i])
template <int T>
__device__ __forceinline__ int hull_face_clip(const HullQ& H, int f, V3 p0, V3 u, float rB, float off, float* out) {
  const V3 nf = ld3(H.pl[f]);
  const float df = H.pl[f][3];
  const float s0 = dot(nf, p0) - df, su = dot(nf, u);
  const V3 q0 = p0 - nf * s0, qu = u - nf * su;
  float lo = 0.0f, hi = 1.0f;
  bool empty = false;
  for (int k = 0; k * T < H.np; k++) {
    const int i = k * T + H.tl;
    if (i >= H.np || i == f) continue;
    const float4 q = *reinterpret_cast<const float4*>(H.pl[i]);
    const float a = q.x * q0.x + q.y * q0.y + q.z * q0.z - q.w - HULL_CLIP_EPS;
    const float b = q.x * qu.x + q.y * qu.y + q.z * qu.z;
    if (b > 0.0f) hi = fminf(hi, -a / b);  // a + t b <= 0
    else if (b < 0.0f) lo = fmaxf(lo, -a / b);
    else if (a > 0.0f) empty = true;
  }
  lo = team_max_dpp<T>(lo);
  hi = team_min_dpp<T>(hi);
  const bool none = ((__ballot(empty) >> H.tb) & (T >= 64 ? ~0ull : ((1ull << T) - 1ull))) != 0ull;
  if (none || !(lo <= hi)) return 0;
  int n = 0;
#pragma unroll
  for (int e = 0; e < 2; e++) {
    const float t = e == 0 ? lo : hi;
    if (!(t > 1e-6f && t < 1.0f - 1e-6f) || (e == 1 && hi - lo < 1e-9f)) continue;
    const float g = s0 + t * su - rB;
    if (!(g < off)) continue;
    const V3 pt = p0 + u * t - nf * (rB + 0.5f * g);
    float* o = out + 7 * n;
    o[0] = pt.x; o[1] = pt.y; o[2] = pt.z;
    o[3] = -nf.x; o[4] = -nf.y; o[5] = -nf.z;
    o[6] = g;
    n++;
  }
  return n;
}

// The exact candidates in the hull's geom frame: core B (+ radius rB); up to 2 contacts (point, normal from the
// object to the hull, gap) in out[7 * i], their count returned.  hv: the hull's vertices (the LDS model tile),
// ctr their centroid, pl its planes.  Every lane of the team calls it with the same
// arguments and gets the same result.
template <int T>
__device__ __forceinline__ int hull_core_contacts(const float (*hv)[3], int nv, V3 ctr, const float (*pl)[4], int np,
                                                  int tl, int tb, const HullCore& B, float rB, float off, float* out,
                                                  unsigned* cyc = nullptr) {
  const HullQ H{hv, pl, nv, np, tl, tb};
#ifdef MG_PHASE_TIMING
  // profiling build: shader cycles of GJK, MPR and the feature / clipping rest into cyc[0..2], on every return path
  struct Report {
    unsigned* o;
    unsigned long long t0, t1, t2;
    int stage;
    const HullQ& h;
    unsigned s1;
    __device__ ~Report() {
      if (!o) return;
      const unsigned long long t3 = __builtin_amdgcn_s_memtime();
      o[4] += stage == 0 ? h.nsup : s1;        // GJK supports
      o[5] += stage == 2 ? h.nsup - s1 : 0u;   // MPR supports
      o[6] += h.tsup;                           // GJK: cycles in the supports
      o[7] += h.tsimp;                          // GJK: cycles in the simplex solver
      if (stage == 0) { o[0] += (unsigned)(t3 - t0); return; }
      o[0] += (unsigned)(t1 - t0);
      if (stage == 2) { o[1] += (unsigned)(t2 - t1); o[2] += (unsigned)(t3 - t2); }
      else o[2] += (unsigned)(t3 - t1);
    }
  } rep{cyc, __builtin_amdgcn_s_memtime(), 0, 0, 0, H, 0u};
#define MG_HULL_T(k, st) { rep.t##k = __builtin_amdgcn_s_memtime(); rep.stage = st; if (st == 1) rep.s1 = H.nsup; }
#else
  (void)cyc;
#define MG_HULL_T(k, st)
#endif
  const V3 cb = B.kind == 0 ? (B.p0 + B.p1) * 0.5f : B.c;
  const V3 v0 = ctr - cb;
  V3 pa, pb, x, nrm, pt;
  float dist, d;
  const int gk = hull_gjk<T>(H, v0, B, rB + off, pa, pb, dist);
  MG_HULL_T(1, 1)
  if (gk == 2) return 0;
  if (gk == 1) {
    if (!(dist > 1e-9f)) return 0;
    nrm = (pa - pb) * (1.0f / dist);
    pt = (pa + pb + nrm * rB) * 0.5f;
    d = dist - rB;
  } else {
    const bool ok = hull_mpr<T>(H, v0, B, x, pa);
    MG_HULL_T(2, 2)
    if (!ok) return 0;
    const float l = sqrtf(dot(x, x));
    if (!(l > 1e-9f)) return 0;
    nrm = x * (-1.0f / l);
    pb = pa - x;
    pt = pa - x * 0.5f + nrm * (0.5f * rB);
    d = -l - rB;
  }
  if (!(isfinite(pt.x) && isfinite(pt.y) && isfinite(pt.z) && isfinite(nrm.x) && isfinite(nrm.y) &&
        isfinite(nrm.z) && isfinite(d)))
    return 0;
  // no contact can be made at or beyond the offset: a face-clip gap is at least the distance, and the cube's
  // sharp edge is at most (sqrt2 - 1) of its rounding nearer than the rounded core
  if (!(d - (B.kind == 1 ? 0.41422f * rB : 0.0f) < off)) return 0;
  // the hull's features at pa: the planes through it (the first two in index order), one ballot per T planes; a plane
  // within 0.5 deg of one already kept is the same face (qhull's triangulation of the curved forearm mesh: a
  // witness on such a seam lies on two planes without being on an edge; oracle hull_core_contacts)
  int kA = 0, fa0 = 0, fa1 = 0;
  float fd0 = 0.0f, fd1 = 0.0f;
  const unsigned long long tm = T >= 64 ? ~0ull : ((1ull << T) - 1ull);
  for (int k = 0; k * T < np; k++) {  // one ballot per T planes, in plane order
    const int f = k * T + tl;
    bool on = false;
    if (f < np) {
      const float4 q = *reinterpret_cast<const float4*>(pl[f]);
      on = fabsf(q.x * pa.x + q.y * pa.y + q.z * pa.z - q.w) < HULL_FEAT_EPS;
    }
    unsigned long long bits = (__ballot(on) >> tb) & tm;
    while (bits) {
      const int i = k * T + __builtin_ctzll(bits);
      bits &= bits - 1;
      const V3 ni = ld3(pl[i]);
      const float di = fabsf(dot(ni, pa) - pl[i][3]);
      if (kA >= 1 && dot(ni, ld3(pl[fa0])) > HULL_COS_COPLANAR) {  // the same face: keep the plane pa is nearer to
        if (di < fd0) { fa0 = i; fd0 = di; }
        continue;
      }
      if (kA >= 2 && dot(ni, ld3(pl[fa1])) > HULL_COS_COPLANAR) {
        if (di < fd1) { fa1 = i; fd1 = di; }
        continue;
      }
      if (kA == 0) { fa0 = i; fd0 = di; }
      else if (kA == 1) { fa1 = i; fd1 = di; }
      kA++;
    }
  }
  if (kA == 0 || kA >= 3) return 0;
  // the core's feature at pb: the edge direction ub
  V3 ub;
  const V3 u = B.p1 - B.p0;
  if (B.kind == 0) {
    const float uu = dot(u, u), lu = sqrtf(uu);
    const float t = uu > 0.0f ? dot(pb - B.p0, u) / uu : 0.0f;
    if (!(t * lu > HULL_FEAT_EPS && (1.0f - t) * lu > HULL_FEAT_EPS)) return 0;
    ub = u;
  } else {
    const V3 dl = mulT(B.R, pb - B.c);
    int kB = 0, freeax = 0;
    if (fabsf(dl.x) > B.h.x - HULL_FEAT_EPS) kB++; else freeax = 0;
    if (fabsf(dl.y) > B.h.y - HULL_FEAT_EPS) kB++; else freeax = 1;
    if (fabsf(dl.z) > B.h.z - HULL_FEAT_EPS) kB++; else freeax = 2;
    if (kB != 2) return 0;
    ub = v3(B.R.m[0][freeax], B.R.m[1][freeax], B.R.m[2][freeax]);
  }
  const float lub = sqrtf(dot(ub, ub));
  // the pen's interior parallel to a face of the hull at the witness: the face case
  int face = -1;
  float falign = -2.0f;
  for (int i = 0; i < kA; i++) {
    const int fi = i == 0 ? fa0 : fa1;
    const V3 nn = ld3(pl[fi]);
    const float al = -dot(nn, nrm);
    if (fabsf(dot(nn, ub)) < HULL_SIN_ON_FACE * lub && al > falign) { face = fi; falign = al; }
  }
  if (face >= 0 || kA == 1) {
    if (B.kind != 0) return 0;
    // the face that clips: among the planes within the coplanar angle of the witness's face, the one highest at
    // the segment's midpoint (the facet under it; ties to the lowest index).  A segment parallel to near-coplanar
    // facets has its witness anywhere along them; the midpoint does not move with it (oracle hull_core_contacts_at)
    const int f0 = face >= 0 ? face : fa0;
    const V3 n0 = ld3(pl[f0]), mid = B.p0 + u * 0.5f;
    float bv = -1e30f;
    int fc = f0;
    for (int k = 0; k * T < np; k++) {
      const int i = k * T + tl;
      if (i < np) {
        const float4 q = *reinterpret_cast<const float4*>(pl[i]);
        if (q.x * n0.x + q.y * n0.y + q.z * n0.z > HULL_COS_COPLANAR) {
          const float v = q.x * mid.x + q.y * mid.y + q.z * mid.z - q.w;
          if (v > bv) { bv = v; fc = i; }
        }
      }
    }
    // team argmax of (bv, -fc): the highest plane, the lowest index among equal ones
    const float tb_v = team_max_dpp<T>(bv);
    fc = team_min_dpp_i<T>(bv == tb_v ? fc : 0x7fffffff);
    return hull_face_clip<T>(H, fc, B.p0, u, rB, off, out);
  }
  // edge against edge
  const V3 ua = cross(ld3(pl[fa0]), ld3(pl[fa1])), cx3 = cross(ua, ub);
  if (!(dot(cx3, cx3) > HULL_SIN_PARALLEL * HULL_SIN_PARALLEL * dot(ua, ua) * dot(ub, ub))) return 0;
  if (B.kind == 1) {  // the hull edge lying on a face of the box adjacent to its witness edge
    const V3 dl = mulT(B.R, pb - B.c);
    const float lua = sqrtf(dot(ua, ua));
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const V3 col = v3(B.R.m[0][k], B.R.m[1][k], B.R.m[2][k]);
      const float lk = k == 0 ? dl.x : (k == 1 ? dl.y : dl.z), hk = k == 0 ? B.h.x : (k == 1 ? B.h.y : B.h.z);
      if (fabsf(dot(col, ub)) < 0.5f && fabsf(dot(col, ua)) < HULL_SIN_ON_FACE * lua && fabsf(lk) > hk - HULL_FEAT_EPS)
        return 0;
    }
  }
  if (B.kind == 1) {
    // the cube's sharp edge: the core edge moved out by the margin along its two faces' normals; the contact on
    // the common perpendicular of the hull edge's line (pa, ua) and that edge's line (q, ub)
    const V3 dl = mulT(B.R, pb - B.c);
    V3 q = pb;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float lk = k == 0 ? dl.x : (k == 1 ? dl.y : dl.z), hk = k == 0 ? B.h.x : (k == 1 ? B.h.y : B.h.z);
      if (fabsf(lk) > hk - HULL_FEAT_EPS) q = q + v3(B.R.m[0][k], B.R.m[1][k], B.R.m[2][k]) * (lk < 0.0f ? -rB : rB);
    }
    V3 np_ = hunit(cross(ua, ub));
    if (dot(np_, nrm) < 0.0f) np_ = -np_;
    const V3 w0 = pa - q;
    const float a_ = dot(ua, ua), b_ = dot(ua, ub), c_ = dot(ub, ub), d_ = dot(ua, w0), e_ = dot(ub, w0);
    const float den = a_ * c_ - b_ * b_;
    const float sa = (b_ * e_ - c_ * d_) / den, tb = (a_ * e_ - b_ * d_) / den;
    pt = ((pa + ua * sa) + (q + ub * tb)) * 0.5f;
    nrm = np_;
    d = dot(w0, np_);
  }
  if (!(d < off)) return 0;
  out[0] = pt.x; out[1] = pt.y; out[2] = pt.z;
  out[3] = nrm.x; out[4] = nrm.y; out[5] = nrm.z;
  out[6] = d;
  return 1;
}
#undef MG_HULL_T

}  // namespace mg

// device_math.hpp — small fp32 vector / quaternion / spatial-algebra helpers
// for the gfx950 kernels.  Spatial vectors are world-aligned and expressed at
// one point per actor (the root origin at the start of a substep); motion
// vectors are [angular; linear], force vectors [moment; force] (DESIGN.md
// §Physics).  Everything is header-only so each kernel is one code object.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mg {

struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ V3 ld3(const float* p) { return v3(p[0], p[1], p[2]); }

struct M3 {
  float m[3][3];
};
__device__ __forceinline__ V3 mul(const M3& A, V3 v) {
  return v3(A.m[0][0] * v.x + A.m[0][1] * v.y + A.m[0][2] * v.z, A.m[1][0] * v.x + A.m[1][1] * v.y + A.m[1][2] * v.z,
            A.m[2][0] * v.x + A.m[2][1] * v.y + A.m[2][2] * v.z);
}
__device__ __forceinline__ V3 mulT(const M3& A, V3 v) {
  return v3(A.m[0][0] * v.x + A.m[1][0] * v.y + A.m[2][0] * v.z, A.m[0][1] * v.x + A.m[1][1] * v.y + A.m[2][1] * v.z,
            A.m[0][2] * v.x + A.m[1][2] * v.y + A.m[2][2] * v.z);
}
__device__ __forceinline__ M3 mul(const M3& A, const M3& B) {
  M3 C;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) C.m[i][j] = A.m[i][0] * B.m[0][j] + A.m[i][1] * B.m[1][j] + A.m[i][2] * B.m[2][j];
  return C;
}
__host__ __device__ __forceinline__ M3 quat_to_mat(float x, float y, float z, float w) {
  M3 R;
  R.m[0][0] = 1 - 2 * (y * y + z * z); R.m[0][1] = 2 * (x * y - z * w); R.m[0][2] = 2 * (x * z + y * w);
  R.m[1][0] = 2 * (x * y + z * w); R.m[1][1] = 1 - 2 * (x * x + z * z); R.m[1][2] = 2 * (y * z - x * w);
  R.m[2][0] = 2 * (x * z - y * w); R.m[2][1] = 2 * (y * z + x * w); R.m[2][2] = 1 - 2 * (x * x + y * y);
  return R;
}
// rotation by angle ang about unit axis a, from the angle's sine and cosine
__device__ __forceinline__ M3 axis_angle_sc(V3 a, float s, float c) {
  float t = 1 - c;
  M3 R;
  R.m[0][0] = t * a.x * a.x + c; R.m[0][1] = t * a.x * a.y - s * a.z; R.m[0][2] = t * a.x * a.z + s * a.y;
  R.m[1][0] = t * a.x * a.y + s * a.z; R.m[1][1] = t * a.y * a.y + c; R.m[1][2] = t * a.y * a.z - s * a.x;
  R.m[2][0] = t * a.x * a.z - s * a.y; R.m[2][1] = t * a.y * a.z + s * a.x; R.m[2][2] = t * a.z * a.z + c;
  return R;
}
__device__ __forceinline__ M3 axis_angle(V3 a, float ang) { return axis_angle_sc(a, sinf(ang), cosf(ang)); }
__device__ __forceinline__ void mat_to_quat(const M3& R, float* q) {
  float tr = R.m[0][0] + R.m[1][1] + R.m[2][2];
  if (tr > 0) {
    float s = sqrtf(tr + 1.0f) * 2;
    q[3] = 0.25f * s; q[0] = (R.m[2][1] - R.m[1][2]) / s; q[1] = (R.m[0][2] - R.m[2][0]) / s;
    q[2] = (R.m[1][0] - R.m[0][1]) / s;
  } else if (R.m[0][0] > R.m[1][1] && R.m[0][0] > R.m[2][2]) {
    float s = sqrtf(1.0f + R.m[0][0] - R.m[1][1] - R.m[2][2]) * 2;
    q[3] = (R.m[2][1] - R.m[1][2]) / s; q[0] = 0.25f * s; q[1] = (R.m[0][1] + R.m[1][0]) / s;
    q[2] = (R.m[0][2] + R.m[2][0]) / s;
  } else if (R.m[1][1] > R.m[2][2]) {
    float s = sqrtf(1.0f + R.m[1][1] - R.m[0][0] - R.m[2][2]) * 2;
    q[3] = (R.m[0][2] - R.m[2][0]) / s; q[0] = (R.m[0][1] + R.m[1][0]) / s; q[1] = 0.25f * s;
    q[2] = (R.m[1][2] + R.m[2][1]) / s;
  } else {
    float s = sqrtf(1.0f + R.m[2][2] - R.m[0][0] - R.m[1][1]) * 2;
    q[3] = (R.m[1][0] - R.m[0][1]) / s; q[0] = (R.m[0][2] + R.m[2][0]) / s; q[1] = (R.m[1][2] + R.m[2][1]) / s;
    q[2] = 0.25f * s;
  }
}

// ---------------------------------------------------------------- spatial
struct SV {  // spatial vector: a = angular/moment, l = linear/force
  V3 a, l;
};
__device__ __forceinline__ SV sv(V3 a, V3 l) { return SV{a, l}; }
__device__ __forceinline__ SV operator+(const SV& x, const SV& y) { return sv(x.a + y.a, x.l + y.l); }
__device__ __forceinline__ SV operator-(const SV& x, const SV& y) { return sv(x.a - y.a, x.l - y.l); }
__device__ __forceinline__ SV operator*(const SV& x, float s) { return sv(x.a * s, x.l * s); }
__device__ __forceinline__ float dot(const SV& x, const SV& y) { return dot(x.a, y.a) + dot(x.l, y.l); }
__device__ __forceinline__ SV crm(const SV& v, const SV& m) {  // v x m (motion)
  return sv(cross(v.a, m.a), cross(v.a, m.l) + cross(v.l, m.a));
}
__device__ __forceinline__ SV crf(const SV& v, const SV& f) {  // v x* f (force)
  return sv(cross(v.a, f.a) + cross(v.l, f.l), cross(v.a, f.l));
}
__device__ __forceinline__ SV szero() { return sv(v3(0, 0, 0), v3(0, 0, 0)); }

// Symmetric 6x6 spatial (articulated) inertia [[A, B], [B^T, C]], A and C symmetric.
struct Sym6 {
  float a[6];  // A: 00 01 02 11 12 22
  float b[9];  // B row-major
  float c[6];  // C: 00 01 02 11 12 22
};
__device__ __forceinline__ V3 symmul(const float* s, V3 v) {
  return v3(s[0] * v.x + s[1] * v.y + s[2] * v.z, s[1] * v.x + s[3] * v.y + s[4] * v.z,
            s[2] * v.x + s[4] * v.y + s[5] * v.z);
}
__device__ __forceinline__ SV mul(const Sym6& I, const SV& v) {
  V3 Bu = v3(I.b[0] * v.l.x + I.b[1] * v.l.y + I.b[2] * v.l.z, I.b[3] * v.l.x + I.b[4] * v.l.y + I.b[5] * v.l.z,
             I.b[6] * v.l.x + I.b[7] * v.l.y + I.b[8] * v.l.z);
  V3 Btw = v3(I.b[0] * v.a.x + I.b[3] * v.a.y + I.b[6] * v.a.z, I.b[1] * v.a.x + I.b[4] * v.a.y + I.b[7] * v.a.z,
              I.b[2] * v.a.x + I.b[5] * v.a.y + I.b[8] * v.a.z);
  return sv(symmul(I.a, v.a) + Bu, Btw + symmul(I.c, v.l));
}
__device__ __forceinline__ void add_to(Sym6& D, const Sym6& S) {
#pragma unroll
  for (int k = 0; k < 6; k++) { D.a[k] += S.a[k]; D.c[k] += S.c[k]; }
#pragma unroll
  for (int k = 0; k < 9; k++) D.b[k] += S.b[k];
}
// D -= U U^T * s
__device__ __forceinline__ void rank1_sub(Sym6& D, const SV& U, float s) {
  float u[6] = {U.a.x, U.a.y, U.a.z, U.l.x, U.l.y, U.l.z};
  D.a[0] -= u[0] * u[0] * s; D.a[1] -= u[0] * u[1] * s; D.a[2] -= u[0] * u[2] * s;
  D.a[3] -= u[1] * u[1] * s; D.a[4] -= u[1] * u[2] * s; D.a[5] -= u[2] * u[2] * s;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) D.b[3 * i + j] -= u[i] * u[3 + j] * s;
  D.c[0] -= u[3] * u[3] * s; D.c[1] -= u[3] * u[4] * s; D.c[2] -= u[3] * u[5] * s;
  D.c[3] -= u[4] * u[4] * s; D.c[4] -= u[4] * u[5] * s; D.c[5] -= u[5] * u[5] * s;
}
// spatial inertia at point o of a body: mass m, COM offset c (from o), rotational inertia Ic (world, sym6)
__device__ __forceinline__ Sym6 body_inertia(float m, V3 c, const float* Ic) {
  Sym6 I;
  float cc = dot(c, c);
  I.a[0] = Ic[0] + m * (cc - c.x * c.x); I.a[1] = Ic[1] - m * c.x * c.y; I.a[2] = Ic[2] - m * c.x * c.z;
  I.a[3] = Ic[3] + m * (cc - c.y * c.y); I.a[4] = Ic[4] - m * c.y * c.z; I.a[5] = Ic[5] + m * (cc - c.z * c.z);
  // B = m [c]x
  I.b[0] = 0; I.b[1] = -m * c.z; I.b[2] = m * c.y;
  I.b[3] = m * c.z; I.b[4] = 0; I.b[5] = -m * c.x;
  I.b[6] = -m * c.y; I.b[7] = m * c.x; I.b[8] = 0;
  I.c[0] = m; I.c[1] = 0; I.c[2] = 0; I.c[3] = m; I.c[4] = 0; I.c[5] = m;
  return I;
}
// reciprocal / square root / inverse square root of the physics: the 1-ulp hardware instructions instead
// of the correctly rounded sequences (~10 instructions each); the task layer keeps IEEE division
// (MG_EXACT_RCP: the correctly rounded forms, a parity A/B only)
#ifndef MG_EXACT_RCP
#define MG_EXACT_RCP 0
#endif
#if MG_EXACT_RCP
__device__ __forceinline__ float prcp(float x) { return 1.0f / x; }
__device__ __forceinline__ float psqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ float prsq(float x) { return 1.0f / sqrtf(x); }
#else
__device__ __forceinline__ float prcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float psqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float prsq(float x) { return __builtin_amdgcn_rsqf(x); }
#endif
// sine and cosine of the physics' angles (joint angles in FK, the root's / object's half rotation per substep; five
// pairs per lane and step).  HW: the hardware v_sin_f32 / v_cos_f32 on the argument in revolutions reduced to
// [-1/2, 1/2] (a few instructions instead of the library's ~60; absolute error tools/trig_probe.hip), used by the
// 16-lane instances (Ant, MA-Ant: +2 % same box); otherwise poly_sincos (round 6; before, the library's sinf / cosf:
// the Humanoid's fast-spin parity case rejects the hardware pair).  The task layer keeps the
// library's everywhere.
//
// poly_sincos: a polynomial pair (one Cody-Waite reduction by pi/2, Cephes' minimax polynomials on [-pi/4, pi/4]),
// the physics' pair of the instances that are not 16-lane (MG_POLY_TRIG below).  Round 5's first form took the
// quadrant as (int)rint(x 2/pi) and its first GPU run faulted; its source was not kept.  This
// form never converts a float to an integer: the quadrant is k - 4 floor(k / 4) in floating point and the result is
// picked by float compares, so a NaN / infinite / huge x can only give a NaN / wrong value, never an address or a
// branch target.  MG_POLY_TRIG=2 rebuilds the integer-quadrant form for the disassembly check
// (tests/test_trig_kat.py: host KAT of both forms over NaN, +-Inf, +-1e30, denormals and Cartpole-range angles).
__host__ __device__ __forceinline__ void poly_sincos(float x, float* s, float* c, bool int_quadrant = false) {
  const float k = rintf(x * 0.636619772367581343f);  // nearest multiple of pi / 2
  const float r = ((x - k * 1.5703125f) - k * 4.837512969970703125e-4f) - k * 7.54978995489188216e-8f;
  const float z = r * r;
  const float sp = r + r * z * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f));
  const float cp = 1.0f - 0.5f * z + z * z * (4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f));
  bool swap, ns, nc;
  if (int_quadrant) {  // round 5's form (A/B disassembly only)
    const int q = (int)k & 3;
    swap = (q & 1) != 0;
    ns = (q & 2) != 0;
    nc = q == 1 || q == 2;
  } else {
    const float kq = k - 4.0f * floorf(k * 0.25f);  // 0, 1, 2, 3 for a finite k
    swap = kq == 1.0f || kq == 3.0f;
    ns = kq >= 2.0f;
    nc = kq == 1.0f || kq == 2.0f;
  }
  const float sv = swap ? cp : sp, cv = swap ? sp : cp;
  *s = ns ? -sv : sv;
  *c = nc ? -cv : cv;
}
// the physics' pair outside the 16-lane instances (Humanoid, the hand, Cartpole): 1 = poly_sincos (round 6: GPU suite
// green, 168 passed, the Humanoid fast-spin case included; same box, two passes, Humanoid 32,768 +1.0 %, ShadowHand
// 4,096 +0.9 %, 16,384 +0.3 %, profiles/r06/ab_poly_trig.txt), 0 = the library's sinf / cosf, 2 = the integer-quadrant
// form (disassembly check only)
#ifndef MG_POLY_TRIG
#define MG_POLY_TRIG 1
#endif
template <bool HW>
__device__ __forceinline__ void psincos(float x, float* s, float* c) {
  if constexpr (HW) {
    float r = x * 0.159154943091895336f;
    r = r - __builtin_rintf(r);
    *s = __builtin_amdgcn_sinf(r);
    *c = __builtin_amdgcn_cosf(r);
  } else if constexpr (MG_POLY_TRIG != 0) {
    poly_sincos(x, s, c, MG_POLY_TRIG == 2);
  } else {
    *s = sinf(x);
    *c = cosf(x);
  }
}
// tanh of the joint friction law: (1 - e) / (1 + e), e = exp(-2|x|) by the hardware exp2 (~7 instructions instead of
// the library's ~50; a few ulp, against a friction torque the oracle checks to 1e-6 relative)
__device__ __forceinline__ float ptanh(float x) {
  const float e = __builtin_amdgcn_exp2f(-2.8853900817779268f * fabsf(x));  // exp(-2|x|) = 2^(-2 log2(e) |x|)
  return copysignf((1.0f - e) * prcp(1.0f + e), x);
}
// Cholesky of a Sym6 into a packed lower-triangular 6x6 (21 floats); returns false if not SPD
__device__ __forceinline__ bool chol6(const Sym6& I, float* L) {
  float M[6][6];
  const int ai[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      M[i][j] = I.a[ai[i][j]];
      M[3 + i][3 + j] = I.c[ai[i][j]];
      M[i][3 + j] = I.b[3 * i + j];
      M[3 + j][i] = I.b[3 * i + j];
    }
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    float s = M[j][j];
#pragma unroll
    for (int k = 0; k < j; k++) s -= M[j][k] * M[j][k];
    ok = ok && (s > 0.0f);
    float d = psqrt(fmaxf(s, 1e-30f));
    M[j][j] = d;
    float inv = prcp(d);
#pragma unroll
    for (int i = j + 1; i < 6; i++) {
      float t = M[i][j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= M[i][k] * M[j][k];
      M[i][j] = t * inv;
    }
  }
  // packed lower triangle, the diagonal stored as its reciprocal: chol6_solve multiplies by it instead of
  // recomputing a reciprocal per step on its dependent chain, and the compiler folds rcp(sqrt(x)) into one
  // v_rsq_f32 (1 ulp, like the pair it replaces; results move by that rounding only).  Same box, with the team
  // observation head and load()'s shuffle-free root: Ant +0.8 %, Humanoid +1.3 % (profiles/r05/ab_micro_*.txt)
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) L[k++] = i == j ? prcp(M[i][i]) : M[i][j];
  return ok;
}
__device__ __forceinline__ SV chol6_solve(const float* L, const SV& b) {
  float x[6] = {b.a.x, b.a.y, b.a.z, b.l.x, b.l.y, b.l.z};
  // forward: L y = b
#pragma unroll
  for (int i = 0; i < 6; i++) {
    float s = x[i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[i * (i + 1) / 2 + k] * x[k];
    x[i] = s * L[i * (i + 1) / 2 + i];
  }
  // backward: L^T x = y
#pragma unroll
  for (int i = 5; i >= 0; i--) {
    float s = x[i];
#pragma unroll
    for (int k = i + 1; k < 6; k++) s -= L[k * (k + 1) / 2 + i] * x[k];
    x[i] = s * L[i * (i + 1) / 2 + i];
  }
  return sv(v3(x[0], x[1], x[2]), v3(x[3], x[4], x[5]));
}

// ---------------------------------------------------------------- RNG (same recipe as the oracle)
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t env, uint64_t counter, uint32_t k) {
  uint64_t h = mix64(mix64(mix64(seed ^ (env * 0xD2B74407B1CE6E93ull)) ^ counter) ^ (uint64_t)k);
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

}  // namespace mg

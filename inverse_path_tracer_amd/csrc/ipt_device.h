// ipt_device.h -- device-side building blocks of the MI355X path tracer.
//
// Everything here follows the canonical arithmetic of DESIGN.md §3 (the same
// arithmetic the CPU oracle states), so kernel results are bit-identical to
// the oracle on equal seeds:
//   * fp32 dot products as fmaf chains (the contraction nvcc --fmad=true
//     applies to the reference's Eigen (x+y)+z reductions), IEEE division and
//     sqrt (hipcc's default correctly-rounded lowering), -ffp-contract=off so
//     no other contraction happens;
//   * the reference's double-precision pow(r,0.5) == sqrt, its sin/cos(phi)
//     as a double Taylor evaluation rounded once to float;
//   * cuRAND XORWOW seeded exactly like curand_init(seed + sample, 0, 0).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "scene_layout.h"

namespace ipt {
namespace dev {

// Address-space-qualified views (LDS = 3, global = 1) for data that lives in
// either place depending on the scene: separate typed accesses per branch
// compile to ds_* / global_* instructions; one pointer that may be either
// compiles to flat ones (vector-memory path and a vmcnt+lgkmcnt wait even
// for LDS data), and LLVM merges untyped per-branch accesses back into one.
typedef __attribute__((address_space(3))) float lds_f32;
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(1))) float gbl_f32;
typedef __attribute__((address_space(1))) double gbl_f64;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4f lds_v4;
typedef __attribute__((address_space(1))) v4f gbl_v4;

// ------------------------------------------------------------ constants
// scene_basics.h:13-14 compare a float against the double literals 1e-4 and
// 1e-2.  For a float x, (double)x < 1e-4  <=>  x < kMinDotUp, where kMinDotUp
// is the smallest float above 1e-4 (1e-4 itself is not a float); same for
// EPSILON.  tests/test_constants.py re-derives both.
constexpr float kMinDotUp = 0x1.a36e30p-14f;   // nextafterf(1e-4 rounded down, +inf)
constexpr float kEpsUp = 0x1.47ae16p-7f;       // smallest float > 1e-2
constexpr float kPRR = 0.9f;                   // scene.h:11
constexpr float kPiF = 3.14159265358979323846f;        // (float)M_PI
constexpr float kInvPiF = (float)(1.0 / 3.14159265358979323846);  // (float)(1/M_PI)
constexpr double kPi = 3.14159265358979323846;

// x / b for the constant divisors b = kInvPiF, kPRR, kPiF in three VALU
// operations (Markstein: q = x*y, r = fma(-q, b, x) exact, fma(r, y, q)),
// with y = RN(1/b).  Equal to the IEEE quotient for every float 2^-100 <= |x|
// < 2^100 -- checked exhaustively for these three b (tools/check_div_const.c,
// tests/test_identities.py); other x (zeros, tiny, huge, non-finite) take
// the IEEE division.  Not a generic division: only those three divisors.
#ifndef IPT_DIV_CONST
#define IPT_DIV_CONST 1
#endif
template <int B>  // 0: kInvPiF, 1: kPRR, 2: kPiF
__device__ __forceinline__ float div_const(float x) {
  constexpr float b = B == 0 ? kInvPiF : (B == 1 ? kPRR : kPiF);
  constexpr float y = (float)(1.0 / (double)b);
  const float ax = fabsf(x);
  if (IPT_DIV_CONST && ax >= 0x1p-100f && ax < 0x1p100f) {
    const float q = x * y;
    return fmaf(fmaf(-q, b, x), y, q);
  }
  return x / b;
}

// ------------------------------------------------------------ XORWOW
struct Rng {
  uint32_t d, v0, v1, v2, v3, v4;
};
__device__ __forceinline__ void rng_init(Rng &s, uint64_t seed) {
  uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
  uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
  uint32_t t0 = 1099087573u * s0;
  uint32_t t1 = 2591861531u * s1;
  s.d = 6615241u + t1 + t0;
  s.v0 = 123456789u + t0;
  s.v1 = 362436069u ^ t0;
  s.v2 = 521288629u + t1;
  s.v3 = 88675123u ^ t1;
  s.v4 = 5783321u + t0;
}
__device__ __forceinline__ float uniform(Rng &s) {
  uint32_t t = s.v0 ^ (s.v0 >> 2);
  s.v0 = s.v1;
  s.v1 = s.v2;
  s.v2 = s.v3;
  s.v3 = s.v4;
  s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
  s.d += 362437u;
  return (float)(s.v4 + s.d) * 2.3283064e-10f + 1.1641532e-10f;
}

// ------------------------------------------------------------ sin/cos(phi)
// sinf/cosf of the float angle phi in [0, 2pi] (path_trace.cu:92,96: `phi` is
// a float, so the reference's sin(phi)/cos(phi) are CUDA's float sinf/cosf,
// documented to 2 ulp) in float arithmetic -- rounds 1-6 evaluated them in
// double (27 FP64 operations per vertex; C2 render -3.6%, adjoint -2.8% with
// this form): three-part Cody-Waite reduction by
// pi/2 (the first step exact: k <= 4), Cephes' degree-7 sine and degree-8
// cosine on |r| <= pi/4.  Every operation is an explicit IEEE fmaf / mul /
// rint, so oracle/ipt_oracle.c::oro_sincos reproduces it bit for bit;
// exhaustively over the floats of [1e-10, 6.2832]: at most 1.49 / 1.56 ulp;
// 76% of uniformly drawn angles correctly rounded (tests/test_oracle.py).
__device__ __forceinline__ void sincos_f(float x, float &sf, float &cf) {
  const float k = rintf(x * 0x1.45f306p-1f);  // 2/pi
  float r = fmaf(-k, 0x1.921fb6p+0f, x);      // pi/2 = C1 + C2 + C3
  r = fmaf(-k, -0x1.777a5cp-25f, r);
  r = fmaf(-k, -0x1.ee59dap-50f, r);
  const float z = r * r;
  float p = fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f);
  p = fmaf(p, z, -1.6666654611e-1f);
  const float s = fmaf(p * z, r, r);
  float q = fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f);
  q = fmaf(q, z, 4.166664568298827e-2f);
  const float c = fmaf(q * z, z, fmaf(-0.5f, z, 1.0f));
  const int n = (int)k;
  // the quadrant by one swap and two sign flips (bitwise the selects of
  // s, c, -s, -c; 4 B less scratch in the 6-wave adjoint, 8 B in the
  // unbounded one, -0.5% on both, variants_sincos_xor_r06zf.log)
  const bool sw = (n & 1) != 0;
  const float a = sw ? c : s, b = sw ? s : c;
  sf = __uint_as_float(__float_as_uint(a) ^ ((uint32_t)(n & 2) << 30));
  cf = __uint_as_float(__float_as_uint(b) ^ ((uint32_t)((n + 1) & 2) << 30));
}

// ------------------------------------------------------------ f64 helpers
__device__ inline double log_d(double x) {
  if (!(x > 0.0)) return x == 0.0 ? -__builtin_inf() : __builtin_nan("");
  if (x == __builtin_inf()) return x;
  uint64_t b = (uint64_t)__double_as_longlong(x);
  int e = (int)((b >> 52) & 0x7ff);
  if (e == 0) {
    x = x * 18014398509481984.0;
    b = (uint64_t)__double_as_longlong(x);
    e = (int)((b >> 52) & 0x7ff) - 54;
  }
  e -= 1023;
  double m = __longlong_as_double((long long)((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull));
  if (m > 1.4142135623730951) {
    m *= 0.5;
    e += 1;
  }
  const double s = (m - 1.0) / (m + 1.0);
  const double z = s * s;
  double p = 1.0 / 23.0;
  p = fma(p, z, 1.0 / 21.0);
  p = fma(p, z, 1.0 / 19.0);
  p = fma(p, z, 1.0 / 17.0);
  p = fma(p, z, 1.0 / 15.0);
  p = fma(p, z, 1.0 / 13.0);
  p = fma(p, z, 1.0 / 11.0);
  p = fma(p, z, 1.0 / 9.0);
  p = fma(p, z, 1.0 / 7.0);
  p = fma(p, z, 1.0 / 5.0);
  p = fma(p, z, 1.0 / 3.0);
  const double lm = 2.0 * fma(p * z, s, s);
  const double de = (double)e;
  return fma(de, 0.6931471805599453, fma(de, 2.3190468138462996e-17, lm));
}
__device__ inline double exp_d(double x) {
  if (x != x) return x;
  if (x > 709.0) return __builtin_inf();
  if (x < -745.0) return 0.0;
  const double k = rint(x * 1.4426950408889634);
  double r = fma(-k, 0.6931471805599453, x);
  r = fma(-k, 2.3190468138462996e-17, r);
  double p = 1.0 / 355687428096000.0;
  p = fma(p, r, 1.0 / 20922789888000.0);
  p = fma(p, r, 1.0 / 1307674368000.0);
  p = fma(p, r, 1.0 / 87178291200.0);
  p = fma(p, r, 1.0 / 6227020800.0);
  p = fma(p, r, 1.0 / 479001600.0);
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  const int ki = (int)k;
  const int k1 = ki / 2, k2 = ki - k1;
  const double s1 = __longlong_as_double((long long)((uint64_t)(k1 + 1023) << 52));
  const double s2 = __longlong_as_double((long long)((uint64_t)(k2 + 1023) << 52));
  return (p * s1) * s2;
}
// Out of line: the megakernel's SPEC instances (materials with a Phong lobe)
// call it from the sampling and BSDF code.  Inlined, its ~35 polynomial
// constants were hoisted out of the trace loop into registers, and every
// SPEC instance spilled 164-292 B per lane inside the loop even on diffuse
// vertices; as a call, the constants live in the callee and the caller saves
// registers only around the (Phong-only) call.
__device__ __attribute__((noinline)) double pow_d(double x, double y) {
  if (y == 0.0) return 1.0;
  if (x == 0.0) return y > 0 ? 0.0 : __builtin_inf();
  return exp_d(y * log_d(x));
}
__device__ inline float pow_f(float x, float y) {  // C powf semantics
  if (y == 0.f) return 1.f;
  if (x == 0.f) return y > 0.f ? 0.f : __builtin_inff();
  if (x < 0.f) {
    if (floorf(y) != y) return __builtin_nanf("");
    const float r = (float)pow_d(-(double)x, (double)y);
    const double half = (double)y * 0.5;
    return (floor(half) != half) ? -r : r;
  }
  return (float)pow_d((double)x, (double)y);
}

// ------------------------------------------------------------ fp32 vectors
struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float dot3(V3 a, V3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ V3 cross3(V3 a, V3 b) {
  return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
// Eigen's normalize with IEEE sqrtf and divisions (the definition).
__device__ __forceinline__ V3 unit_ieee(V3 v) {
  const float n2 = dot3(v, v);
  if (n2 > 0.f) {
    const float s = sqrtf(n2);
    v = mk(v.x / s, v.y / s, v.z / s);
  }
  return v;
}
__device__ __forceinline__ V3 along(V3 p, V3 d, float t) {
  return mk(fmaf(d.x, t, p.x), fmaf(d.y, t, p.y), fmaf(d.z, t, p.z));
}

// ------------------------------------------------------------ division
// Correctly rounded a/b for the closest-hit test's operand range.  This is
// hipcc's IEEE f32 division lowering (v_rcp + Newton + the final residual
// fma) without v_div_scale / v_div_fixup: those only rescale operands whose
// quotient or reciprocal would leave the normal range and patch inf/NaN/0
// inputs.  In the hit test |b| = |n.d| lies in [1e-4, 1] and |a| <= scene
// extent whenever the quotient is used (smaller |b| rejects the triangle
// before t matters), so the scaling is the identity and the result equals
// `a / b` bit for bit -- except -0 / (b > 0), which gives +0 where IEEE
// gives -0 (harmless at both call sites: the hit test rejects t = +-0 by
// t < eps, the camera's numerator is positive).  Checked on the device by
// ipt_selftest_math (tests/test_gpu.py).
#ifndef IPT_FASTDIV
#define IPT_FASTDIV 1
#endif
__device__ __forceinline__ float div_inrange(float a, float b) {
#if IPT_FASTDIV
  const float nb = -b;
  const float r0 = __builtin_amdgcn_rcpf(b);
  const float e0 = fmaf(nb, r0, 1.0f);
  const float r1 = fmaf(e0, r0, r0);
  const float q0 = a * r1;
  const float e1 = fmaf(nb, q0, a);
  const float q1 = fmaf(e1, r1, q0);
  const float e2 = fmaf(nb, q1, a);
  return fmaf(e2, r1, q1);
#else
  return a / b;
#endif
}

// ---- in-range cores of the IEEE sqrt / division lowerings
// hipcc lowers sqrtf to v_sqrt_f32 plus a one-ulp correction, wrapped in a
// rescale for x < 2^-96 and a class test for +-0/+inf; sqrt (f64) to v_rsq_f64
// plus Goldschmidt/Newton steps, wrapped in a rescale for x < 2^-767 and the
// same class test.  Inside those ranges the wrappers are the identity, so the
// cores below (the same instructions, same operands) ARE the IEEE results.
__device__ __forceinline__ float sqrt_core(float x) {  // x in [2^-96, FLT_MAX]
  float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float rm = fmaf(-sm, s, x);
  const float rp = fmaf(-sp, s, x);
  s = (0.f >= rm) ? sm : s;
  s = (0.f < rp) ? sp : s;
  return s;
}
__device__ __forceinline__ double dsqrt_core(double x) {  // x in [2^-767, DBL_MAX]
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  g = fma(d, h, g);
  return g;
}
// v / s (s > 0) for three numerators sharing the divisor's reciprocal
// refinement (div_inrange with the r0/e0/r1 steps computed once).  The
// residuals are formed as -fma(s, q, -a): the same value as fma(-s, q, a) for
// every nonzero residual (round-to-nearest is symmetric under negation), but
// a -0 numerator then yields -0 as IEEE division does (fma(-s, -0, -0) would
// give +0).  The negation folds into the next fma's input modifier.
__device__ __forceinline__ V3 div3_core(V3 v, float s) {
  const float ns = -s;
  const float r0 = __builtin_amdgcn_rcpf(s);
  const float e0 = fmaf(ns, r0, 1.0f);
  const float r1 = fmaf(e0, r0, r0);
  auto one = [&](float a) {
    const float q0 = a * r1;
    const float e1 = -fmaf(s, q0, -a);
    const float q1 = fmaf(e1, r1, q0);
    const float e2 = -fmaf(s, q1, -a);
    return fmaf(e2, r1, q1);
  };
  return mk(one(v.x), one(v.y), one(v.z));
}
// unit_ieee(v) exactly.  Fast path when n2 in [2^-6, 2^60] (sqrt core valid;
// s in [2^-3, 2^30]) and every component is 0 or >= 2^-90 in magnitude (so
// each quotient is normal and no division would be rescaled): checked on the
// bit patterns, (|bits| << 1) - 1 >= (bits(2^-90) << 1) - 1, with 0 wrapping
// to the top.  Anything else takes the IEEE operations.
__device__ __forceinline__ V3 unit(V3 v) {
  const float n2 = dot3(v, v);
  const uint32_t kLo = (0x25u << 24) - 1u;  // (bits(2^-90) << 1) - 1 = 0x24ffffff
  const uint32_t m = min(min((__float_as_uint(v.x) << 1) - 1u, (__float_as_uint(v.y) << 1) - 1u),
                         (__float_as_uint(v.z) << 1) - 1u);
  if (n2 >= 0x1p-6f && n2 <= 0x1p60f && m >= kLo) return div3_core(v, sqrt_core(n2));
  return unit_ieee(v);
}
// unit() for operands proven in range by construction (no test).
__device__ __forceinline__ V3 unit_in_range(V3 v) { return div3_core(v, sqrt_core(dot3(v, v))); }

// ------------------------------------------------------------ closest hit
// Object::getIntersection (scene_basics.h:426-459) over every triangle in
// object order (BVH::getIntersection with its single leaf, bvh.h:55-77):
// strict '<' keeps the first of equal-t hits.  The triangle loop is wave-
// uniform, so the 80-B records come in through scalar loads; the test is
// evaluated branch-free per lane and committed with a select.  Each skip
// condition is written exactly as the reference's (negated) so NaNs take the
// same branch.
// One triangle of the closest-hit loop: branch-free test, select on accept.
__device__ __forceinline__ void hit_test(const TriIsect &T, int i, V3 p, V3 d, float &bt, int &bi) {
  const float denom = fmaf(T.n[2], d.z, fmaf(T.n[1], d.y, T.n[0] * d.x));
  const float px = p.x - T.c[0], py = p.y - T.c[1], pz = p.z - T.c[2];
  const float num = fmaf(pz, T.n[2], fmaf(py, T.n[1], px * T.n[0]));
  const float t = div_inrange(num, -denom);
  const float qx = fmaf(d.x, t, p.x), qy = fmaf(d.y, t, p.y), qz = fmaf(d.z, t, p.z);
  const float s0 = fmaf(qz, T.e0[2], fmaf(qy, T.e0[1], fmaf(qx, T.e0[0], T.e0[3])));
  const float s1 = fmaf(qz, T.e1[2], fmaf(qy, T.e1[1], fmaf(qx, T.e1[0], T.e1[3])));
  const float s2 = fmaf(qz, T.e2[2], fmaf(qy, T.e2[1], fmaf(qx, T.e2[0], T.e2[3])));
  const bool take = !(fabsf(denom) < kMinDotUp) && !(t < kEpsUp) && !(t >= bt) && !(s0 > 0.f) &&
                    !(s1 > 0.f) && !(s2 > 0.f);
  bt = take ? t : bt;
  bi = take ? i : bi;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc2(float x) { return f2{x, x}; }
__device__ __forceinline__ f2 ld2(const TriPair &T, int k) { return f2{T.f[k][0], T.f[k][1]}; }

// hit_test on triangles i (half x) and i+1 (half y) with packed FP32: the same
// IEEE operations in the same order per half, then the two accept/select
// steps in index order (strict '<' still prefers the first of equal t).
struct PairOrigin {
  f2 px, py, pz, num;
};
__device__ __forceinline__ PairOrigin pair_origin(const TriPair &T, V3 p) {
  const f2 c0 = ld2(T, 0), c1 = ld2(T, 1), c2 = ld2(T, 2), n0 = ld2(T, 3), n1 = ld2(T, 4), n2 = ld2(T, 5);
  PairOrigin o;
  o.px = bc2(p.x) - c0;
  o.py = bc2(p.y) - c1;
  o.pz = bc2(p.z) - c2;
  o.num = fma2(o.pz, n2, fma2(o.py, n1, o.px * n0));
  return o;
}
// LEX = false: the reference's in-order strict '<' (triangles ia < ib come in
// index order).  LEX = true: keep the lexicographic minimum of (t, index) --
// the same result whatever order the triangles are visited in (BVH scenes).
template <bool LEX = false>
__device__ __forceinline__ void pair_ray(const TriPair &T, const PairOrigin &o, int ia, int ib, V3 p, V3 d, float &bt,
                                         int &bi, f2 e03, f2 e13, f2 e23) {
  const f2 n0 = ld2(T, 3), n1 = ld2(T, 4), n2 = ld2(T, 5);
  const f2 denom = fma2(n2, bc2(d.z), fma2(n1, bc2(d.y), n0 * bc2(d.x)));
  const f2 num = o.num;
#if IPT_FASTDIV
  // div_inrange(num, -denom), both halves
  const f2 nb = denom;
  const f2 r0 = f2{__builtin_amdgcn_rcpf(-denom.x), __builtin_amdgcn_rcpf(-denom.y)};
  const f2 e0 = fma2(nb, r0, bc2(1.0f));
  const f2 r1 = fma2(e0, r0, r0);
  const f2 q0 = num * r1;
  const f2 e1 = fma2(nb, q0, num);
  const f2 q1 = fma2(e1, r1, q0);
  const f2 e2 = fma2(nb, q1, num);
  const f2 t = fma2(e2, r1, q1);
#else
  const f2 t = f2{num.x / -denom.x, num.y / -denom.y};
#endif
  const f2 qx = fma2(bc2(d.x), t, bc2(p.x)), qy = fma2(bc2(d.y), t, bc2(p.y)), qz = fma2(bc2(d.z), t, bc2(p.z));
  const f2 s0 = fma2(qz, ld2(T, 8), fma2(qy, ld2(T, 7), fma2(qx, ld2(T, 6), e03)));
  const f2 s1 = fma2(qz, ld2(T, 12), fma2(qy, ld2(T, 11), fma2(qx, ld2(T, 10), e13)));
  const f2 s2 = fma2(qz, ld2(T, 16), fma2(qy, ld2(T, 15), fma2(qx, ld2(T, 14), e23)));
  if (LEX) {
    const bool va = !(fabsf(denom.x) < kMinDotUp) && !(t.x < kEpsUp) && !(s0.x > 0.f) && !(s1.x > 0.f) &&
                    !(s2.x > 0.f);
    const bool ta = va & ((t.x < bt) | ((t.x == bt) & (ia < bi)));  // bitwise: no exec-mask branches
    bt = ta ? t.x : bt;
    bi = ta ? ia : bi;
    const bool vb = !(fabsf(denom.y) < kMinDotUp) && !(t.y < kEpsUp) && !(s0.y > 0.f) && !(s1.y > 0.f) &&
                    !(s2.y > 0.f);
    const bool tb = vb & ((t.y < bt) | ((t.y == bt) & (ib < bi)));
    bt = tb ? t.y : bt;
    bi = tb ? ib : bi;
    return;
  }
  const bool ta = !(fabsf(denom.x) < kMinDotUp) && !(t.x < kEpsUp) && !(t.x >= bt) && !(s0.x > 0.f) &&
                  !(s1.x > 0.f) && !(s2.x > 0.f);
  bt = ta ? t.x : bt;
  bi = ta ? ia : bi;
  const bool tb = !(fabsf(denom.y) < kMinDotUp) && !(t.y < kEpsUp) && !(t.y >= bt) && !(s0.y > 0.f) &&
                  !(s1.y > 0.f) && !(s2.y > 0.f);
  bt = tb ? t.y : bt;
  bi = tb ? ib : bi;
}
// pair_ray's arithmetic reduced to "does either triangle accept with t below
// its bound" (ba for the first, bb for the second) -- the culled shadow cast.
__device__ __forceinline__ bool pair_occludes(const TriPair &T, const PairOrigin &o, float ba, float bb, V3 p, V3 d,
                                              f2 e03, f2 e13, f2 e23) {
  const f2 n0 = ld2(T, 3), n1 = ld2(T, 4), n2 = ld2(T, 5);
  const f2 denom = fma2(n2, bc2(d.z), fma2(n1, bc2(d.y), n0 * bc2(d.x)));
  const f2 num = o.num;
#if IPT_FASTDIV
  const f2 nb = denom;
  const f2 r0 = f2{__builtin_amdgcn_rcpf(-denom.x), __builtin_amdgcn_rcpf(-denom.y)};
  const f2 e0 = fma2(nb, r0, bc2(1.0f));
  const f2 r1 = fma2(e0, r0, r0);
  const f2 q0 = num * r1;
  const f2 e1 = fma2(nb, q0, num);
  const f2 q1 = fma2(e1, r1, q0);
  const f2 e2 = fma2(nb, q1, num);
  const f2 t = fma2(e2, r1, q1);  // == div_inrange(num, -denom) per half
#else
  const f2 t = f2{num.x / -denom.x, num.y / -denom.y};
#endif
  const f2 qx = fma2(bc2(d.x), t, bc2(p.x)), qy = fma2(bc2(d.y), t, bc2(p.y)), qz = fma2(bc2(d.z), t, bc2(p.z));
  const f2 s0 = fma2(qz, ld2(T, 8), fma2(qy, ld2(T, 7), fma2(qx, ld2(T, 6), e03)));
  const f2 s1 = fma2(qz, ld2(T, 12), fma2(qy, ld2(T, 11), fma2(qx, ld2(T, 10), e13)));
  const f2 s2 = fma2(qz, ld2(T, 16), fma2(qy, ld2(T, 15), fma2(qx, ld2(T, 14), e23)));
  const bool oa = !(fabsf(denom.x) < kMinDotUp) && !(t.x < kEpsUp) && (t.x < ba) && !(s0.x > 0.f) &&
                  !(s1.x > 0.f) && !(s2.x > 0.f);
  const bool ob = !(fabsf(denom.y) < kMinDotUp) && !(t.y < kEpsUp) && (t.y < bb) && !(s0.y > 0.f) &&
                  !(s1.y > 0.f) && !(s2.y > 0.f);
  return oa | ob;
}
__device__ __forceinline__ void hit_test_pair(const TriPair &T, int i, V3 p, V3 d, float &bt, int &bi) {
  pair_ray(T, pair_origin(T, p), i, i + 1, p, d, bt, bi, ld2(T, 9), ld2(T, 13), ld2(T, 17));
}

// Small scenes (nT <= 2 * kSmallPairs): the pair loop fully unrolled, and the
// three edge-plane offsets of each pair read from an LDS copy (e3[3j + k] =
// pair j's plane-k offset).  fma(q, e_k0, e_k3) has two wave-uniform operands,
// which the constant bus cannot feed to one VOP3P instruction, so from SGPRs
// each costs two v_mov; from LDS (immediate offsets) it costs no VALU.  The
// unrolled triangle index is an inline constant (no v_mov either).
constexpr int kSmallPairs = 16;
constexpr int kE3Floats = 6;  // LDS floats per pair: 3 plane offsets x 2
__device__ __forceinline__ int closest_hit_pairs_small(const TriPair *__restrict__ pairs, const f2 *e3, int nT,
                                                       V3 p, V3 d, float &best_t) {
  float bt = __builtin_inff();
  int bi = -1;
  // opaque copy: keeps the 16 per-pair guards as compare+branch here instead
  // of being hoisted out of the megakernel loop as SGPR masks (which spill)
  int nP = (nT + 1) >> 1;
  asm volatile("" : "+s"(nP));
  // The LDS base of the plane offsets pinned in one VGPR for the whole cast:
  // left alone, the compiler re-materialises it (a v_mov per pair, 1 of 46
  // VALU) because a ds_read takes its address from a VGPR.
  typedef __attribute__((address_space(3))) const f2 lds_f2;
  lds_f2 *e3l = (lds_f2 *)e3;
#ifndef IPT_PIN_E3
#define IPT_PIN_E3 1
#endif
  if (IPT_PIN_E3) asm volatile("" : "+v"(e3l));
#pragma unroll
  for (int j = 0; j < kSmallPairs; ++j) {
    if (j < nP) {  // wave-uniform
      const TriPair T = pairs[j];
      pair_ray(T, pair_origin(T, p), 2 * j, 2 * j + 1, p, d, bt, bi, e3l[3 * j], e3l[3 * j + 1], e3l[3 * j + 2]);
    }
  }
  best_t = bt;
  return bi;
}

__device__ __forceinline__ int closest_hit_pairs(const TriPair *__restrict__ pairs, int nT, V3 p, V3 d,
                                                 float &best_t) {
  float bt = __builtin_inff();
  int bi = -1;
  const int nP = (nT + 1) >> 1;
  TriPair nxt = pairs[0];
  for (int j = 0; j < nP; ++j) {
    const TriPair T = nxt;
    nxt = pairs[j + 1 < nP ? j + 1 : j];
    hit_test_pair(T, 2 * j, p, d, bt, bi);
  }
  best_t = bt;
  return bi;
}

// ------------------------------------------------------------ BVH closest hit
// Exact replacement of the brute-force loop for large scenes (bvh.cpp states
// why): a per-lane pre-pass over the large triangles, then the cooperative
// traversal of the 8-wide tree below; every accept keeps the lexicographic
// minimum of (t, original triangle index) -- the result of the reference's
// in-order strict-'<' loop, whatever order the triangles come in.
struct BvhView {
  const TriIsect *isect;    // original-order records (shadow target test)
  // brute-force pre-pass over the large triangles (bvh.cpp kBigFrac)
  const TriPair *big;
  const int32_t *big_idx;   // original indices, 2 per pair
  const f2 *big_e3;         // LDS: the pairs' edge-plane offsets
  int nbig;                 // pairs (<= kSmallPairs)
  const PairBox2 *big_boxes;  // the pairs' acceptance boxes (culled shadow pre-pass)
  const float *big_lds;       // LDS copy of the pairs + their indices (culled path pre-pass), or nullptr
  const float *emit_is;       // LDS copy of the emitters' TriIsect records (shadow target test), or nullptr
};
constexpr int kBvhDone = (int)0x80000000;
// Profiling build (make variant DEFS=-DIPT_BVH_STATS): work counters summed
// over all lanes (ipt_debug_bvh_stats) -- the "tests actually executed" of
// the roofline.  Cooperative traversal: [0] tree rays, [1] 8-wide node
// visits, [2] leaf visits, [3] shadow rays occluded in the tree, [4] leaf
// triangle tests, [5] coop calls with >= 1 ray (per wave), [6] coop rounds
// (per wave); pre-pass: [7] casts, [8] large-triangle tests, [9] shadow
// target tests, [10] shadow rays decided before the tree.
constexpr int kBvhStats = 23;  // [12..17]: culled shadow casts (shadow_hit_pairs_small); [18..22]: culled path casts
#ifdef IPT_BVH_STATS
__device__ unsigned long long g_bvh_stats[kBvhStats];
#endif

// The large triangles, unrolled like closest_hit_pairs_small (scalar-loaded
// pairs, plane offsets from LDS) with the lexicographic accept.
// LEX = false is exact only from the empty state (bt = inf): the pairs come
// in ascending original index, so the strict in-order accept is then already
// the lexicographic minimum (2-3 fewer VALU per triangle); the shadow
// pre-pass starts from the target's (t, index) and needs LEX.
// The pairs and indices are read through the constant address space: the
// kernel writes global memory, so through a plain pointer (reached via the
// TraceArgs kernarg, not a __restrict__ parameter) the compiler may not use
// the scalar cache and emits per-lane vector loads of the same 144 B.
typedef __attribute__((address_space(4))) const float cst_f32;
typedef __attribute__((address_space(4))) const int32_t cst_i32;
__device__ __forceinline__ TriPair load_pair_cst(const TriPair *p) {
  const cst_f32 *q = (const cst_f32 *)p;
  TriPair T;
#pragma unroll
  for (int i = 0; i < 36; ++i) T.f[i >> 1][i & 1] = q[i];
  return T;
}
template <bool LEX>
__device__ __forceinline__ void bvh_big_pass(const BvhView &B, V3 p, V3 d, float &bt, int &bi) {
  int nP = B.nbig;
  asm volatile("" : "+s"(nP));
  typedef __attribute__((address_space(3))) const f2 lds_f2;  // LDS base pinned in a VGPR (see closest_hit_pairs_small)
  lds_f2 *e3l = (lds_f2 *)B.big_e3;
  if (IPT_PIN_E3) asm volatile("" : "+v"(e3l));
  const cst_i32 *bidx = (const cst_i32 *)B.big_idx;
#pragma unroll
  for (int j = 0; j < kSmallPairs; ++j) {
    if (j < nP) {  // wave-uniform
      const TriPair T = load_pair_cst(B.big + j);
      pair_ray<LEX>(T, pair_origin(T, p), bidx[2 * j], bidx[2 * j + 1], p, d, bt, bi, e3l[3 * j], e3l[3 * j + 1],
                    e3l[3 * j + 2]);
    }
  }
}

// Slab form of a ray: t = fma(box, 1/d, -p/d) per axis; |d| < 2^-60 makes
// that axis's parameters NaN, which min/max ignore (the slab is dropped:
// conservative).  bvh.cpp states why the rounding of this form is covered.
__device__ __forceinline__ int lane_rank64(uint64_t m) {  // set bits of m below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
struct SlabRay {
  f2 ix, iy, iz, ox, oy, oz;
};
__device__ __forceinline__ SlabRay slab_ray(V3 p, V3 d) {
  const float qnan = __builtin_nanf("");
  const float ix = fabsf(d.x) < 0x1p-60f ? 0.f : __builtin_amdgcn_rcpf(d.x);
  const float iy = fabsf(d.y) < 0x1p-60f ? 0.f : __builtin_amdgcn_rcpf(d.y);
  const float iz = fabsf(d.z) < 0x1p-60f ? 0.f : __builtin_amdgcn_rcpf(d.z);
  const float ox = fabsf(d.x) < 0x1p-60f ? qnan : -(p.x * ix);
  const float oy = fabsf(d.y) < 0x1p-60f ? qnan : -(p.y * iy);
  const float oz = fabsf(d.z) < 0x1p-60f ? qnan : -(p.z * iz);
  return SlabRay{bc2(ix), bc2(iy), bc2(iz), bc2(ox), bc2(oy), bc2(oz)};
}
// Shadow ray of the small-scene loop (closest_hit_pairs_small's scenes)
// towards emitter triangle `target`, with pair culling.  Only `result ==
// target` and then t are used by the caller, so: (1) the target is tested
// first (a miss decides the lane); (2) the pairs are then visited in index
// order keeping the lexicographic minimum of (t, index) -- the same hit as the
// in-order strict '<' loop whatever is skipped, as long as no skipped pair
// could be accepted with t <= bt (bvh.cpp, BVH traversal); (3) a pair is
// skipped for the whole wave when no live lane's ray enters its acceptance
// box (PairBox2) within [kEpsUp, bt].  The lower bound is kEpsUp, not 0: the
// test rejects t < kEpsUp, and bvh.cpp's padding keeps the computed t of
// every acceptable hit inside the computed [entry, exit].  A shadow ray
// starts ON its vertex's wall, inside that wall's thin box, but leaves it
// long before t = 1e-2 unless it grazes the wall; all rays of a wave head for
// the light, so most pairs are skipped for every lane.  A lane is done as
// soon as the best hit is not the target (occluded).
#ifndef IPT_SHADOW_CULL
#define IPT_SHADOW_CULL 1
#endif
// IPT_SHADOW_PO=1: the culled shadow cast also skips, per lane, the pairs
// that cannot occlude any shadow ray from its vertex's triangle to its
// emitter (static potential-occluder masks, bvh.cpp shadow_occluder_masks)
#ifndef IPT_SHADOW_PO
#define IPT_SHADOW_PO 1
#endif
typedef __attribute__((address_space(3))) const uint32_t lds_u32c;
// Bit j: the ray enters pair j's acceptance box within [kEpsUp, bt] (the
// pairs' boxes two per PairBox2 record; scalar loads).
// allow: the pairs this lane may need at all (shadow rays: the potential
// occluders of its (source triangle, emitter), bvh.cpp
// shadow_occluder_masks); a record no lane allows is skipped by the wave.
__device__ __forceinline__ uint32_t pair_box_bits(const PairBox2 *boxes, int nP, V3 p, V3 d, float bt,
                                                  uint32_t allow = 0xffffffffu) {
  uint32_t need = 0;
  const SlabRay r = slab_ray(p, d);
#pragma unroll
  for (int J = 0; J < kSmallPairs / 2; ++J) {
    if (2 * J < nP && __builtin_amdgcn_ballot_w64((allow >> (2 * J)) & 3u)) {  // wave-uniform
      const cst_f32 *B = (const cst_f32 *)(boxes + J);
      const f2 tx0 = fma2(f2{B[0], B[1]}, r.ix, r.ox), tx1 = fma2(f2{B[2], B[3]}, r.ix, r.ox);
      const f2 ty0 = fma2(f2{B[4], B[5]}, r.iy, r.oy), ty1 = fma2(f2{B[6], B[7]}, r.iy, r.oy);
      const f2 tz0 = fma2(f2{B[8], B[9]}, r.iz, r.oz), tz1 = fma2(f2{B[10], B[11]}, r.iz, r.oz);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float en =
            fmaxf(fmaxf(fminf(tx0[h], tx1[h]), fminf(ty0[h], ty1[h])), fmaxf(fminf(tz0[h], tz1[h]), kEpsUp));
        const float ex = fminf(fminf(fmaxf(tx0[h], tx1[h]), fmaxf(ty0[h], ty1[h])), fminf(fmaxf(tz0[h], tz1[h]), bt));
        need |= (en <= ex ? 1u : 0u) << (2 * J + h);
      }
    }
  }
  // an odd nP's last record has an all-+inf second half, which a ray with
  // three positive direction components "enters" when bt = inf: not a pair
  return need & allow & ((1u << nP) - 1u);
}

// The occlusion part of a culled shadow cast over nP pairs (pair_at(j):
// the TriPair, idx_at(k): original triangle index k of the pass, e3l: the
// pairs' plane offsets in LDS).  A pair is tested only when some live lane's
// box bit is set; only "is the target still the lexicographic minimum"
// matters, so bt stays t_e: pair triangle i occludes iff it is accepted with
// t < t_e, or t == t_e and i < target, i.e. t < bound_i with bound_i =
// nextup(t_e) for i < target (t_e >= kEpsUp > 0 is finite: +1 on the bits is
// nextup).  Returns the lane's "still visible".
typedef __attribute__((address_space(3))) const f2 lds_f2c;
template <class PairAt, class IdxAt>
__device__ __forceinline__ bool occlusion_pass(PairAt pair_at, IdxAt idx_at, lds_f2c *e3l, int nP, uint32_t need, V3 p,
                                               V3 d, int target, float te, bool live) {
  const float teu = __uint_as_float(__float_as_uint(te) + 1u);
#pragma unroll
  for (int j = 0; j < kSmallPairs; ++j) {
    if (j < nP) {  // wave-uniform
      if (__builtin_amdgcn_ballot_w64(live && ((need >> j) & 1u))) {
#ifdef IPT_BVH_STATS
        if (__lane_id() == __ffsll((unsigned long long)__builtin_amdgcn_ballot_w64(true)) - 1)
          atomicAdd(&g_bvh_stats[15], 1ull);                // wave-level pair tests
#endif
        if (live) {
#ifdef IPT_BVH_STATS
          atomicAdd(&g_bvh_stats[16], 1ull);                // lane pair tests
#endif
          const TriPair T = pair_at(j);
          const bool occ = pair_occludes(T, pair_origin(T, p), idx_at(2 * j) < target ? teu : te,
                                         idx_at(2 * j + 1) < target ? teu : te, p, d, e3l[3 * j], e3l[3 * j + 1],
                                         e3l[3 * j + 2]);
          live = live && !occ;
        }
      }
    }
  }
  return live;
}

// A TriPair from an LDS copy (per-lane gather: nine 16-B reads).
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f4v lds_f4c;
__device__ __forceinline__ TriPair load_pair_lds(const lds_f32 *pl, int j) {
  const lds_f4c *q = (const lds_f4c *)(pl + 36 * j);
  TriPair T;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const f4v v = q[k];
    T.f[2 * k][0] = v.x;
    T.f[2 * k][1] = v.y;
    T.f[2 * k + 1][0] = v.z;
    T.f[2 * k + 1][1] = v.w;
  }
  return T;
}
// The target's record comes from the workgroup's LDS copy of the TriIsect array.
__device__ __forceinline__ int shadow_hit_pairs_small(const lds_f32 *isect_lds, const TriPair *__restrict__ pairs,
                                                      const PairBox2 *__restrict__ boxes, const f2 *e3, int nT, V3 p,
                                                      V3 d, int target, float &best_t, uint32_t allow = 0xffffffffu) {
  float bt = __builtin_inff();
  int bi = -1;
  bool live;
  {
    TriIsect T;
    float *tf = reinterpret_cast<float *>(&T);
    const lds_f32 *q = isect_lds + 20 * target;
#pragma unroll
    for (int k = 0; k < 20; ++k) tf[k] = q[k];
    hit_test(T, target, p, d, bt, bi);
    live = bi >= 0;
  }
  int nP = (nT + 1) >> 1;
  asm volatile("" : "+s"(nP));
  lds_f2c *e3l = (lds_f2c *)e3;
  if (IPT_PIN_E3) asm volatile("" : "+v"(e3l));
#ifdef IPT_BVH_STATS
  atomicAdd(&g_bvh_stats[12], 1ull);                      // shadow lanes
  if (live) atomicAdd(&g_bvh_stats[13], 1ull);            // ... whose target is accepted
  if (live) atomicAdd(&g_bvh_stats[17], (unsigned long long)nP);  // lane box tests
  if (__lane_id() == __ffsll((unsigned long long)__builtin_amdgcn_ballot_w64(true)) - 1)
    atomicAdd(&g_bvh_stats[14], 1ull);                    // wave-level calls
#endif
  // opaque per cast: the compiler would otherwise hoist the loop-invariant
  // box loads out of the megakernel loop into SGPRs, which then spill
  asm volatile("" : "+s"(boxes));
  if (__builtin_amdgcn_ballot_w64(live)) {
    // box bits first, so that the slab registers are dead before the pair tests
    // the target's own pair is always needed (the ray ends in its box and the
    // partner may tie ahead of the target): its bit is set without a box test
    const uint32_t tbit = 1u << (target >> 1);
    const uint32_t need = live ? (pair_box_bits(boxes, nP, p, d, bt, allow & ~tbit) | tbit) : 0u;
    live = occlusion_pass([&](int j) { return pairs[j]; }, [&](int k) { return k; }, e3l, nP, need, p, d, target, bt,
                          live);
    if (!live && bi >= 0) bi = -1;  // occluded: not the target (the caller only compares with it)
  }
  if (!live) bi = -1;
  best_t = bt;
  return bi;
}

// Path ray of the small-scene loop with per-lane pair culling
// (IPT_PATH_CULL): a lane tests only the pairs whose acceptance box its ray
// enters within [kEpsUp, inf) -- no other triangle can accept it (the shadow
// cull's argument with an unbounded far end) -- in ascending index order with
// pair_ray's arithmetic and in-order strict accept.  Over a subsequence that
// still holds every triangle the ray can accept, that is the full loop's hit
// (the lexicographic minimum of (t, index) over the accepting triangles).
// The pairs come per lane from the workgroup's LDS copy (nine 16-B reads), so
// the wave runs the test max-over-lanes(pairs entered) times instead of once
// per pair: a path ray in a room enters the box of the wall it hits (and, at
// edges and corners, a neighbour's; crossing an object, its two faces'),
// whereas the wave's lanes together hit nearly every wall.
#ifndef IPT_PATH_CULL
#define IPT_PATH_CULL 1
#endif
__device__ __forceinline__ int closest_hit_pairs_culled(const lds_f32 *pairs_lds, const PairBox2 *__restrict__ boxes,
                                                        int nT, V3 p, V3 d, float &best_t) {
  float bt = __builtin_inff();
  int bi = -1;
  int nP = (nT + 1) >> 1;
  asm volatile("" : "+s"(nP));
  asm volatile("" : "+s"(boxes));  // see shadow_hit_pairs_small
  uint32_t need = pair_box_bits(boxes, nP, p, d, bt);
#ifdef IPT_BVH_STATS
  atomicAdd(&g_bvh_stats[18], 1ull);                                            // path casts
  atomicAdd(&g_bvh_stats[19], (unsigned long long)__builtin_popcount(need));    // lane pair tests
  atomicAdd(&g_bvh_stats[20], (unsigned long long)nP);                          // lane box tests
  {
    const uint64_t act = __builtin_amdgcn_ballot_w64(true);
    const bool first = __lane_id() == __ffsll((unsigned long long)act) - 1;
    uint32_t mx = need;  // wave loop trips = max over lanes of popcount(need)
    int trips = __builtin_popcount(mx);
    for (int o = 32; o >= 1; o >>= 1) trips = max(trips, __shfl_xor(trips, o));
    if (first) {
      atomicAdd(&g_bvh_stats[21], 1ull);                                        // wave-level calls
      atomicAdd(&g_bvh_stats[22], (unsigned long long)trips);                   // wave-level loop trips
    }
  }
#endif
  while (need) {  // per lane: the wave loops while any lane has a pair left
    const int j = __builtin_ctz(need);
    need &= need - 1u;
    const TriPair T = load_pair_lds(pairs_lds, j);
    pair_ray(T, pair_origin(T, p), 2 * j, 2 * j + 1, p, d, bt, bi, ld2(T, 9), ld2(T, 13), ld2(T, 17));
  }
  best_t = bt;
  return bi;
}

// The large-triangle pre-pass of a path ray with closest_hit_pairs_culled's
// per-lane pair culling (boxes: big_boxes; pairs and original indices from
// the LDS copy big_lds).  From the empty state over ascending original
// indices the strict in-order accept is the lexicographic minimum, as in
// bvh_big_pass<false>.
typedef __attribute__((address_space(3))) const int32_t lds_i32c;
__device__ __forceinline__ void bvh_big_pass_culled(const BvhView &B, V3 p, V3 d, float &bt, int &bi) {
  int nP = B.nbig;
  asm volatile("" : "+s"(nP));
  const PairBox2 *boxes = B.big_boxes;
  asm volatile("" : "+s"(boxes));
  uint32_t need = pair_box_bits(boxes, nP, p, d, bt);
  const lds_f32 *pl = (const lds_f32 *)B.big_lds;
  const lds_i32c *il = (const lds_i32c *)(B.big_lds + 36 * nP);
#ifdef IPT_BVH_STATS
  atomicAdd(&g_bvh_stats[17], (unsigned long long)nP);  // lane box tests
  atomicAdd(&g_bvh_stats[8], 2ull * (unsigned long long)__builtin_popcount(need));
#endif
  while (need) {
    const int j = __builtin_ctz(need);
    need &= need - 1u;
    const TriPair T = load_pair_lds(pl, j);
    pair_ray(T, pair_origin(T, p), il[2 * j], il[2 * j + 1], p, d, bt, bi, ld2(T, 9), ld2(T, 13), ld2(T, 17));
  }
}

// The part of a cast done before the traversal: the shadow target's own
// test (target >= 0) and the large-triangle pre-pass.  Returns false when
// the cast is already decided (shadow target missed or occluded).
template <bool SHADOW>
// eidx: the target's emitter index (its record in B.emit_is), < 0 = unknown.
__device__ __forceinline__ bool bvh_prepass(const BvhView &B, V3 p, V3 d, float &bt, int &bi, int target,
                                            uint32_t allow = 0xffffffffu, int eidx = -1) {
  bt = __builtin_inff();
  bi = -1;
#ifdef IPT_BVH_STATS
  atomicAdd(&g_bvh_stats[7], 1ull);
  if (!(SHADOW && IPT_SHADOW_CULL) && !(!SHADOW && IPT_PATH_CULL && B.big_lds))
    atomicAdd(&g_bvh_stats[8], 2ull * (unsigned long long)B.nbig);
  if (SHADOW && IPT_SHADOW_CULL) atomicAdd(&g_bvh_stats[17], (unsigned long long)B.nbig);  // lane box tests
  if (SHADOW) atomicAdd(&g_bvh_stats[9], 1ull);
#endif
  if (SHADOW) {
    if (B.emit_is && eidx >= 0) {  // from the LDS copy (per-lane gather) instead of L2
      TriIsect T;
      float *tf = reinterpret_cast<float *>(&T);
      const lds_f32 *q = (const lds_f32 *)B.emit_is + 20 * eidx;
#pragma unroll
      for (int k = 0; k < 20; ++k) tf[k] = q[k];
      hit_test(T, target, p, d, bt, bi);
    } else {
      hit_test(B.isect[target], target, p, d, bt, bi);
    }
    if (bi < 0) {  // the target itself is missed: not the closest hit either
#ifdef IPT_BVH_STATS
      atomicAdd(&g_bvh_stats[10], 1ull);
#endif
      return false;
    }
  }
  if (SHADOW && IPT_SHADOW_CULL && B.nbig > 0) {
    // the large triangles as in the small scenes' culled shadow cast: only
    // the pairs whose acceptance box some lane's ray enters within
    // [kEpsUp, t_target], reduced to "does it occlude the target"
    int nP = B.nbig;
    asm volatile("" : "+s"(nP));
    lds_f2c *e3l = (lds_f2c *)B.big_e3;
    if (IPT_PIN_E3) asm volatile("" : "+v"(e3l));
    const cst_i32 *bidx = (const cst_i32 *)B.big_idx;
    const PairBox2 *boxes = B.big_boxes;
    asm volatile("" : "+s"(boxes));
    const uint32_t need = pair_box_bits(boxes, nP, p, d, bt, allow);
    const bool vis = occlusion_pass([&](int j) { return load_pair_cst(B.big + j); }, [&](int k) { return bidx[k]; },
                                    e3l, nP, need, p, d, target, bt, true);
    if (!vis) {  // occluded by a large triangle: decided
      bi = -1;
#ifdef IPT_BVH_STATS
      atomicAdd(&g_bvh_stats[10], 1ull);
#endif
      return false;
    }
  } else if (!SHADOW && IPT_PATH_CULL && B.big_lds && B.nbig > 0) {
    bvh_big_pass_culled(B, p, d, bt, bi);
  } else if (B.nbig > 0) {
    bvh_big_pass<SHADOW>(B, p, d, bt, bi);
    if (SHADOW && bi != target) {  // occluded by a large triangle: decided
#ifdef IPT_BVH_STATS
      atomicAdd(&g_bvh_stats[10], 1ull);
#endif
      return false;
    }
  }
  return true;
}

// ------------------------------------------------------------ cooperative BVH traversal
// The per-lane traversal above is latency-bound: the ~10% of lanes whose ray
// reaches the tree each walk ~13 dependent node/leaf steps while the rest of
// the wave idles.  Here the wave splits into 8 groups of 8 lanes and each
// group carries ONE ray through an 8-wide tree (WideNode): lane j tests child
// j's box, the group picks the nearest hit child with a DPP min-reduction and
// pushes the others on a group stack in LDS; at a leaf lane j tests triangle
// j and a lexicographic (t, index) DPP reduction merges the results.  About
// 3 levels + a leaf or two instead of ~13 steps, 8 rays per wave per round.
// All lanes of a group hold identical copies of the ray state, so every
// branch is group-uniform and the DPP reductions (xor 1, xor 2 within quads,
// half-row mirror) only read lanes of the same, active group.
constexpr int kWideF4 = 16;  // float4 per wide node (WideNode, 256 B)
// Children are visited in the ray octant's precomputed front-to-back order
// (bvh.cpp: slot o's pad word holds each child's rank): lane j reads child j
// and that word with independent LDS reads, the group ORs 1 << rank(j) of its
// hit children (three DPP stages) and the next node is the hit child of the
// lowest rank, broadcast by a DPP min -- one LDS round trip per visit.  (Round
// 2's form read the word first, then child perm[j], and broadcast the next
// node with ds_bpermute: three dependent LDS round trips.)  Exact either way:
// the visit order never changes the lexicographic result.  (Rejected: a step
// that first issued every group's reads -- node from LDS, or the leaf's
// triangles -- and then computed, so node and leaf latencies would overlap:
// north-star forward 3.78 -> 4.92 ms, adjoint 4.55 -> 7.53, the triangle
// registers held across the step spilled; profiles/r04/variants_coop_split_r04p.log.)
struct CoopView {
  const float4 *wn;    // wide nodes (WideNode, kWideF4 float4 each)
  bool wn_lds;         // wn points into LDS (else global memory)
  const TriIsect *wt;  // leaf triangles, pad[0] = original index
  uint32_t *stk;       // LDS: this wave's 8 group stacks, `stride` entries each
  int stride;
  float root[6];       // the tree's box: lo xyz, hi xyz
  float sphere[4];     // the tree's bounding sphere: centre xyz, padded radius^2 (bvh.cpp tree_cull)
};

// Whole-wave neighbour shifts (GFX9 DPP wave_shr:1 / wave_shl:1, one VALU
// move): lane i receives lane i-1's (shr) or lane i+1's (shl) value; lane 0
// (shr) / lane 63 (shl) receive 0 -- callers never consume those.
__device__ __forceinline__ float wave_shr1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float wave_shl1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}

// One step of the adjoint sweep's two neighbour chains (ipt_hip.hip, the
// wave-parallel sweep), with the wave shifts fused into the VALU operations
// that consume them (the compiler keeps them as separate DPP moves and packs
// the products into v_pk_mul_f32, which issues at half rate: 27 VALU slots
// per step instead of these 18-20).  Same IEEE operations, same order:
//  chain_step_shifted (operands pre-shifted once per round, loop-invariant
//  keep masks; ADJ / ADJW):
//    m = keepM ? m : (shr(m) * tl) * cl        s = keepS ? s : al + shl(s) * bl
//  chain_step_select (ADJU: a lane takes its neighbour's product at its step):
//    m = (km == i) ? shr((m * t) * c) : m      s = (kr == i) ? shl(a + b * s) : s
// shr / shl read lane i-1 / i+1 (wave_shr:1 / wave_shl:1), 0 at the wave's
// edge, as wave_shr1 / wave_shl1.  A DPP source written by a VALU needs two
// wait states: the shifted form's sources are the previous step's selects
// (the leading s_nop), the select form's are written >= 2 instructions before.
__device__ __forceinline__ void chain_step_shifted(float &mx, float &my, float &mz, float &sx, float &sy, float &sz,
                                                   V3 tl, float cl, V3 al, V3 bl, uint64_t keepM, uint64_t keepS) {
  float t0, t1, t2, u0, u1, u2;
  asm volatile(
      "s_nop 1\n\t"
      "v_mul_f32_dpp %6, %0, %12 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_mul_f32_dpp %7, %1, %13 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_mul_f32_dpp %8, %2, %14 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_mul_f32_dpp %9, %3, %19 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_mul_f32_dpp %10, %4, %20 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_mul_f32_dpp %11, %5, %21 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_mul_f32_e32 %6, %6, %15\n\t"
      "v_mul_f32_e32 %7, %7, %15\n\t"
      "v_mul_f32_e32 %8, %8, %15\n\t"
      "v_add_f32_e32 %9, %16, %9\n\t"
      "v_add_f32_e32 %10, %17, %10\n\t"
      "v_add_f32_e32 %11, %18, %11\n\t"
      "v_cndmask_b32_e64 %0, %6, %0, %22\n\t"
      "v_cndmask_b32_e64 %1, %7, %1, %22\n\t"
      "v_cndmask_b32_e64 %2, %8, %2, %22\n\t"
      "v_cndmask_b32_e64 %3, %9, %3, %23\n\t"
      "v_cndmask_b32_e64 %4, %10, %4, %23\n\t"
      "v_cndmask_b32_e64 %5, %11, %5, %23"
      : "+v"(mx), "+v"(my), "+v"(mz), "+v"(sx), "+v"(sy), "+v"(sz), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(u0),
        "=&v"(u1), "=&v"(u2)
      : "v"(tl.x), "v"(tl.y), "v"(tl.z), "v"(cl), "v"(al.x), "v"(al.y), "v"(al.z), "v"(bl.x), "v"(bl.y), "v"(bl.z),
        "s"(keepM), "s"(keepS));
}
__device__ __forceinline__ void chain_step_select(float &mx, float &my, float &mz, float &sx, float &sy, float &sz,
                                                  V3 t, float c, V3 a, V3 b, int km, int kr, int i) {
  float t0, t1, t2, u0, u1, u2;
  asm volatile(
      "v_mul_f32_e32 %6, %0, %12\n\t"
      "v_mul_f32_e32 %7, %1, %13\n\t"
      "v_mul_f32_e32 %8, %2, %14\n\t"
      "v_mul_f32_e32 %9, %3, %19\n\t"
      "v_mul_f32_e32 %10, %4, %20\n\t"
      "v_mul_f32_e32 %11, %5, %21\n\t"
      "v_mul_f32_e32 %6, %6, %15\n\t"
      "v_mul_f32_e32 %7, %7, %15\n\t"
      "v_mul_f32_e32 %8, %8, %15\n\t"
      "v_add_f32_e32 %9, %16, %9\n\t"
      "v_add_f32_e32 %10, %17, %10\n\t"
      "v_add_f32_e32 %11, %18, %11\n\t"
      "v_cmp_ne_u32_e32 vcc, %24, %22\n\t"
      "v_cndmask_b32_dpp %0, %6, %0, vcc wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %1, %7, %1, vcc wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %2, %8, %2, vcc wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cmp_ne_u32_e32 vcc, %24, %23\n\t"
      "v_cndmask_b32_dpp %3, %9, %3, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %4, %10, %4, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %5, %11, %5, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "+v"(mx), "+v"(my), "+v"(mz), "+v"(sx), "+v"(sy), "+v"(sz), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(u0),
        "=&v"(u1), "=&v"(u2)
      : "v"(t.x), "v"(t.y), "v"(t.z), "v"(c), "v"(a.x), "v"(a.y), "v"(a.z), "v"(b.x), "v"(b.y), "v"(b.z), "v"(km),
        "v"(kr), "s"(i)
      : "vcc");
}

// Minimum of a 32-bit int over the 8 lanes of each group: three DPP stages
// (quad_perm [1,0,3,2]: lane ^ 1, [2,3,0,1]: lane ^ 2, row_half_mirror: the
// other quad), each fused by the compiler into one v_min_i32_dpp.
template <int CTRL>
__device__ __forceinline__ int min_dpp(int v) {
  return min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ int group_min_i32(int v) { return min_dpp<0x141>(min_dpp<0x4E>(min_dpp<0xB1>(v))); }
template <int CTRL>
__device__ __forceinline__ uint32_t or_dpp(uint32_t v) {
  return v | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
// OR over the 8 lanes of each group (same three stages as group_min_i32)
__device__ __forceinline__ uint32_t group_or_u32(uint32_t v) { return or_dpp<0x141>(or_dpp<0x4E>(or_dpp<0xB1>(v))); }
// Lexicographic minimum of (t, i) over the 8 lanes of each group.  Every t
// here is an accepted hit parameter (>= kEpsUp) or +inf, never NaN or
// negative, so its bit pattern orders like its value: the minimum t is an
// integer minimum of the bits, then the minimum index among the lanes that
// hold it (7 VALU instead of ~21 for a (t, i) compare-select per stage).
__device__ __forceinline__ void group_lexmin(float &t, int &i) {
  const int tb = group_min_i32(__float_as_int(t));
  i = group_min_i32(__float_as_int(t) == tb ? i : 0x7fffffff);
  t = __int_as_float(tb);
}
__device__ __forceinline__ float bperm_f(int addr, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}

// Does the ray reach the tree's box within [0, bt], and its bounding sphere?
// The sphere (bvh.cpp tree_cull: every tree triangle's acceptance region
// inside, the radius padded far past this test's rounding) drops the rays
// that cross the box's corners: a ball fills ~half of a box's mean projected
// area.  A ray whose origin lies outside it and whose line misses it (or
// points away from it) accepts no tree triangle.
#ifndef IPT_TREE_SPHERE
#define IPT_TREE_SPHERE 1
#endif
// The sphere test (b^2 - cc with b = oc.d) and tree_skip's fixed dot margin
// assume |d| = 1: the megakernel's rays come from unit().  `unit` false (a
// caller's ray of any length, closest_hit_kernel) keeps the box test only.
__device__ __forceinline__ bool coop_root_test(const CoopView &C, V3 p, V3 d, float bt, bool unit = true) {
  const SlabRay r = slab_ray(p, d);
  const float tx0 = fmaf(C.root[0], r.ix.x, r.ox.x), tx1 = fmaf(C.root[3], r.ix.x, r.ox.x);
  const float ty0 = fmaf(C.root[1], r.iy.x, r.oy.x), ty1 = fmaf(C.root[4], r.iy.x, r.oy.x);
  const float tz0 = fmaf(C.root[2], r.iz.x, r.oz.x), tz1 = fmaf(C.root[5], r.iz.x, r.oz.x);
  const float en = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
  const float ex = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), bt));
  if (IPT_TREE_SPHERE && unit) {
    const V3 oc = mk(p.x - C.sphere[0], p.y - C.sphere[1], p.z - C.sphere[2]);
    const float b = dot3(oc, d), cc = dot3(oc, oc) - C.sphere[3];
    const bool miss = cc > 0.f && (b > 0.f || fmaf(b, b, -cc) < 0.f);
    return en <= ex && !miss;
  }
  return en <= ex;
}
// The source-plane test (bvh.cpp tree_cull): the ray leaves a point that
// triangle s accepted, and dot(n_s, d) >= tau_s puts every tree triangle
// behind s's plane at every t the hit test accepts.  sc: {n_s, tau_s} per
// triangle; s < 0 (camera rays): no skip.
#ifndef IPT_TREE_SKIP
#define IPT_TREE_SKIP 1
#endif
__device__ __forceinline__ bool tree_skip(const float4 *sc, int s, V3 d, bool unit = true) {
  if (s < 0 || !unit) return false;
  const float4 v = sc[s];
  return dot3(mk(v.x, v.y, v.z), d) >= v.w;
}

// The fp32 test of one triangle without the best-t condition (hit_test's
// arithmetic): t if it accepts, +inf if not.  A NaN t (only from a NaN or
// infinite ray) is mapped to +inf: group_lexmin orders t by its bit pattern,
// where a negative NaN would win the group minimum and hide a real hit.
__device__ __forceinline__ float tri_accept_t(const TriIsect &T, V3 p, V3 d) {
  const float denom = fmaf(T.n[2], d.z, fmaf(T.n[1], d.y, T.n[0] * d.x));
  const float px = p.x - T.c[0], py = p.y - T.c[1], pz = p.z - T.c[2];
  const float num = fmaf(pz, T.n[2], fmaf(py, T.n[1], px * T.n[0]));
  const float t = div_inrange(num, -denom);
  const float qx = fmaf(d.x, t, p.x), qy = fmaf(d.y, t, p.y), qz = fmaf(d.z, t, p.z);
  const float s0 = fmaf(qz, T.e0[2], fmaf(qy, T.e0[1], fmaf(qx, T.e0[0], T.e0[3])));
  const float s1 = fmaf(qz, T.e1[2], fmaf(qy, T.e1[1], fmaf(qx, T.e1[0], T.e1[3])));
  const float s2 = fmaf(qz, T.e2[2], fmaf(qy, T.e2[1], fmaf(qx, T.e2[0], T.e2[3])));
  const bool ok = !(fabsf(denom) < kMinDotUp) && t >= kEpsUp && !(s0 > 0.f) && !(s1 > 0.f) && !(s2 > 0.f);
  return ok ? t : __builtin_inff();
}

// One group's walk of the tree with its ray (gp, gd) from (gt, gi): the 8
// lanes of the group hold identical copies of the ray state, so every branch
// is group-uniform.  SHADOW: gi on entry is the target emitter; the walk
// stops as soon as gi is no longer the target (occluded).
template <bool SHADOW>
__device__ __forceinline__ void coop_traverse(const CoopView &C, V3 gp, V3 gd, float &gt, int &gi) {
  const int lane = (int)__lane_id();
  const int g = lane >> 3, j = lane & 7;
  const int target = gi;
  const SlabRay r = slab_ray(gp, gd);
  const int oct = (gd.x < 0.f ? 1 : 0) | (gd.y < 0.f ? 2 : 0) | (gd.z < 0.f ? 4 : 0);
  uint32_t *stk = C.stk + g * C.stride;
  int node = 0, sp = 0;
#ifdef IPT_BVH_STATS
  uint32_t st_nodes = 0, st_leaves = 0;
#endif
  for (;;) {
    if (node >= 0) {  // wide node: lane j tests child j
#ifdef IPT_BVH_STATS
      ++st_nodes;
#endif
      // lane j tests child j; its rank in the ray octant's front-to-back order
      float4 a, b;
      uint32_t rw;
      if (C.wn_lds) {  // typed per branch: ds_read_b128, not a flat load
        const lds_f32 *pw = (const lds_f32 *)C.wn + 4 * (2 * (8 * node + oct) + 1) + 3;
        const lds_v4 *q = (const lds_v4 *)C.wn + 2 * (8 * node + j);
        rw = __float_as_uint(*pw);
        const v4f qa = q[0], qb = q[1];
        a = make_float4(qa.x, qa.y, qa.z, qa.w);
        b = make_float4(qb.x, qb.y, qb.z, qb.w);
      } else {
        const gbl_f32 *pw = (const gbl_f32 *)C.wn + 4 * (2 * (8 * node + oct) + 1) + 3;
        const gbl_v4 *q = (const gbl_v4 *)C.wn + 2 * (8 * node + j);
        rw = __float_as_uint(*pw);
        const v4f qa = q[0], qb = q[1];
        a = make_float4(qa.x, qa.y, qa.z, qa.w);
        b = make_float4(qb.x, qb.y, qb.z, qb.w);
      }
      const uint32_t rj = (rw >> (3 * j)) & 7u;
      const int ref = __float_as_int(b.z);
      const float tx0 = fmaf(a.x, r.ix.x, r.ox.x), tx1 = fmaf(a.w, r.ix.x, r.ox.x);
      const float ty0 = fmaf(a.y, r.iy.x, r.oy.x), ty1 = fmaf(b.x, r.iy.x, r.oy.x);
      const float tz0 = fmaf(a.z, r.iz.x, r.oz.x), tz1 = fmaf(b.y, r.iz.x, r.oz.x);
      const float en = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
      const float ex = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), gt));
      const bool h = en <= ex && ref != kWideEmpty;
      const uint32_t hm = group_or_u32(h ? 1u << rj : 0u);  // hit children by rank
      if (hm == 0) {
        node = sp > 0 ? (int)stk[--sp] : kBvhDone;
      } else {
        // next = the nearest-ranked hit child; the other hits are pushed
        // farthest first, so they pop in front-to-back order
        const uint32_t f = (uint32_t)__builtin_ctz(hm);
        const int nx = group_min_i32(h && rj == f ? ref : 0x7fffffff);
        const uint32_t others = hm & (hm - 1u);
        if ((others >> rj) & 1u) stk[sp + __popc(others >> (rj + 1))] = (uint32_t)ref;
        sp += __popc(others);
        node = nx;
      }
    } else {  // leaf: lane j tests triangle j (8 per round)
#ifdef IPT_BVH_STATS
      ++st_leaves;
#endif
      const int code = ~node;
      const int first = code >> 4, cnt = (code & 15) + 1;
#ifdef IPT_BVH_STATS
      if (j == 0) atomicAdd(&g_bvh_stats[4], (unsigned long long)cnt);
#endif
      for (int base = 0; base < cnt; base += 8) {
        float tj = __builtin_inff();
        int ij = 0x7fffffff;
        if (base + j < cnt) {
          const TriIsect &T = C.wt[first + base + j];
          tj = tri_accept_t(T, gp, gd);
          ij = __float_as_int(T.pad[0]);
        }
        group_lexmin(tj, ij);
        const bool take = (tj < gt) | ((tj == gt) & (ij < gi));
        gt = take ? tj : gt;
        gi = take ? ij : gi;
      }
      node = (SHADOW && gi != target) ? kBvhDone : (sp > 0 ? (int)stk[--sp] : kBvhDone);
    }
    if (node == kBvhDone) break;
  }
#ifdef IPT_BVH_STATS
  if (j == 0) {
    atomicAdd(&g_bvh_stats[0], 1ull);
    atomicAdd(&g_bvh_stats[1], (unsigned long long)st_nodes);
    atomicAdd(&g_bvh_stats[2], (unsigned long long)st_leaves);
    if (SHADOW && gi != target) atomicAdd(&g_bvh_stats[3], 1ull);
  }
#endif
}

// Cooperative closest hit.  Called by ALL 64 lanes of the wave (convergent);
// lanes with `need` have their (bt, bi) continued through the tree
// lexicographically.  SHADOW: the lanes' entry bi is the target emitter; a
// group stops as soon as its bi is no longer the target (occluded).
template <bool SHADOW>
__device__ __forceinline__ void coop_cast(const CoopView &C, bool need, V3 p, V3 d, float &bt, int &bi) {
  const int lane = (int)__lane_id();
  const int g = lane >> 3;
  uint64_t M = __ballot(need);
#ifdef IPT_BVH_STATS
  if (M && lane == (int)__builtin_ctzll(__ballot(1))) atomicAdd(&g_bvh_stats[5], 1ull);
#endif
  while (M) {
#ifdef IPT_BVH_STATS
    if (lane == (int)__builtin_ctzll(__ballot(1))) atomicAdd(&g_bvh_stats[6], 1ull);
#endif
    uint64_t Mr = M;  // the first (up to) 8 rays: group k takes the k-th
    int src = -1;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (Mr) {
        const int idx = __builtin_ctzll(Mr);
        Mr &= Mr - 1;
        src = (g == k) ? idx : src;
      }
    }
    const uint64_t taken = M & ~Mr;
    M = Mr;
    const int sa = (src < 0 ? lane : src) << 2;
    const V3 gp = mk(bperm_f(sa, p.x), bperm_f(sa, p.y), bperm_f(sa, p.z));
    const V3 gd = mk(bperm_f(sa, d.x), bperm_f(sa, d.y), bperm_f(sa, d.z));
    float gt = bperm_f(sa, bt);
    int gi = __builtin_amdgcn_ds_bpermute(sa, bi);
    if (src >= 0) {
      coop_traverse<SHADOW>(C, gp, gd, gt, gi);
    }
    // results back to the owners: the ray of group k came from the k-th lane of `taken`
    const int ra = (8 * lane_rank64(taken)) << 2;
    const float rt = bperm_f(ra, gt);
    const int ri = __builtin_amdgcn_ds_bpermute(ra, gi);
    if ((taken >> lane) & 1ull) {
      bt = rt;
      bi = ri;
    }
  }
}

// Triangle::getNormal (scene_basics.h:100-109)
__device__ __forceinline__ V3 shading_normal(const TriGeom &g, V3 q) {
  if (g.flags & GEOM_AXIS_FLAT) return mk(g.vn[0][0], g.vn[0][1], g.vn[0][2]);  // exact, scene_layout.h
  const V3 v0 = mk(g.v[0][0], g.v[0][1], g.v[0][2]);
  const V3 v1 = mk(g.v[1][0], g.v[1][1], g.v[1][2]);
  const V3 v2 = mk(g.v[2][0], g.v[2][1], g.v[2][2]);
  const V3 c0 = cross3(sub(v1, q), sub(v2, q));
  const V3 c1 = cross3(sub(v2, q), sub(v0, q));
  const V3 c2 = cross3(sub(v0, q), sub(v1, q));
  const float w0 = (0.5f * sqrtf(dot3(c0, c0))) / g.area;
  const float w1 = (0.5f * sqrtf(dot3(c1, c1))) / g.area;
  const float w2 = (0.5f * sqrtf(dot3(c2, c2))) / g.area;
  const V3 n = mk(fmaf(g.vn[2][0], w2, fmaf(g.vn[1][0], w1, g.vn[0][0] * w0)),
                  fmaf(g.vn[2][1], w2, fmaf(g.vn[1][1], w1, g.vn[0][1] * w0)),
                  fmaf(g.vn[2][2], w2, fmaf(g.vn[1][2], w1, g.vn[0][2] * w0)));
  return unit(n);
}

// Camera ray (path_trace.cu:155-165) + Ray::transform (scene_basics.h:307-319)
// rcW / rcH: 1/W and 1/H when W and H are powers of two (then x * rcW == x / W
// exactly: a power-of-two scale of a normal float), else 0 (divide).
// org: the camera origin M * (0,0,0,1) = fma(M3, 1, fma(M2, 0, fma(M1, 0, M0 * 0)))
// per row, the same for every ray: evaluated once on the host with these
// operations (the launch arguments' cam_org) instead of per lane.
__device__ __forceinline__ void camera_ray(const float *cam, const float *org, Rng &st, int r, int c, int W, int H,
                                           float rcW, float rcH, V3 &p, V3 &d) {
  const float u0 = uniform(st), u1 = uniform(st);
  // (2(c+u0)) / W: numerator in [2^-32, 2W], W >= 1 -- in div_inrange's range.
  // d0 = (x, y, 1): x and y are 0 or multiples of 2^-24 (Sterbenz), n2 in
  // [1, 3] -- in unit_in_range's range.
  const float nx = 2.f * ((float)c + u0), ny = 2.f * ((float)r + u1);
  const float x = (rcW != 0.f ? nx * rcW : div_inrange(nx, (float)W)) - 1.f;
  const float y = 1.f - (rcH != 0.f ? ny * rcH : div_inrange(ny, (float)H));
  const V3 d0 = unit_in_range(mk(x, y, 1.f));
  float dr[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float *M = cam + 4 * i;
    dr[i] = fmaf(M[3], 0.f, fmaf(M[2], d0.z, fmaf(M[1], d0.y, M[0] * d0.x)));
  }
  p = mk(org[0], org[1], org[2]);
  d = unit(mk(dr[0], dr[1], dr[2]));
}

// Phong lobe of BSDF (path_trace.cu:19-22)
__device__ inline float phong(float shin, V3 nrm, V3 w, V3 wi) {
  const float dn = dot3(nrm, wi);
  const V3 refl = mk(fmaf(2.f * dn, nrm.x, -wi.x), fmaf(2.f * dn, nrm.y, -wi.y), fmaf(2.f * dn, nrm.z, -wi.z));
  const float pw = pow_f(dot3(refl, w), shin);
  const float mx = pw > 0.f ? pw : 0.f;
  return (float)((((double)(shin + 2.f)) / 2.0 / kPi) * (double)mx);
}

}  // namespace dev
}  // namespace ipt

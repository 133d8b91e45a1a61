// mm_numerics.h -- bit-exact float32 numerics of the reference's reprojection path.
//
// The reference (VTM-17.2 + MM extension) computes every reprojection in IEEE float32
// (`typedef float TCoord`, source/Lib/CommonLib/TypeDef.h:284) through two libraries
// that are not part of the reference tree:
//   * glibc 2.35 libm (scalar `std::sin/cos/acos/asin/atan/atan2/tan/sqrt/round` on float,
//     plus double `::sin/::cos` where TangentialMotionModel.cpp:27-28 calls them unqualified),
//   * Eigen 3.3.7 SSE packet math (`psin/pcos/psqrt<Packet4f>`) for array expressions whose
//     every operation has packet support.
// This header restates both, written once for host and device (`MM_HD`), so that the HIP
// kernels and any host code produce the same bits.  Each function names the algorithm it
// follows; tests/test_numerics.py + tools/check_numerics.cpp verify them exhaustively
// against this container's glibc (and the tabulated rsqrtps of the fixture CPU).
//
// Build rules that the bit-exactness depends on: `-ffp-contract=off`, no fast-math,
// correctly rounded f32 division and sqrt (hipcc default), f32 denormals preserved.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define MM_HD __host__ __device__ __forceinline__
#define MM_HD_CONST __device__ __constant__
// Rare paths (huge-argument reductions, double-double fallbacks, scalar libm for Eigen tail
// lanes).  Inlined: out-of-line calls measured slower than the instruction-cache misses they save
// (k_reproj_dev +10 us at C3).
#define MM_HD_COLD __host__ __device__ __forceinline__
#else
#define MM_HD inline
#define MM_HD_CONST static const
#define MM_HD_COLD inline
#endif

#include "mm_rsqrtps_table.h"

namespace mmnum {

// ------------------------------------------------------------------------------------------
// bit helpers
// ------------------------------------------------------------------------------------------
MM_HD uint32_t asu(float f) { return __builtin_bit_cast(uint32_t, f); }
MM_HD float asf(uint32_t u) { return __builtin_bit_cast(float, u); }
MM_HD uint64_t asu64(double d) { return __builtin_bit_cast(uint64_t, d); }
MM_HD double asd(uint64_t u) { return __builtin_bit_cast(double, u); }
MM_HD float fabsf_(float x) { return asf(asu(x) & 0x7fffffffu); }
MM_HD double fabs_d_(double x) { return __builtin_fabs(x); }
MM_HD double fabs_(double x) { return asd(asu64(x) & 0x7fffffffffffffffull); }
MM_HD bool isnanf_(float x) { return (asu(x) & 0x7fffffffu) > 0x7f800000u; }
MM_HD float sqrtf_(float x) { return __builtin_sqrtf(x); }   // IEEE correctly rounded
MM_HD double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

// ------------------------------------------------------------------------------------------
// Numerics modes: every belief about Eigen 3.3.7 that cannot be verified
// offline is a compile-time switch, defaulting to the belief.  tools/numerics_sensitivity.py
// builds the CPU twin in each alternative mode and counts what changes at C3.
//   MM_ROUND_MODE      0: std::round (ties away) for every element (A6 belief: cast<int> is not
//                         packet-enabled, so the whole rounding expression is scalar)
//                      1: packet elements use SSE4.1 pround (ties to even), tail elements std::round
//   MM_PROD3_MODE      0: 3x3 product coefficient p0 + (p1 + p2) (A7 belief)   1: (p0 + p1) + p2
//   MM_TAN_CENTRE_MODE 0: TAN centre terms via double ::sin / ::cos (A9)         1: float sinf / cosf
//   MM_PSQRT_EXACT     0: psqrt = rsqrtps + one Newton step (A3 EIGEN_FAST_MATH) 1: IEEE sqrt
// ------------------------------------------------------------------------------------------
#ifndef MM_ROUND_MODE
#define MM_ROUND_MODE 0
#endif
#ifndef MM_PROD3_MODE
#define MM_PROD3_MODE 0
#endif
#ifndef MM_TAN_CENTRE_MODE
#define MM_TAN_CENTRE_MODE 0
#endif

// std::round(float) == roundf: half-way cases away from zero (Eigen 3.3.7 round_impl with
// EIGEN_HAS_CXX11_MATH -> std::round; MVReprojection.cpp:163-164).
MM_HD float roundf_(float x) {
  uint32_t ix = asu(x);
  uint32_t ax = ix & 0x7fffffffu;
  if (ax >= 0x4b000000u) return x;                 // |x| >= 2^23 (or inf/nan): integral
  if (ax < 0x3f000000u) return asf(ix & 0x80000000u);  // |x| < 0.5 -> +-0
  int e = (int)(ax >> 23) - 127;                   // 0 <= e <= 22 here, or -1 for [0.5,1)
  if (e < 0) return asf((ix & 0x80000000u) | 0x3f800000u);  // [0.5,1) -> +-1
  uint32_t frac_mask = 0x007fffffu >> e;
  uint32_t half = 0x00400000u >> e;
  uint32_t r = (ix + half) & ~frac_mask;
  return asf(r);
}
// _mm_round_ps(x, _MM_FROUND_TO_NEAREST_INT): ties to even (MM_ROUND_MODE 1 packet lanes)
MM_HD float roundeven_(float x) { return __builtin_rintf(x); }

// ------------------------------------------------------------------------------------------
// glibc 2.35 sinf / cosf  (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h,
// sincosf_poly/reduce_fast/reduce_large; the x86_64 IFUNC selects the -mfma build on FMA
// CPUs, whose GCC contraction turns every `a + b*c` below into one fused multiply-add).
// ------------------------------------------------------------------------------------------
#ifndef MM_SINCOSF_FMA
#define MM_SINCOSF_FMA 1
#endif
MM_HD double mad_(double a, double b, double c) {
#if MM_SINCOSF_FMA
  return fma_(a, b, c);
#else
  return a * b + c;
#endif
}

// abstop12: top 12 bits of |x| (sign dropped)
MM_HD uint32_t abstop12_(float x) { return (asu(x) >> 20) & 0x7ff; }

struct SinCosfC {
  static constexpr double hpi_inv = 0x1.45F306DC9C883p+23;   // 2/pi * 2^24 (!TOINT_INTRINSICS)
  static constexpr double hpi = 0x1.921FB54442D18p0;
  static constexpr double c0 = 0x1p0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5,
                          c3 = -0x1.6c087e89a359dp-10, c4 = 0x1.99343027bf8c3p-16;
  static constexpr double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7,
                          s3 = -0x1.994eb3774cf24p-13;
  static constexpr double pi63 = 0x1.921FB54442D18p-62;
};

// sinf_poly with table 0 coefficients; `neg_cos` reproduces table 1 (all cosine
// coefficients negated -> the fused evaluation is exactly the negation).
MM_HD float sincosf_poly_(double x, double x2, int n, bool neg_cos) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = mad_(x2, SinCosfC::s3, SinCosfC::s2);
    double x7 = x3 * x2;
    double s = mad_(x3, SinCosfC::s1, x);
    return (float)mad_(x7, s1, s);
  } else {
    double x4 = x2 * x2;
    double c2 = mad_(x2, SinCosfC::c4, SinCosfC::c3);
    double c1 = mad_(x2, SinCosfC::c1, SinCosfC::c0);
    double x6 = x4 * x2;
    double c = mad_(x4, SinCosfC::c2, c1);
    double r = mad_(x6, c2, c);
    return (float)(neg_cos ? -r : r);
  }
}

MM_HD double reduce_fast_(double x, int* np) {
  double r = x * SinCosfC::hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
#if MM_SINCOSF_FMA
  return fma_(-(double)n, SinCosfC::hpi, x);
#else
  return x - (double)n * SinCosfC::hpi;
#endif
}

// 4/pi bits (glibc sysdeps/ieee754/flt-32/s_sincosf_data.c __inv_pio4)
// (entry i is bits 8*(i-3) .. 8*i+31 of 2/pi's fraction; written as a switch so that no
// per-thread table is materialised)
MM_HD uint32_t inv_pio4_(int i) {
  switch (i) {
    case 0: return 0xa2u;          case 1: return 0xa2f9u;        case 2: return 0xa2f983u;
    case 3: return 0xa2f9836eu;    case 4: return 0xf9836e4eu;    case 5: return 0x836e4e44u;
    case 6: return 0x6e4e4415u;    case 7: return 0x4e441529u;    case 8: return 0x441529fcu;
    case 9: return 0x1529fc27u;    case 10: return 0x29fc2757u;   case 11: return 0xfc2757d1u;
    case 12: return 0x2757d1f5u;   case 13: return 0x57d1f534u;   case 14: return 0xd1f534ddu;
    case 15: return 0xf534ddc0u;   case 16: return 0x34ddc0dbu;   case 17: return 0xddc0db62u;
    case 18: return 0xc0db6295u;   case 19: return 0xdb629599u;   case 20: return 0x6295993cu;
    case 21: return 0x95993c43u;   case 22: return 0x993c4390u;   default: return 0x3c439041u;
  }
}

MM_HD_COLD double reduce_large_(uint32_t xi, int* np) {
  int idx = (xi >> 26) & 15;
  int shift = (xi >> 23) & 7;
  uint64_t n, res0, res1, res2;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  res0 = (uint32_t)(xi * inv_pio4_(idx));
  res1 = (uint64_t)xi * inv_pio4_(idx + 4);
  res2 = (uint64_t)xi * inv_pio4_(idx + 8);
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * SinCosfC::pi63;
}

MM_HD float g_sinf(float y) {
  double x = y;
  int n;
  const uint32_t top = abstop12_(y);
  if (top < abstop12_(0x1.921FB6p-1f)) {
    double s = x * x;
    if (top < abstop12_(0x1p-12f)) return y;
    return sincosf_poly_(x, s, 0, false);
  } else if (top < abstop12_(120.0f)) {
    x = reduce_fast_(x, &n);
    double s = ((n & 3) == 0 || (n & 3) == 3) ? 1.0 : -1.0;
    return sincosf_poly_(x * s, x * x, n, (n & 2) != 0);
  } else if (top < abstop12_(__builtin_inff())) {
    uint32_t xi = asu(y);
    int sign = xi >> 31;
    x = reduce_large_(xi, &n);
    int q = (n + sign) & 3;
    double s = (q == 0 || q == 3) ? 1.0 : -1.0;
    return sincosf_poly_(x * s, x * x, n, ((n + sign) & 2) != 0);
  }
  return (y - y) / (y - y);
}

MM_HD float g_cosf(float y) {
  double x = y;
  int n;
  const uint32_t top = abstop12_(y);
  if (top < abstop12_(0x1.921FB6p-1f)) {
    double x2 = x * x;
    if (top < abstop12_(0x1p-12f)) return 1.0f;
    return sincosf_poly_(x, x2, 1, false);
  } else if (top < abstop12_(120.0f)) {
    x = reduce_fast_(x, &n);
    double s = ((n & 3) == 0 || (n & 3) == 3) ? 1.0 : -1.0;
    return sincosf_poly_(x * s, x * x, n ^ 1, (n & 2) != 0);
  } else if (top < abstop12_(__builtin_inff())) {
    uint32_t xi = asu(y);
    int sign = xi >> 31;
    x = reduce_large_(xi, &n);
    int q = (n + sign) & 3;
    double s = (q == 0 || q == 3) ? 1.0 : -1.0;
    return sincosf_poly_(x * s, x * x, n ^ 1, ((n + sign) & 2) != 0);
  }
  return (y - y) / (y - y);
}

// ------------------------------------------------------------------------------------------
// glibc 2.35 atanf (sysdeps/ieee754/flt-32/s_atanf.c, fdlibm float)
// ------------------------------------------------------------------------------------------
MM_HD float g_atanf(float x) {
  const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f, atanhi2 = 9.8279368877e-01f,
              atanhi3 = 1.5707962513e+00f;
  const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f, atanlo2 = 3.4473217170e-08f,
              atanlo3 = 7.5497894159e-08f;
  const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
              aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
              aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
              aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
  const float one = 1.0f;
  float w, s1, s2, z;
  int32_t ix, hx, id;
  hx = (int32_t)asu(x);
  ix = hx & 0x7fffffff;
  if (ix >= 0x4c000000) {  // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;
    if (hx > 0) return atanhi3 + atanlo3;
    return -atanhi3 - atanlo3;
  }
  if (ix < 0x3ee00000) {  // |x| < 0.4375
    if (ix < 0x31000000) return x;  // |x| < 2^-29
    id = -1;
  } else {
    x = fabsf_(x);
    if (ix < 0x3f980000) {    // |x| < 1.1875
      if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
        id = 0;
        x = (2.0f * x - one) / (2.0f + x);
      } else {  // 11/16 <= |x| < 19/16
        id = 1;
        x = (x - one) / (x + one);
      }
    } else {
      if (ix < 0x401c0000) {  // |x| < 2.4375
        id = 2;
        x = (x - 1.5f) / (one + 1.5f * x);
      } else {
        id = 3;
        x = -1.0f / x;
      }
    }
  }
  z = x * x;
  w = z * z;
  s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return (hx < 0) ? -z : z;
}

MM_HD_COLD float g_atanf_cold(float x) { return g_atanf(x); }

// glibc 2.35 atan2f (sysdeps/ieee754/flt-32/e_atan2f.c)
MM_HD float g_atan2f(float y, float x) {
  const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
              pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
  float z;
  int32_t k, m, hx, hy, ix, iy;
  hx = (int32_t)asu(x);
  ix = hx & 0x7fffffff;
  hy = (int32_t)asu(y);
  iy = hy & 0x7fffffff;
  if ((ix > 0x7f800000) || (iy > 0x7f800000)) return x + y;
  if (hx == 0x3f800000) return g_atanf_cold(y);  // x == 1
  m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    } else {
      switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
      }
    }
  }
  if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  k = (iy - ix) >> 23;
  if (k > 60)
    z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60)
    z = 0.0f;
  else
    z = g_atanf(fabsf_(y / x));
  switch (m) {
    case 0: return z;
    case 1: return asf(asu(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// glibc 2.35 acosf (sysdeps/ieee754/flt-32/e_acosf.c, fdlibm float; constants checked
// against libm.so.6 .rodata)
MM_HD float g_acosf(float x) {
  const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f,
              pio2_lo = 7.5497894159e-08f, pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f,
              pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f,
              pS5 = 3.4793309169e-05f, qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f,
              qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
  float z, p, q, r, w, s, c, df;
  int32_t hx, ix;
  hx = (int32_t)asu(x);
  ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) {
    if (hx > 0) return 0.0f;
    return pi + 2.0f * pio2_lo;
  } else if (ix > 0x3f800000) {
    return (x - x) / (x - x);
  }
  if (ix < 0x3f000000) {
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;
    z = x * x;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  } else if (hx < 0) {
    z = (one + x) * 0.5f;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    s = sqrtf_(z);
    r = p / q;
    w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  } else {
    z = (one - x) * 0.5f;
    s = sqrtf_(z);
    df = asf(asu(s) & 0xfffff000u);
    c = (z - df * df) / (s + df);
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    w = r * s + c;
    return 2.0f * (df + w);
  }
}

// glibc 2.35 asinf (sysdeps/ieee754/flt-32/e_asinf.c, Shimizu's float variant)
MM_HD float g_asinf(float x) {
  const float one = 1.0f, huge = 1.000e+30f, pio2_hi = 1.57079637050628662109375f,
              pio2_lo = -4.37113900018624283e-8f, pio4_hi = 0.785398185253143310546875f,
              p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f,
              p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
  float t, w, p, q, c, r, s;
  int32_t hx, ix;
  hx = (int32_t)asu(x);
  ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) {
    return x * pio2_hi + x * pio2_lo;
  } else if (ix > 0x3f800000) {
    return (x - x) / (x - x);
  } else if (ix < 0x3f000000) {
    if (ix < 0x32000000) {
      if (huge + x > one) return x;
    } else {
      t = x * x;
      w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
      return x + x * w;
    }
  }
  w = one - fabsf_(x);
  t = w * 0.5f;
  p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
  s = sqrtf_(t);
  if (ix >= 0x3F79999A) {
    t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
  } else {
    w = asf(asu(s) & 0xfffff000u);
    c = (t - w * w) / (s + w);
    r = p;
    p = 2.0f * s * r - (pio2_lo - 2.0f * c);
    q = pio4_hi - 2.0f * w;
    t = pio4_hi - (p - q);
  }
  return (hx > 0) ? t : -t;
}

// glibc 2.35 tanf (sysdeps/ieee754/flt-32/s_tanf.c + k_tanf.c + e_rem_pio2f.c, fdlibm float).
// Only the |x| <= 2^7*pi/2 reduction is restated: the reference evaluates tanf on polar
// angles theta in [0, pi] (Projection.cpp:198, PerspectiveProjection::radius).
MM_HD float g_kernel_tanf(float x, float y, int iy) {
  const float one = 1.0f, pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
  const float T0 = 3.3333334327e-01f, T1 = 1.3333334029e-01f, T2 = 5.3968254477e-02f,
              T3 = 2.1869488060e-02f, T4 = 8.8632395491e-03f, T5 = 3.5920790397e-03f,
              T6 = 1.4562094584e-03f, T7 = 5.8804126456e-04f, T8 = 2.4646313977e-04f,
              T9 = 7.8179444245e-05f, T10 = 7.1407252108e-05f, T11 = -1.8558637748e-05f,
              T12 = 2.5907305826e-05f;
  float z, r, v, w, s;
  int32_t ix, hx;
  hx = (int32_t)asu(x);
  ix = hx & 0x7fffffff;
  if (ix < 0x39000000) {  // |x| < 2^-13 (glibc k_tanf.c; checked in libm.so.6)
    if ((int)x == 0) {
      if ((ix | (iy + 1)) == 0) return one / fabsf_(x);
      if (iy == 1) return x;
      return -one / x;
    }
  }
  if (ix >= 0x3f2ca140) {  // |x| >= 0.6744
    if (hx < 0) {
      x = -x;
      y = -y;
    }
    z = pio4 - x;
    w = pio4lo - y;
    x = z + w;
    y = 0.0f;
    if (fabsf_(x) < 0x1p-13f) return (float)(1 - ((hx >> 30) & 2)) * iy * (1.0f - 2 * iy * x);
  }
  z = x * x;
  w = z * z;
  r = T1 + w * (T3 + w * (T5 + w * (T7 + w * (T9 + w * T11))));
  v = z * (T2 + w * (T4 + w * (T6 + w * (T8 + w * (T10 + w * T12)))));
  s = z * x;
  r = y + z * (s * (r + v) + y);
  r += T0 * s;
  w = x + r;
  if (ix >= 0x3f2ca140) {
    v = (float)iy;
    return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
  }
  if (iy == 1) return w;
  {
    float a, t;
    z = asf(asu(w) & 0xfffff000u);
    v = r - (z - x);
    t = a = -1.0f / w;
    t = asf(asu(t) & 0xfffff000u);
    s = 1.0f + t * z;
    return t + a * (s + t * v);
  }
}

// tanf's reduction in glibc 2.35 (s_tanf.c rem_pio2f): the sincosf reduce_fast/reduce_large in
// double, compiled without FMA (tanf is not an IFUNC), split into a float high/low pair.
MM_HD int g_rem_pio2f(float x, float* y) {
  double dx = x;
  int n;
  if (abstop12_(x) < abstop12_(120.0f)) {
    double r = dx * SinCosfC::hpi_inv;
    n = ((int32_t)r + 0x800000) >> 24;
    dx = dx - (double)n * SinCosfC::hpi;
  } else {
    uint32_t xi = asu(x);
    int sign = xi >> 31;
    dx = reduce_large_(xi, &n);
    dx = sign ? -dx : dx;
  }
  y[0] = (float)dx;
  y[1] = (float)(dx - (double)y[0]);
  return n;
}

MM_HD float g_tanf(float x) {
  float y[2], z = 0.0f;
  int32_t n, ix;
  ix = (int32_t)asu(x) & 0x7fffffff;
  if (ix <= 0x3f490fda) return g_kernel_tanf(x, z, 1);
  if (ix >= 0x7f800000) return x - x;
  n = g_rem_pio2f(x, y);
  return g_kernel_tanf(y[0], y[1], 1 - ((n & 1) << 1));
}

// ------------------------------------------------------------------------------------------
// float(::sin((double)x)) and float(::cos((double)x)) for float x: glibc's double sin/cos
// (IBM accurate library, < 0.55 ulp) rounded to float.  TangentialMotionModel.cpp:27-28,38,40
// call the unqualified double functions on float block-centre angles.  Restated as
// a double-double evaluation rounded to the nearest double, then to float; equality with glibc
// is verified over every float in [-4, 4] (tools/check_numerics.cpp).
// ------------------------------------------------------------------------------------------
struct dd_ { double hi, lo; };
MM_HD dd_ two_sum_(double a, double b) {
  double s = a + b;
  double bb = s - a;
  double err = (a - (s - bb)) + (b - bb);
  return {s, err};
}
MM_HD dd_ two_prod_(double a, double b) {
  double p = a * b;
  return {p, fma_(a, b, -p)};
}
MM_HD dd_ dd_add_(dd_ a, dd_ b) {
  dd_ s = two_sum_(a.hi, b.hi);
  dd_ t = two_sum_(a.lo, b.lo);
  s.lo += t.hi;
  s = two_sum_(s.hi, s.lo);
  s.lo += t.lo;
  return two_sum_(s.hi, s.lo);
}
MM_HD dd_ dd_mul_(dd_ a, dd_ b) {
  dd_ p = two_prod_(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return two_sum_(p.hi, p.lo);
}
MM_HD dd_ dd_mul_d_(dd_ a, double b) {
  dd_ p = two_prod_(a.hi, b);
  p.lo += a.lo * b;
  return two_sum_(p.hi, p.lo);
}
// Taylor series of sin/cos around 0 in double-double; |r| <= 0.8
MM_HD dd_ dd_sin_small_(dd_ r) {
  dd_ r2 = dd_mul_(r, r);
  dd_ term = r, sum = r;
  for (int k = 1; k <= 13; k++) {
    term = dd_mul_(term, r2);
    double den = (double)((2 * k) * (2 * k + 1));
    // term /= -den  (exact enough in dd: divide hi, correct lo)
    double q1 = term.hi / den;
    dd_ pr = two_prod_(q1, den);
    double q2 = ((term.hi - pr.hi) - pr.lo + term.lo) / den;
    term = two_sum_(-q1, -q2);
    sum = dd_add_(sum, term);
  }
  return sum;
}
MM_HD dd_ dd_cos_small_(dd_ r) {
  dd_ r2 = dd_mul_(r, r);
  dd_ term = {1.0, 0.0}, sum = {1.0, 0.0};
  for (int k = 1; k <= 13; k++) {
    term = dd_mul_(term, r2);
    double den = (double)((2 * k - 1) * (2 * k));
    double q1 = term.hi / den;
    dd_ pr = two_prod_(q1, den);
    double q2 = ((term.hi - pr.hi) - pr.lo + term.lo) / den;
    term = two_sum_(-q1, -q2);
    sum = dd_add_(sum, term);
  }
  return sum;
}
// quadrant reduction by pi/2 in triple-double precision (|x| < 2^20)
MM_HD dd_ dd_reduce_pio2_(double x, int* q) {
  const double pio2_1 = 0x1.921fb54442d18p0, pio2_2 = 0x1.1a62633145c07p-54,
               pio2_3 = -0x1.f1976b7ed8fbcp-110;
  double k = __builtin_rint(x * 0x1.45f306dc9c883p-1);
  *q = (int)k;
  dd_ a = two_prod_(-k, pio2_1);
  dd_ b = two_prod_(-k, pio2_2);
  dd_ s = dd_add_({x, 0.0}, a);
  s = dd_add_(s, b);
  s = dd_add_(s, {-k * pio2_3, 0.0});
  return s;
}
MM_HD_COLD float sinf_via_double_dd(float xf) {
  double x = xf;
  if (xf == 0.0f) return xf;
  int q;
  dd_ r = dd_reduce_pio2_(x, &q);
  dd_ v;
  switch (q & 3) {
    case 0: v = dd_sin_small_(r); break;
    case 1: v = dd_cos_small_(r); break;
    case 2: v = dd_sin_small_(r); v.hi = -v.hi; v.lo = -v.lo; break;
    default: v = dd_cos_small_(r); v.hi = -v.hi; v.lo = -v.lo; break;
  }
  return (float)(v.hi + v.lo);
}
MM_HD_COLD float cosf_via_double_dd(float xf) {
  double x = xf;
  int q;
  dd_ r = dd_reduce_pio2_(x, &q);
  dd_ v;
  switch (q & 3) {
    case 0: v = dd_cos_small_(r); break;
    case 1: v = dd_sin_small_(r); v.hi = -v.hi; v.lo = -v.lo; break;
    case 2: v = dd_cos_small_(r); v.hi = -v.hi; v.lo = -v.lo; break;
    default: v = dd_sin_small_(r); break;
  }
  return (float)(v.hi + v.lo);
}

// Fast path: plain-double sin/cos (Cody-Waite pi/2 reduction with FMA, Taylor polynomials in
// Horner form, a few double ulps) rounded to float.  glibc's double result is within a few
// double ulps of it, so both round to the same float unless the value lies near a float
// rounding midpoint; those (rare) inputs take the double-double path above.  The combination is
// checked against glibc over every float in [-4, 4] (tools/check_numerics.cpp); TAN's angles
// epsC = pi/2 - thetaC lie in [-pi/2, pi/2].
MM_HD double d_sin_poly_(double r) {
  const double z = r * r;
  double p = 1.0 / 121645100408832000.0;          // 1/19!  (|r| <= pi/4 + eps: next term < 2^-60)
  p = fma_(p, -z, 1.0 / 355687428096000.0);       // 1/17!
  p = fma_(p, -z, 1.0 / 1307674368000.0);         // 1/15!
  p = fma_(p, -z, 1.0 / 6227020800.0);            // 1/13!
  p = fma_(p, -z, 1.0 / 39916800.0);              // 1/11!
  p = fma_(p, -z, 1.0 / 362880.0);                // 1/9!
  p = fma_(p, -z, 1.0 / 5040.0);                  // 1/7!
  p = fma_(p, -z, 1.0 / 120.0);                   // 1/5!
  p = fma_(p, -z, 1.0 / 6.0);                     // 1/3!
  return fma_(-r * z, p, r);
}
MM_HD double d_cos_poly_(double r) {
  const double z = r * r;
  double p = 1.0 / 2432902008176640000.0;         // 1/20!
  p = fma_(p, -z, 1.0 / 6402373705728000.0);      // 1/18!
  p = fma_(p, -z, 1.0 / 20922789888000.0);        // 1/16!
  p = fma_(p, -z, 1.0 / 87178291200.0);           // 1/14!
  p = fma_(p, -z, 1.0 / 479001600.0);             // 1/12!
  p = fma_(p, -z, 1.0 / 3628800.0);               // 1/10!
  p = fma_(p, -z, 1.0 / 40320.0);                 // 1/8!
  p = fma_(p, -z, 1.0 / 720.0);                   // 1/6!
  p = fma_(p, -z, 1.0 / 24.0);                    // 1/4!
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + z * z * p);
}
// true when RN_float(v) is the same for every double within 2^-48 |v| of v
MM_HD bool float_rounding_robust_(double v, float f) {
  const uint32_t b = asu(f);
  const double up = (double)asf(b + 1u), dn = (double)asf(b - 1u);
  const double mid_hi = ((double)f + up) * 0.5, mid_lo = ((double)f + dn) * 0.5;
  const double tol = fabs_d_(v) * 0x1p-48;
  return fabs_d_(v - mid_hi) > tol && fabs_d_(v - mid_lo) > tol;
}
MM_HD double d_reduce_pio2_fast_(double x, int* q) {
  const double pio2_1 = 0x1.921fb54442d18p0, pio2_2 = 0x1.1a62633145c07p-54;
  const double k = __builtin_rint(x * 0x1.45f306dc9c883p-1);
  *q = (int)k;
  return fma_(-k, pio2_2, fma_(-k, pio2_1, x));
}
MM_HD float sinf_via_double(float xf) {
  if (xf == 0.0f) return xf;
  int q;
  const double r = d_reduce_pio2_fast_((double)xf, &q);
  double v = (q & 1) ? d_cos_poly_(r) : d_sin_poly_(r);
  if (q & 2) v = -v;
  const float f = (float)v;
  return (f != 0.0f && float_rounding_robust_(v, f)) ? f : sinf_via_double_dd(xf);
}
MM_HD float cosf_via_double(float xf) {
  int q;
  const double r = d_reduce_pio2_fast_((double)xf, &q);
  double v = (q & 1) ? d_sin_poly_(r) : d_cos_poly_(r);
  if ((q + 1) & 2) v = -v;
  const float f = (float)v;
  return (f != 0.0f && float_rounding_robust_(v, f)) ? f : cosf_via_double_dd(xf);
}

// ------------------------------------------------------------------------------------------
// Eigen 3.3.7 SSE packet math (Eigen/src/Core/arch/SSE/MathFunctions.h), one lane.
// SURVEY.md Appendix C.  pmadd(a,b,c) = a*b + c with two roundings (SSE4.1, no FMA).
// ------------------------------------------------------------------------------------------
MM_HD int32_t cvttps_(float y) {  // _mm_cvttps_epi32: out-of-range/NaN -> INT_MIN
  if (!(fabsf_(y) < 2147483648.0f)) return (int32_t)0x80000000u;
  return (int32_t)y;
}

MM_HD float e_psin(float xin) {
  uint32_t sign_bit = asu(xin) & 0x80000000u;
  float x = fabsf_(xin);
  float y = x * 1.27323954473516f;
  int32_t emm2 = cvttps_(y);
  emm2 = (int32_t)(((uint32_t)emm2 + 1u) & ~1u);
  y = (float)emm2;
  uint32_t emm0 = ((uint32_t)emm2 & 4u) << 29;
  bool poly_sin = ((uint32_t)emm2 & 2u) == 0;
  sign_bit ^= emm0;
  float xmm1 = y * -0.78515625f;
  float xmm2 = y * -2.4187564849853515625e-4f;
  float xmm3 = y * -3.77489497744594108e-8f;
  x = x + xmm1;
  x = x + xmm2;
  x = x + xmm3;
  float z = x * x;
  float yc = 2.443315711809948E-005f;
  yc = yc * z + -1.388731625493765E-003f;
  yc = yc * z + 4.166664568298827E-002f;
  yc = yc * z;
  yc = yc * z;
  float tmp = z * 0.5f;
  yc = yc - tmp;
  yc = yc + 1.0f;
  float y2 = -1.9515295891E-4f;
  y2 = y2 * z + 8.3321608736E-3f;
  y2 = y2 * z + -1.6666654611E-1f;
  y2 = y2 * z;
  y2 = y2 * x;
  y2 = y2 + x;
  float r = poly_sin ? y2 : yc;
  return asf(asu(r) ^ sign_bit);
}

MM_HD float e_pcos(float xin) {
  float x = fabsf_(xin);
  float y = x * 1.27323954473516f;
  int32_t emm2 = cvttps_(y);
  emm2 = (int32_t)(((uint32_t)emm2 + 1u) & ~1u);
  y = (float)emm2;
  emm2 = (int32_t)((uint32_t)emm2 - 2u);
  uint32_t emm0 = (~(uint32_t)emm2 & 4u) << 29;
  bool poly_sin = ((uint32_t)emm2 & 2u) == 0;
  uint32_t sign_bit = emm0;
  float xmm1 = y * -0.78515625f;
  float xmm2 = y * -2.4187564849853515625e-4f;
  float xmm3 = y * -3.77489497744594108e-8f;
  x = x + xmm1;
  x = x + xmm2;
  x = x + xmm3;
  float z = x * x;
  float yc = 2.443315711809948E-005f;
  yc = yc * z + -1.388731625493765E-003f;
  yc = yc * z + 4.166664568298827E-002f;
  yc = yc * z;
  yc = yc * z;
  float tmp = z * 0.5f;
  yc = yc - tmp;
  yc = yc + 1.0f;
  float y2 = -1.9515295891E-4f;
  y2 = y2 * z + 8.3321608736E-3f;
  y2 = y2 * z + -1.6666654611E-1f;
  y2 = y2 * z;
  y2 = y2 * x + x;
  float r = poly_sin ? y2 : yc;
  return asf(asu(r) ^ sign_bit);
}

// _mm_rsqrt_ps of the fixture CPU (tabulated by tools/gen_rsqrtps_table.c)
MM_HD float rsqrtps_(float x) {
  uint32_t ix = asu(x);
  uint32_t ax = ix & 0x7fffffffu;
  if (ax > 0x7f800000u) return asf(ix | 0x00400000u);        // NaN -> quiet NaN
  if (ax < 0x00800000u) return asf((ix & 0x80000000u) | 0x7f800000u);  // +-0, denormal -> +-inf
  if (ix & 0x80000000u) return asf(0xffc00000u);               // negative -> default NaN
  if (ax == 0x7f800000u) return 0.0f;                           // +inf -> +0
  int e = (int)(ax >> 23) - 127;
  int half = (e >= 0) ? e / 2 : -((-e + 1) / 2);
  return asf(((uint32_t)(126 - half) << 23) | MM_RSQRTPS_MANT[e & 1][(ax >> 13) & 1023]);
}

#ifndef MM_PSQRT_EXACT
#define MM_PSQRT_EXACT 0
#endif
// psqrt<Packet4f> under EIGEN_FAST_MATH: rsqrt + one Newton step, denormal inputs -> 0
MM_HD float e_psqrt(float x) {
#if MM_PSQRT_EXACT
  return sqrtf_(x);
#else
  float half = x * 0.5f;
  bool denorm = (x >= 0.0f) && (x < 1.17549435e-38f);
  float r = rsqrtps_(x);
  r = r * (1.5f - half * (r * r));
  float res = x * r;
  return denorm ? 0.0f : res;
#endif
}

// Packet-or-scalar selection (Eigen LinearVectorizedTraversal on a 16-byte aligned
// destination: elements [0, n - n%4) use packets, the tail uses the scalar functors).
// Scalar sinf/cosf of an Eigen tail lane (out of line: tail lanes are rare, call sites many)
MM_HD_COLD float g_sinf_tail(float x) { return g_sinf(x); }
MM_HD_COLD float g_cosf_tail(float x) { return g_cosf(x); }
struct Math {
  int packet;  // int, not bool: an i1 member defeats SROA and lands in LDS
  MM_HD float sin(float x) const { return packet ? e_psin(x) : g_sinf_tail(x); }
  MM_HD float cos(float x) const { return packet ? e_pcos(x) : g_cosf_tail(x); }
  MM_HD float sqrt(float x) const { return packet ? e_psqrt(x) : sqrtf_(x); }
};
MM_HD bool packet_lane(int index, int n) { return index < n - (n & 3); }

}  // namespace mmnum

// Exhaustive check of csrc/mm_numerics.h against this container's glibc 2.35 libm and
// against Eigen-3.3.7-style SSE intrinsic kernels (psin/pcos/psqrt) executed natively.
//
//   g++ -O2 -std=c++17 -mfma -msse4.1 -ffp-contract=off -fopenmp \
//       -I vvc-extension-mm_amd/csrc tools/check_numerics.cpp -o /tmp/check_numerics -lm
//   /tmp/check_numerics [quick]
//
// Prints one line per function: name, inputs tested, mismatches.  Exit status 1 on any
// mismatch.  "quick" tests a 1/64 stride instead of every float.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>
#include <omp.h>
#include <random>
#include "mm_numerics.h"

using namespace mmnum;

static bool same(float a, float b) {
  if (std::isnan(a) && std::isnan(b)) return true;
  return asu(a) == asu(b);
}

// ---- Eigen 3.3.7 SSE kernels written with the intrinsics (reference for e_psin/...) ----
static __m128 sse_psin(__m128 x) {
  const __m128 p1 = _mm_set1_ps(1.0f), half = _mm_set1_ps(0.5f);
  const __m128i i1 = _mm_set1_epi32(1), inot1 = _mm_set1_epi32(~1), i2 = _mm_set1_epi32(2),
                i4 = _mm_set1_epi32(4);
  const __m128 sign_mask = _mm_castsi128_ps(_mm_set1_epi32(0x80000000));
  __m128 sign_bit = x;
  x = _mm_and_ps(x, _mm_castsi128_ps(_mm_set1_epi32(0x7fffffff)));
  sign_bit = _mm_and_ps(sign_bit, sign_mask);
  __m128 y = _mm_mul_ps(x, _mm_set1_ps(1.27323954473516f));
  __m128i emm2 = _mm_cvttps_epi32(y);
  emm2 = _mm_add_epi32(emm2, i1);
  emm2 = _mm_and_si128(emm2, inot1);
  y = _mm_cvtepi32_ps(emm2);
  __m128i emm0 = _mm_and_si128(emm2, i4);
  emm0 = _mm_slli_epi32(emm0, 29);
  emm2 = _mm_and_si128(emm2, i2);
  emm2 = _mm_cmpeq_epi32(emm2, _mm_setzero_si128());
  __m128 swap_sign_bit = _mm_castsi128_ps(emm0);
  __m128 poly_mask = _mm_castsi128_ps(emm2);
  sign_bit = _mm_xor_ps(sign_bit, swap_sign_bit);
  __m128 xmm1 = _mm_mul_ps(y, _mm_set1_ps(-0.78515625f));
  __m128 xmm2 = _mm_mul_ps(y, _mm_set1_ps(-2.4187564849853515625e-4f));
  __m128 xmm3 = _mm_mul_ps(y, _mm_set1_ps(-3.77489497744594108e-8f));
  x = _mm_add_ps(x, xmm1);
  x = _mm_add_ps(x, xmm2);
  x = _mm_add_ps(x, xmm3);
  y = _mm_set1_ps(2.443315711809948E-005f);
  __m128 z = _mm_mul_ps(x, x);
  y = _mm_add_ps(_mm_mul_ps(y, z), _mm_set1_ps(-1.388731625493765E-003f));
  y = _mm_add_ps(_mm_mul_ps(y, z), _mm_set1_ps(4.166664568298827E-002f));
  y = _mm_mul_ps(y, z);
  y = _mm_mul_ps(y, z);
  __m128 tmp = _mm_mul_ps(z, half);
  y = _mm_sub_ps(y, tmp);
  y = _mm_add_ps(y, p1);
  __m128 y2 = _mm_set1_ps(-1.9515295891E-4f);
  y2 = _mm_add_ps(_mm_mul_ps(y2, z), _mm_set1_ps(8.3321608736E-3f));
  y2 = _mm_add_ps(_mm_mul_ps(y2, z), _mm_set1_ps(-1.6666654611E-1f));
  y2 = _mm_mul_ps(y2, z);
  y2 = _mm_mul_ps(y2, x);
  y2 = _mm_add_ps(y2, x);
  y2 = _mm_and_ps(poly_mask, y2);
  y = _mm_andnot_ps(poly_mask, y);
  y = _mm_or_ps(y, y2);
  return _mm_xor_ps(y, sign_bit);
}
static __m128 sse_pcos(__m128 x) {
  const __m128 p1 = _mm_set1_ps(1.0f), half = _mm_set1_ps(0.5f);
  const __m128i i1 = _mm_set1_epi32(1), inot1 = _mm_set1_epi32(~1), i2 = _mm_set1_epi32(2),
                i4 = _mm_set1_epi32(4);
  x = _mm_and_ps(x, _mm_castsi128_ps(_mm_set1_epi32(0x7fffffff)));
  __m128 y = _mm_mul_ps(x, _mm_set1_ps(1.27323954473516f));
  __m128i emm2 = _mm_cvttps_epi32(y);
  emm2 = _mm_add_epi32(emm2, i1);
  emm2 = _mm_and_si128(emm2, inot1);
  y = _mm_cvtepi32_ps(emm2);
  emm2 = _mm_sub_epi32(emm2, i2);
  __m128i emm0 = _mm_andnot_si128(emm2, i4);
  emm0 = _mm_slli_epi32(emm0, 29);
  emm2 = _mm_and_si128(emm2, i2);
  emm2 = _mm_cmpeq_epi32(emm2, _mm_setzero_si128());
  __m128 sign_bit = _mm_castsi128_ps(emm0);
  __m128 poly_mask = _mm_castsi128_ps(emm2);
  __m128 xmm1 = _mm_mul_ps(y, _mm_set1_ps(-0.78515625f));
  __m128 xmm2 = _mm_mul_ps(y, _mm_set1_ps(-2.4187564849853515625e-4f));
  __m128 xmm3 = _mm_mul_ps(y, _mm_set1_ps(-3.77489497744594108e-8f));
  x = _mm_add_ps(x, xmm1);
  x = _mm_add_ps(x, xmm2);
  x = _mm_add_ps(x, xmm3);
  y = _mm_set1_ps(2.443315711809948E-005f);
  __m128 z = _mm_mul_ps(x, x);
  y = _mm_add_ps(_mm_mul_ps(y, z), _mm_set1_ps(-1.388731625493765E-003f));
  y = _mm_add_ps(_mm_mul_ps(y, z), _mm_set1_ps(4.166664568298827E-002f));
  y = _mm_mul_ps(y, z);
  y = _mm_mul_ps(y, z);
  __m128 tmp = _mm_mul_ps(z, half);
  y = _mm_sub_ps(y, tmp);
  y = _mm_add_ps(y, p1);
  __m128 y2 = _mm_set1_ps(-1.9515295891E-4f);
  y2 = _mm_add_ps(_mm_mul_ps(y2, z), _mm_set1_ps(8.3321608736E-3f));
  y2 = _mm_add_ps(_mm_mul_ps(y2, z), _mm_set1_ps(-1.6666654611E-1f));
  y2 = _mm_mul_ps(y2, z);
  y2 = _mm_add_ps(_mm_mul_ps(y2, x), x);
  y2 = _mm_and_ps(poly_mask, y2);
  y = _mm_andnot_ps(poly_mask, y);
  y = _mm_or_ps(y, y2);
  return _mm_xor_ps(y, sign_bit);
}
static __m128 sse_psqrt(__m128 _x) {
  __m128 half = _mm_mul_ps(_x, _mm_set1_ps(.5f));
  __m128 denormal_mask = _mm_and_ps(_mm_cmpge_ps(_x, _mm_setzero_ps()),
                                    _mm_cmplt_ps(_x, _mm_set1_ps(1.17549435e-38f)));
  __m128 x = _mm_rsqrt_ps(_x);
  x = _mm_mul_ps(x, _mm_sub_ps(_mm_set1_ps(1.5f), _mm_mul_ps(half, _mm_mul_ps(x, x))));
  return _mm_andnot_ps(denormal_mask, _mm_mul_ps(_x, x));
}
static float lane(__m128 (*fn)(__m128), float x) {
  float r;
  _mm_store_ss(&r, fn(_mm_set1_ps(x)));
  return r;
}

typedef float (*F1)(float);
static long check_range(const char* name, F1 mine, F1 ref, uint64_t lo, uint64_t hi, uint64_t stride) {
  long bad = 0, n = 0;
  uint32_t first = 0;
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(+ : bad, n)
  for (int64_t i = (int64_t)lo; i < (int64_t)hi; i += (int64_t)stride) {
    float x = asf((uint32_t)i);
    n++;
    if (!same(mine(x), ref(x))) {
      bad++;
#pragma omp critical
      if (!first) first = (uint32_t)i;
    }
  }
  printf("%-14s tested %11ld mismatches %ld", name, n, bad);
  if (bad) printf("  first x=%08x (%.9g) mine=%.9g ref=%.9g", first, asf(first), mine(asf(first)), ref(asf(first)));
  printf("\n");
  fflush(stdout);
  return bad;
}
static long check_both_signs(const char* name, F1 mine, F1 ref, uint32_t maxabs, uint64_t stride) {
  long b = check_range(name, mine, ref, 0, (uint64_t)maxabs + 1, stride);
  b += check_range(name, mine, ref, 0x80000000ull, 0x80000000ull + maxabs + 1, stride);
  return b;
}

static float r_sinf(float x) { return sinf(x); }
static float r_cosf(float x) { return cosf(x); }
static float r_atanf(float x) { return atanf(x); }
static float r_acosf(float x) { return acosf(x); }
static float r_asinf(float x) { return asinf(x); }
static float r_tanf(float x) { return tanf(x); }
static float r_roundf(float x) { return roundf(x); }
static float r_dsin(float x) { return (float)sin((double)x); }
static float r_dcos(float x) { return (float)cos((double)x); }
static float r_psin(float x) { return lane(sse_psin, x); }
static float r_pcos(float x) { return lane(sse_pcos, x); }
static float r_psqrt(float x) { return lane(sse_psqrt, x); }
static float m_sinf(float x) { return g_sinf(x); }
static float m_cosf(float x) { return g_cosf(x); }
static float m_atanf(float x) { return g_atanf(x); }
static float m_acosf(float x) { return g_acosf(x); }
static float m_asinf(float x) { return g_asinf(x); }
static float m_tanf(float x) { return g_tanf(x); }
static float m_roundf(float x) { return roundf_(x); }
static float m_dsin(float x) { return sinf_via_double(x); }
static float m_dcos(float x) { return cosf_via_double(x); }
static float m_psin(float x) { return e_psin(x); }
static float m_pcos(float x) { return e_pcos(x); }
static float m_psqrt(float x) { return e_psqrt(x); }

int main(int argc, char** argv) {
  uint64_t stride = (argc > 1 && !strcmp(argv[1], "quick")) ? 61 : 1;
  const char* only = argc > 2 ? argv[2] : nullptr;
  long bad = 0;
  auto want = [&](const char* n) { return !only || !strcmp(only, n); };
  const uint32_t ALL = 0x7fffffff;
  if (want("sinf")) bad += check_both_signs("sinf", m_sinf, r_sinf, ALL, stride);
  if (want("cosf")) bad += check_both_signs("cosf", m_cosf, r_cosf, ALL, stride);
  if (want("atanf")) bad += check_both_signs("atanf", m_atanf, r_atanf, ALL, stride);
  if (want("acosf")) bad += check_both_signs("acosf", m_acosf, r_acosf, 0x3f800100, stride);
  if (want("asinf")) bad += check_both_signs("asinf", m_asinf, r_asinf, 0x3f800100, stride);
  if (want("tanf")) bad += check_both_signs("tanf", m_tanf, r_tanf, ALL, stride);
  if (want("roundf")) bad += check_both_signs("roundf", m_roundf, r_roundf, ALL, stride);
  if (want("dsin")) bad += check_both_signs("sin(double)", m_dsin, r_dsin, 0x40800000, stride);
  if (want("dcos")) bad += check_both_signs("cos(double)", m_dcos, r_dcos, 0x40800000, stride);
  if (want("psin")) bad += check_both_signs("psin", m_psin, r_psin, ALL, stride);
  if (want("pcos")) bad += check_both_signs("pcos", m_pcos, r_pcos, ALL, stride);
  if (want("psqrt")) bad += check_both_signs("psqrt", m_psqrt, r_psqrt, ALL, stride);
  if (want("atan2f")) {
    // structured + random pairs
    long n = 0, b = 0;
    uint32_t fy = 0, fx = 0;
#pragma omp parallel reduction(+ : n, b)
    {
      std::mt19937_64 rng(1234 + omp_get_thread_num());
      long iters = stride == 1 ? (1L << 28) : (1L << 22);
      for (long i = 0; i < iters / omp_get_num_threads(); i++) {
        uint64_t r = rng();
        float y, x;
        switch (r & 3) {
          case 0: y = asf((uint32_t)(r >> 2)); x = asf((uint32_t)(r >> 34)); break;  // any bits
          case 1: {  // unit-sphere like
            y = (float)((double)(uint32_t)(r >> 2) / 4294967296.0 * 2 - 1);
            x = (float)((double)(uint32_t)(r >> 34) / 1073741824.0 * 2 - 1);
          } break;
          case 2: y = asf((uint32_t)(r >> 2) & 0x807fffffu | 0x3f000000u); x = asf((uint32_t)(r >> 33)); break;
          default: {
            float a = asf((uint32_t)(r >> 2) & 0x3fffffffu);
            y = (r >> 62) & 1 ? -a : a;
            x = asf(asu(a) + (uint32_t)((r >> 40) & 0xff) - 128u);
            if ((r >> 63) & 1) x = -x;
          } break;
        }
        n++;
        if (!same(g_atan2f(y, x), atan2f(y, x))) {
          b++;
#pragma omp critical
          if (!fy && !fx) { fy = asu(y); fx = asu(x); }
        }
      }
    }
    printf("%-14s tested %11ld mismatches %ld", "atan2f[rand]", n, b);
    if (b) printf("  first y=%08x x=%08x mine=%.9g ref=%.9g", fy, fx, g_atan2f(asf(fy), asf(fx)), atan2f(asf(fy), asf(fx)));
    printf("\n");
    bad += b;
  }
  printf(bad ? "NUMERICS: MISMATCH\n" : "NUMERICS: ALL EXACT\n");
  return bad ? 1 : 0;
}

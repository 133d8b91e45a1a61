/* mm_oracle.c -- CPU restatement of the reference's 360-degree multi-model MC path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker for the HIP path: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is never part of
 * the product (vvc-extension-mm_amd/), which fails loudly without its HIP library.
 *
 * Parity status: UNPINNED.  The reference (/root/reference, VTM-17.2 + MM extension) cannot be
 * built here: every CommonLib translation unit reaches Eigen/Dense (Coordinate.h:11, via
 * InterpolationFilter.h:43 -> CacheModel.h -> Picture.h -> Slice.h), Eigen 3.3.7 is a network
 * fetch (source/3rdparty/External-Eigen3.cmake:4-6) and stand-in headers are not allowed; the
 * reference ships no tests, fixtures or bitstreams.  What pins this file
 * is (a) the filter tap tables checked against the reference source text
 * (tests/golden/filter_taps.json, tools/extract_filter_taps.py), (b) this container's glibc
 * 2.35 libm, called directly for every scalar transcendental, and (c) Eigen 3.3.7's SSE
 * psin/pcos/psqrt kernels written here with the same SSE intrinsics Eigen uses (rsqrtps taken
 * from the fixture CPU's table, oracle/rsqrtps_table.h).
 *
 * Structure: the Eigen array code is restated array-at-a-time (one C loop per Eigen assignment
 * expression).  An assignment whose every operation has packet support is evaluated with SSE
 * packets on elements [0, N - N%4) and with scalar glibc calls on the tail (Eigen 3.3.7
 * LinearVectorizedTraversal).
 *
 * Build: gcc -O2 -msse4.1 -ffp-contract=off -fPIC -shared (no -mfma: the reference build has
 * none, CMakeLists.txt:90-93).  File:line citations are into source/Lib/CommonLib.
 */
#include <limits.h>
#include <math.h>
#include <smmintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mm360.h"
#include "rsqrtps_table.h"

#define PI_F ((float)M_PI)
#define NUM_MODELS 11

/* ------------------------------------------------------------------------------------------
 * Eigen 3.3.7 SSE packet kernels (Eigen/src/Core/arch/SSE/MathFunctions.h)
 * ------------------------------------------------------------------------------------------ */
static __m128 orc_psin(__m128 x) {
  const __m128 sign_mask = _mm_castsi128_ps(_mm_set1_epi32((int)0x80000000));
  __m128 sign_bit = _mm_and_ps(x, sign_mask);
  x = _mm_and_ps(x, _mm_castsi128_ps(_mm_set1_epi32(0x7fffffff)));
  __m128 y = _mm_mul_ps(x, _mm_set1_ps(1.27323954473516f));
  __m128i emm2 = _mm_cvttps_epi32(y);
  emm2 = _mm_add_epi32(emm2, _mm_set1_epi32(1));
  emm2 = _mm_and_si128(emm2, _mm_set1_epi32(~1));
  y = _mm_cvtepi32_ps(emm2);
  __m128i emm0 = _mm_slli_epi32(_mm_and_si128(emm2, _mm_set1_epi32(4)), 29);
  emm2 = _mm_cmpeq_epi32(_mm_and_si128(emm2, _mm_set1_epi32(2)), _mm_setzero_si128());
  __m128 poly_mask = _mm_castsi128_ps(emm2);
  sign_bit = _mm_xor_ps(sign_bit, _mm_castsi128_ps(emm0));
  x = _mm_add_ps(x, _mm_mul_ps(y, _mm_set1_ps(-0.78515625f)));
  x = _mm_add_ps(x, _mm_mul_ps(y, _mm_set1_ps(-2.4187564849853515625e-4f)));
  x = _mm_add_ps(x, _mm_mul_ps(y, _mm_set1_ps(-3.77489497744594108e-8f)));
  __m128 z = _mm_mul_ps(x, x);
  y = _mm_set1_ps(2.443315711809948E-005f);
  y = _mm_add_ps(_mm_mul_ps(y, z), _mm_set1_ps(-1.388731625493765E-003f));
  y = _mm_add_ps(_mm_mul_ps(y, z), _mm_set1_ps(4.166664568298827E-002f));
  y = _mm_mul_ps(_mm_mul_ps(y, z), z);
  y = _mm_sub_ps(y, _mm_mul_ps(z, _mm_set1_ps(0.5f)));
  y = _mm_add_ps(y, _mm_set1_ps(1.0f));
  __m128 y2 = _mm_set1_ps(-1.9515295891E-4f);
  y2 = _mm_add_ps(_mm_mul_ps(y2, z), _mm_set1_ps(8.3321608736E-3f));
  y2 = _mm_add_ps(_mm_mul_ps(y2, z), _mm_set1_ps(-1.6666654611E-1f));
  y2 = _mm_add_ps(_mm_mul_ps(_mm_mul_ps(y2, z), x), x);
  y = _mm_or_ps(_mm_andnot_ps(poly_mask, y), _mm_and_ps(poly_mask, y2));
  return _mm_xor_ps(y, sign_bit);
}

static __m128 orc_pcos(__m128 x) {
  x = _mm_and_ps(x, _mm_castsi128_ps(_mm_set1_epi32(0x7fffffff)));
  __m128 y = _mm_mul_ps(x, _mm_set1_ps(1.27323954473516f));
  __m128i emm2 = _mm_cvttps_epi32(y);
  emm2 = _mm_add_epi32(emm2, _mm_set1_epi32(1));
  emm2 = _mm_and_si128(emm2, _mm_set1_epi32(~1));
  y = _mm_cvtepi32_ps(emm2);
  emm2 = _mm_sub_epi32(emm2, _mm_set1_epi32(2));
  __m128i emm0 = _mm_slli_epi32(_mm_andnot_si128(emm2, _mm_set1_epi32(4)), 29);
  emm2 = _mm_cmpeq_epi32(_mm_and_si128(emm2, _mm_set1_epi32(2)), _mm_setzero_si128());
  __m128 sign_bit = _mm_castsi128_ps(emm0);
  __m128 poly_mask = _mm_castsi128_ps(emm2);
  x = _mm_add_ps(x, _mm_mul_ps(y, _mm_set1_ps(-0.78515625f)));
  x = _mm_add_ps(x, _mm_mul_ps(y, _mm_set1_ps(-2.4187564849853515625e-4f)));
  x = _mm_add_ps(x, _mm_mul_ps(y, _mm_set1_ps(-3.77489497744594108e-8f)));
  __m128 z = _mm_mul_ps(x, x);
  y = _mm_set1_ps(2.443315711809948E-005f);
  y = _mm_add_ps(_mm_mul_ps(y, z), _mm_set1_ps(-1.388731625493765E-003f));
  y = _mm_add_ps(_mm_mul_ps(y, z), _mm_set1_ps(4.166664568298827E-002f));
  y = _mm_mul_ps(_mm_mul_ps(y, z), z);
  y = _mm_sub_ps(y, _mm_mul_ps(z, _mm_set1_ps(0.5f)));
  y = _mm_add_ps(y, _mm_set1_ps(1.0f));
  __m128 y2 = _mm_set1_ps(-1.9515295891E-4f);
  y2 = _mm_add_ps(_mm_mul_ps(y2, z), _mm_set1_ps(8.3321608736E-3f));
  y2 = _mm_add_ps(_mm_mul_ps(y2, z), _mm_set1_ps(-1.6666654611E-1f));
  y2 = _mm_add_ps(_mm_mul_ps(_mm_mul_ps(y2, z), x), x);
  y = _mm_or_ps(_mm_andnot_ps(poly_mask, y), _mm_and_ps(poly_mask, y2));
  return _mm_xor_ps(y, sign_bit);
}

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* _mm_rsqrt_ps of the fixture CPU (the GPU box host may be another vendor): table lookup */
static float orc_rsqrtps1(float x) {
  uint32_t ix = f2u(x), ax = ix & 0x7fffffffu;
  if (ax > 0x7f800000u) return u2f(ix | 0x00400000u);
  if (ax < 0x00800000u) return u2f((ix & 0x80000000u) | 0x7f800000u);
  if (ix & 0x80000000u) return u2f(0xffc00000u);
  if (ax == 0x7f800000u) return 0.0f;
  int e = (int)(ax >> 23) - 127;
  int half = e >= 0 ? e / 2 : -((-e + 1) / 2);
  return u2f(((uint32_t)(126 - half) << 23) | MM_RSQRTPS_MANT[e & 1][(ax >> 13) & 1023]);
}
static __m128 orc_psqrt(__m128 _x) {
#if MM_PSQRT_EXACT
  return _mm_sqrt_ps(_x);
#endif
  float in[4], r[4];
  _mm_storeu_ps(in, _x);
  for (int i = 0; i < 4; i++) r[i] = orc_rsqrtps1(in[i]);
  __m128 half = _mm_mul_ps(_x, _mm_set1_ps(.5f));
  __m128 denormal_mask = _mm_and_ps(_mm_cmpge_ps(_x, _mm_setzero_ps()), _mm_cmplt_ps(_x, _mm_set1_ps(1.17549435e-38f)));
  __m128 x = _mm_loadu_ps(r);
  x = _mm_mul_ps(x, _mm_sub_ps(_mm_set1_ps(1.5f), _mm_mul_ps(half, _mm_mul_ps(x, x))));
  return _mm_andnot_ps(denormal_mask, _mm_mul_ps(_x, x));
}

/* array.sin() / .cos() / .sqrt() on a packet-able assignment: packets then glibc tail */
typedef __m128 (*pkfn)(__m128);
typedef float (*scfn)(float);
static void arr_unary(float* out, const float* in, int n, pkfn pk, scfn sc) {
  int aligned_end = n - (n % 4);
  for (int i = 0; i < aligned_end; i += 4) _mm_storeu_ps(out + i, pk(_mm_loadu_ps(in + i)));
  for (int i = aligned_end; i < n; i++) out[i] = sc(in[i]);
}
static float sc_sin(float x) { return sinf(x); }
static float sc_cos(float x) { return cosf(x); }
static float sc_sqrt(float x) { return sqrtf(x); }
static void arr_sin(float* o, const float* i, int n) { arr_unary(o, i, n, orc_psin, sc_sin); }
static void arr_cos(float* o, const float* i, int n) { arr_unary(o, i, n, orc_pcos, sc_cos); }
static void arr_sqrt(float* o, const float* i, int n) { arr_unary(o, i, n, orc_psqrt, sc_sqrt); }

/* ------------------------------------------------------------------------------------------
 * Coordinates (Coordinate.cpp) -- array forms operate on N-element arrays
 * ------------------------------------------------------------------------------------------ */
typedef struct { float *x, *y, *z; } A3;

static float* fa(int n) { return (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1)); }
static A3 a3_new(int n) { A3 a = {fa(n), fa(n), fa(n)}; return a; }
static void a3_free(A3 a) { free(a.x); free(a.y); free(a.z); }

/* cartesianToSpherical, array form (Coordinate.cpp:98-106 incl. header offset) */
static void c2s_arr(const A3 c, float* R, float* th, float* ph, int n) {
  float* t = fa(n);
  for (int i = 0; i < n; i++) t[i] = c.x[i] * c.x[i] + c.y[i] * c.y[i] + c.z[i] * c.z[i];
  arr_sqrt(R, t, n);  /* (x.square() + y.square() + z.square()).sqrt() : packet */
  for (int i = 0; i < n; i++) {
    float v = c.z[i] / R[i];
    v = (1.0f < v) ? 1.0f : v;    /* cwiseMin(1): std::min(v, 1) */
    v = (v < -1.0f) ? -1.0f : v;  /* cwiseMax(-1): std::max(v, -1) */
    th[i] = acosf(v);             /* acos: no packet -> scalar for all elements */
    ph[i] = atan2f(c.y[i], c.x[i]);
  }
  free(t);
}

/* sphericalToCartesian, array form: R * sin(th) * cos(ph) ... (packet) */
static void s2c_arr(const float* R, const float* th, const float* ph, A3 out, int n) {
  float *st = fa(n), *ct = fa(n), *sp = fa(n), *cp = fa(n);
  arr_sin(st, th, n);
  arr_cos(ct, th, n);
  arr_sin(sp, ph, n);
  arr_cos(cp, ph, n);
  for (int i = 0; i < n; i++) {
    out.x[i] = R[i] * st[i] * cp[i];
    out.y[i] = R[i] * st[i] * sp[i];
    out.z[i] = R[i] * ct[i];
  }
  free(st); free(ct); free(sp); free(cp);
}

/* scalar Array3 forms (Coordinate.cpp:40-45 / :55-61 in SURVEY numbering) */
static void c2s_scalar(float x, float y, float z, float* R, float* th, float* ph) {
  *R = sqrtf((x * x) + (y * y) + (z * z));
  float v = z / *R;
  float w = (-1.0f < v) ? v : -1.0f; /* std::max(TCoord(-1), v) */
  w = (w < 1.0f) ? w : 1.0f;         /* std::min(TCoord(1), .) */
  *th = acosf(w);
  *ph = atan2f(y, x);
}

/* ------------------------------------------------------------------------------------------
 * Projections (Projection.cpp)
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  int W, H, Wc, Hc, chroma, bd, maxcu_w, maxcu_h, ged_flavor;
  float off, focal, res;
  uint32_t active;
  /* frame grid + MPA caches, row-major [j][i] of (H/4) x (W/4) */
  float* mpa_px[3];
  float* mpa_py[3];
  unsigned char* mpa_vip[3];
  /* epipoles */
  int n_epi;
  int epi_key[256][2];
  int32_t epi_q[256][3];
  char err[256];
} Orc;

/* EquirectangularProjection::toSphere, array form (pixelOffset 0) */
static void erp_to_sphere_arr(const Orc* o, const float* x, const float* y, A3 out, int n) {
  float *R = fa(n), *th = fa(n), *ph = fa(n);
  for (int i = 0; i < n; i++) {
    R[i] = 1.0f;
    ph[i] = -((x[i] + 0.0f) / (float)o->W) * 2.0f * PI_F;
    th[i] = ((y[i] + 0.0f) / (float)o->H) * PI_F;
  }
  s2c_arr(R, th, ph, out, n);
  free(R); free(th); free(ph);
}

/* EquirectangularProjection::fromSphere, array form */
static void erp_from_sphere_arr(const Orc* o, const A3 c, float* x, float* y, int n) {
  float *R = fa(n), *th = fa(n), *ph = fa(n);
  c2s_arr(c, R, th, ph, n);
  for (int i = 0; i < n; i++) {
    float p = ph[i] > 0 ? ph[i] - 2.0f * PI_F : ph[i];
    x[i] = -(p / (2.0f * PI_F)) * (float)o->W - 0.0f;
    y[i] = (th[i] / PI_F) * (float)o->H - 0.0f;
  }
  free(R); free(th); free(ph);
}

/* EquirectangularProjection::toSphere, scalar form */
static void erp_to_sphere1(const Orc* o, float x, float y, float* X, float* Y, float* Z) {
  float ph = -((x + 0.0f) / (float)o->W) * 2.0f * PI_F;
  float th = ((y + 0.0f) / (float)o->H) * PI_F;
  *X = 1.0f * sinf(th) * cosf(ph);
  *Y = 1.0f * sinf(th) * sinf(ph);
  *Z = 1.0f * cosf(th);
}

/* PerspectiveProjection::fromSphere, array form (optical centre 0) */
static void persp_from_sphere_arr(const Orc* o, const A3 c, float* px, float* py, unsigned char* vip, int n) {
  A3 rot = a3_new(n);
  for (int i = 0; i < n; i++) {
    rot.x[i] = c.y[i];
    rot.y[i] = -c.z[i];
    rot.z[i] = -c.x[i];
  }
  float *R = fa(n), *th = fa(n), *ph = fa(n), *pr = fa(n), *cp = fa(n), *sp = fa(n);
  c2s_arr(rot, R, th, ph, n);
  for (int i = 0; i < n; i++) pr[i] = o->focal * tanf(th[i]); /* tan: scalar */
  arr_cos(cp, ph, n);
  arr_sin(sp, ph, n);
  for (int i = 0; i < n; i++) {
    px[i] = pr[i] * cp[i] + 0.0f;
    py[i] = pr[i] * sp[i] + 0.0f;
    vip[i] = pr[i] < 0;
  }
  a3_free(rot);
  free(R); free(th); free(ph); free(pr); free(cp); free(sp);
}

/* PerspectiveProjection::toSphere, array form */
static void persp_to_sphere_arr(const Orc* o, const float* x, const float* y, const unsigned char* vip, A3 out,
                                int n) {
  float *xx = fa(n), *yy = fa(n), *t = fa(n), *r = fa(n), *ph = fa(n), *th = fa(n), *R = fa(n);
  for (int i = 0; i < n; i++) {
    xx[i] = x[i] - 0.0f;
    yy[i] = y[i] - 0.0f;
    t[i] = xx[i] * xx[i] + yy[i] * yy[i];
  }
  arr_sqrt(r, t, n); /* cartesianToPolar R: packet */
  for (int i = 0; i < n; i++) {
    ph[i] = atan2f(yy[i], xx[i]);
    th[i] = atanf(r[i] / o->focal);
    float v = vip[i] ? 1.0f : 0.0f;
    th[i] = th[i] - v * (2.0f * th[i] - PI_F);
    ph[i] = ph[i] - v * PI_F;
    R[i] = 1.0f;
  }
  A3 c = a3_new(n);
  s2c_arr(R, th, ph, c, n);
  for (int i = 0; i < n; i++) {
    out.x[i] = -c.z[i];
    out.y[i] = c.x[i];
    out.z[i] = -c.y[i];
  }
  a3_free(c);
  free(xx); free(yy); free(t); free(r); free(ph); free(th); free(R);
}

/* ------------------------------------------------------------------------------------------
 * Motion models (the MotionModels directory)
 * ------------------------------------------------------------------------------------------ */
static void mpa_to_perspective_arr(const Orc* o, int plane, const float* gx, const float* gy, float* px, float* py,
                                   unsigned char* vip, int n) {
  A3 s = a3_new(n), q = a3_new(n);
  erp_to_sphere_arr(o, gx, gy, s, n);
  for (int i = 0; i < n; i++) {
    if (plane == 1) { q.x[i] = s.x[i]; q.y[i] = s.y[i]; q.z[i] = s.z[i]; }
    else if (plane == 2) { q.x[i] = s.y[i]; q.y[i] = -s.x[i]; q.z[i] = s.z[i]; }
    else { q.x[i] = -s.z[i]; q.y[i] = s.y[i]; q.z[i] = s.x[i]; }
  }
  persp_from_sphere_arr(o, q, px, py, vip, n);
  a3_free(s); a3_free(q);
}

static void mpa_to_projection_arr(const Orc* o, int plane, const float* px, const float* py, const unsigned char* vip,
                                  float* ox, float* oy, int n) {
  A3 q = a3_new(n), s = a3_new(n);
  persp_to_sphere_arr(o, px, py, vip, q, n);
  for (int i = 0; i < n; i++) {
    if (plane == 1) { s.x[i] = q.x[i]; s.y[i] = q.y[i]; s.z[i] = q.z[i]; }
    else if (plane == 2) { s.x[i] = -q.y[i]; s.y[i] = q.x[i]; s.z[i] = q.z[i]; }
    else { s.x[i] = q.z[i]; s.y[i] = q.y[i]; s.z[i] = -q.x[i]; }
  }
  erp_from_sphere_arr(o, s, ox, oy, n);
  a3_free(q); a3_free(s);
}

/* Numerics modes (same switches as the product's mm_numerics.h): MM_ROUND_MODE,
 * MM_PROD3_MODE, MM_TAN_CENTRE_MODE, MM_PSQRT_EXACT; 0 = the believed Eigen 3.3.7 behaviour. */
#ifndef MM_ROUND_MODE
#define MM_ROUND_MODE 0
#endif
#ifndef MM_PROD3_MODE
#define MM_PROD3_MODE 0
#endif
#ifndef MM_TAN_CENTRE_MODE
#define MM_TAN_CENTRE_MODE 0
#endif
#ifndef MM_PSQRT_EXACT
#define MM_PSQRT_EXACT 0
#endif

/* Eigen lazy coefficient-based 3x3 product coefficient: p0 + (p1 + p2) */
static float dot3(float a0, float b0, float a1, float b1, float a2, float b2) {
#if MM_PROD3_MODE
  return (a0 * b0 + a1 * b1) + a2 * b2;
#else
  return a0 * b0 + (a1 * b1 + a2 * b2);
#endif
}
static void matmul3(const float* A, const float* B, float* C) {
  float T[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) T[3 * i + j] = dot3(A[3 * i], B[j], A[3 * i + 1], B[3 + j], A[3 * i + 2], B[6 + j]);
  memcpy(C, T, sizeof(T));
}
static void transpose3(const float* A, float* T) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) T[3 * j + i] = A[3 * i + j];
}

/* Eigen::AngleAxis<float>::toRotationMatrix */
static void angle_axis(float angle, const float* a, float* res) {
  float s = sinf(angle), c = cosf(angle);
  float sin_axis[3] = {s * a[0], s * a[1], s * a[2]};
  float cos1_axis[3] = {(1.0f - c) * a[0], (1.0f - c) * a[1], (1.0f - c) * a[2]};
  float tmp;
  tmp = cos1_axis[0] * a[1];
  res[1] = tmp - sin_axis[2];
  res[3] = tmp + sin_axis[2];
  tmp = cos1_axis[0] * a[2];
  res[2] = tmp + sin_axis[1];
  res[6] = tmp - sin_axis[1];
  tmp = cos1_axis[1] * a[2];
  res[5] = tmp - sin_axis[0];
  res[7] = tmp + sin_axis[0];
  res[0] = cos1_axis[0] * a[0] + c;
  res[4] = cos1_axis[1] * a[1] + c;
  res[8] = cos1_axis[2] * a[2] + c;
}

/* GeodesicMotionModel::setEpipole (GeodesicMotionModel.cpp:14-46) -> row-major 3x3 */
static void ged_set_epipole(const float* e, float* Mout) {
  float nrm = sqrtf(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
  float pa[3] = {e[0] / nrm, e[1] / nrm, e[2] / nrm};
  float cr[3] = {-pa[1], pa[0], 0};
  float s = sqrtf(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
  if (s == 0) {
    float I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (pa[2] < 0) I[8] = -1;
    memcpy(Mout, I, sizeof(I));
    return;
  }
  float mn = pa[2] < 1.0f ? pa[2] : 1.0f;
  float c = -1.0f < mn ? mn : -1.0f;
  float K[9] = {0};
  K[1] = -cr[2];
  K[2] = cr[1];
  K[3] = cr[2];
  K[5] = -cr[0];
  K[6] = -cr[1];
  K[7] = cr[0];
  float K2[9];
  matmul3(K, K, K2);
  float f = (1 - c) / (s * s);
  float M[9];
  for (int i = 0; i < 9; i++) {
    float I = (i % 4 == 0) ? 1.0f : 0.0f;
    M[i] = I + K[i] + K2[i] * f;
  }
  transpose3(M, Mout);
}

/* GeodesicMotionModel::toRotatedSphere + modelGeodesicMotion + fromRotatedSphere */
static void ged_model(const Orc* o, const float* Rm, const float* gx, const float* gy, int n, float mvx, float mvy,
                      float cx, float cy, float* ox, float* oy) {
  A3 c = a3_new(n), rot = a3_new(n);
  erp_to_sphere_arr(o, gx, gy, c, n);
  for (int i = 0; i < n; i++) {
    rot.x[i] = dot3(Rm[0], c.x[i], Rm[1], c.y[i], Rm[2], c.z[i]);
    rot.y[i] = dot3(Rm[3], c.x[i], Rm[4], c.y[i], Rm[5], c.z[i]);
    rot.z[i] = dot3(Rm[6], c.x[i], Rm[7], c.y[i], Rm[8], c.z[i]);
  }
  float *R = fa(n), *th = fa(n), *ph = fa(n);
  c2s_arr(rot, R, th, ph, n);
  if (o->ged_flavor == 1) {
    float X, Y, Z, r, tc, pc;
    erp_to_sphere1(o, cx, cy, &X, &Y, &Z);
    float crx = dot3(Rm[0], X, Rm[1], Y, Rm[2], Z), cry = dot3(Rm[3], X, Rm[4], Y, Rm[5], Z),
          crz = dot3(Rm[6], X, Rm[7], Y, Rm[8], Z);
    c2s_scalar(crx, cry, crz, &r, &tc, &pc);
    float k = sinf(tc + o->res * mvx) / sinf(o->res * mvx);
    for (int i = 0; i < n; i++) th[i] = th[i] + atanf(sinf(th[i]) / (k - cosf(th[i]))); /* atan: scalar */
  } else {
    for (int i = 0; i < n; i++) th[i] = th[i] + o->res * mvx;
  }
  for (int i = 0; i < n; i++) ph[i] = ph[i] + o->res * mvy;
  A3 m = a3_new(n), back = a3_new(n);
  s2c_arr(R, th, ph, m, n);
  for (int i = 0; i < n; i++) {
    back.x[i] = dot3(Rm[0], m.x[i], Rm[3], m.y[i], Rm[6], m.z[i]);
    back.y[i] = dot3(Rm[1], m.x[i], Rm[4], m.y[i], Rm[7], m.z[i]);
    back.z[i] = dot3(Rm[2], m.x[i], Rm[5], m.y[i], Rm[8], m.z[i]);
  }
  erp_from_sphere_arr(o, back, ox, oy, n);
  a3_free(c); a3_free(rot); a3_free(m); a3_free(back);
  free(R); free(th); free(ph);
}

/* RotationalMotionModel::modelMotion (RotationalMotionModel.cpp:8-78) */
static void rot_model(const Orc* o, const float* gx, const float* gy, int n, float mvx, float mvy, float cx, float cy,
                      float* ox, float* oy) {
  float X, Y, Z, r, tc, pc;
  erp_to_sphere1(o, cx, cy, &X, &Y, &Z);
  c2s_scalar(X, Y, Z, &r, &tc, &pc);
  const float uz[3] = {0, 0, 1}, uy[3] = {0, 1, 0};
  float A[9], B[9], rotm[9], uphi[9], uth[9], unrot[9], unrotT[9], tmp[9], really[9];
  angle_axis(-mvx * o->res, uz, A);
  angle_axis(mvy * o->res, uy, B);
  matmul3(A, B, rotm);
  angle_axis(-pc, uz, uphi);
  angle_axis((float)(M_PI_2 - tc), uy, uth);
  matmul3(uth, uphi, unrot);
  transpose3(unrot, unrotT);
  matmul3(rotm, unrot, tmp);
  matmul3(unrotT, tmp, really);
  A3 c = a3_new(n), mv = a3_new(n);
  erp_to_sphere_arr(o, gx, gy, c, n);
  for (int i = 0; i < n; i++) {
    mv.x[i] = dot3(really[0], c.x[i], really[1], c.y[i], really[2], c.z[i]);
    mv.y[i] = dot3(really[3], c.x[i], really[4], c.y[i], really[5], c.z[i]);
    mv.z[i] = dot3(really[6], c.x[i], really[7], c.y[i], really[8], c.z[i]);
  }
  erp_from_sphere_arr(o, mv, ox, oy, n);
  a3_free(c); a3_free(mv);
}

/* TangentialMotionModel::modelMotion (TangentialMotionModel.cpp:8-48) */
static void tan_model(const Orc* o, const float* gx, const float* gy, int n, float mvx, float mvy, float cx, float cy,
                      float* ox, float* oy) {
  float X, Y, Z, r, tc, pc;
  erp_to_sphere1(o, cx, cy, &X, &Y, &Z);
  c2s_scalar(X, Y, Z, &r, &tc, &pc);
  const float epsC = (float)(M_PI_2 - (double)tc);
  const float alphaC = pc;
  /* unqualified sin/cos on a float -> double ::sin/::cos, result promoted to float in the array expr */
#if MM_TAN_CENTRE_MODE
  const float sE = sinf(epsC), cE = cosf(epsC);
#else
  const float sE = (float)sin((double)epsC), cE = (float)cos((double)epsC);
#endif
  A3 c = a3_new(n);
  erp_to_sphere_arr(o, gx, gy, c, n);
  float *R = fa(n), *th = fa(n), *ph = fa(n);
  c2s_arr(c, R, th, ph, n);
  float *eps = fa(n), *dA = fa(n), *se = fa(n), *ce = fa(n), *cdA = fa(n), *sdA = fa(n);
  for (int i = 0; i < n; i++) {
    eps[i] = (float)M_PI_2 - th[i];
    dA[i] = ph[i] - alphaC;
  }
  arr_sin(se, eps, n);
  arr_cos(ce, eps, n);
  arr_cos(cdA, dA, n);
  arr_sin(sdA, dA, n);
  float *cosPsi = fa(n), *yP = fa(n), *xP = fa(n), *yM = fa(n), *xM = fa(n), *t = fa(n), *rho = fa(n), *eta = fa(n);
  for (int i = 0; i < n; i++) cosPsi[i] = sE * se[i] + cE * ce[i] * cdA[i];
  for (int i = 0; i < n; i++) yP[i] = (se[i] * cE - sE * ce[i] * cdA[i]) / cosPsi[i];
  for (int i = 0; i < n; i++) xP[i] = (sdA[i] * ce[i]) / cosPsi[i];
  for (int i = 0; i < n; i++) {
    yM[i] = yP[i] - mvy * o->res;
    xM[i] = xP[i] - mvx * o->res;
    t[i] = xM[i] * xM[i] + yM[i] * yM[i];
  }
  arr_sqrt(rho, t, n);
  for (int i = 0; i < n; i++) eta[i] = atanf(rho[i]);
  float *seta = fa(n), *ceta = fa(n), *gam = fa(n), *aM = fa(n), *eM = fa(n), *thM = fa(n), *one = fa(n);
  arr_sin(seta, eta, n);
  arr_cos(ceta, eta, n);
  for (int i = 0; i < n; i++) gam[i] = rho[i] * cE * ceta[i] - yM[i] * sE * seta[i];
  /* atan / asin: the whole assignment is scalar (glibc sinf/cosf inside) */
  for (int i = 0; i < n; i++) aM[i] = alphaC + atanf((xM[i] * sinf(eta[i])) / gam[i]);
  for (int i = 0; i < n; i++) eM[i] = asinf(cosf(eta[i]) * sE + (yM[i] * sinf(eta[i]) * cE) / rho[i]);
  for (int i = 0; i < n; i++) {
    thM[i] = (float)M_PI_2 - eM[i];
    one[i] = 1.0f;
  }
  A3 m = a3_new(n);
  s2c_arr(one, thM, aM, m, n);
  erp_from_sphere_arr(o, m, ox, oy, n);
  a3_free(c); a3_free(m);
  free(R); free(th); free(ph); free(eps); free(dA); free(se); free(ce); free(cdA); free(sdA);
  free(cosPsi); free(yP); free(xP); free(yM); free(xM); free(t); free(rho); free(eta);
  free(seta); free(ceta); free(gam); free(aM); free(eM); free(thM); free(one);
}

/* ThreeDTranslationalMotionModel::modelMotion (ThreeDTranslationalMotionModel.cpp:7-24) */
static void t3d_model(const Orc* o, const float* gx, const float* gy, int n, float mvx, float mvy, float cx, float cy,
                      float* ox, float* oy) {
  float X, Y, Z, Xm, Ym, Zm;
  erp_to_sphere1(o, cx, cy, &X, &Y, &Z);
  erp_to_sphere1(o, cx + mvx, cy + mvy, &Xm, &Ym, &Zm);
  float d[3] = {Xm - X, Ym - Y, Zm - Z};
  A3 c = a3_new(n);
  erp_to_sphere_arr(o, gx, gy, c, n);
  for (int i = 0; i < n; i++) {
    c.x[i] = c.x[i] + d[0];
    c.y[i] = c.y[i] + d[1];
    c.z[i] = c.z[i] + d[2];
  }
  erp_from_sphere_arr(o, c, ox, oy, n);
  a3_free(c);
}

/* ------------------------------------------------------------------------------------------
 * MVReprojection::reprojectMotionVectorSubblocks (MVReprojection.cpp:80-166)
 * comp: 0 luma, else chroma 4:2:0.  pos/size in component units.  out: 2*N ints, Eigen
 * column-major element order.
 * ------------------------------------------------------------------------------------------ */
static int find_epipole(const Orc* o, int cur, int ref, float* e) {
  int keys[3][2] = {{cur, ref}, {cur, -1}, {-1, -1}};
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < o->n_epi; i++)
      if (o->epi_key[i][0] == keys[k][0] && o->epi_key[i][1] == keys[k][1]) {
        for (int d = 0; d < 3; d++) {
          int32_t v = o->epi_q[i][d];
          e[d] = (float)(v >> 24) + (float)(v & ((1 << 24) - 1)) / (float)(1 << 24);
        }
        return 0;
      }
  return -1;
}

static int reproject(Orc* o, int px_, int py_, int w, int h, int mvh, int mvv, int model, int comp, int cur, int ref,
                     int32_t* out) {
  const int chroma = comp != 0;
  const int sbw = chroma ? 2 : 4, sbh = chroma ? 2 : 4;
  const int rows = h / sbh, cols = w / sbw, n = rows * cols;
  const float scale = chroma ? 2.0f : 1.0f;
  const int shift = 4 + (chroma ? 1 : 0);
  float *gx = fa(n), *gy = fa(n), *mx = fa(n), *my = fa(n);
  /* grid: luma block of the frame cache (LinSpaced(W/4, off, W-4+off)), chroma LinSpaced */
  for (int c = 0; c < cols; c++)
    for (int r = 0; r < rows; r++) {
      int i = c * rows + r;
      if (!chroma) {
        gx[i] = 4.0f * (float)(px_ / 4 + c) + o->off;
        gy[i] = 4.0f * (float)(py_ / 4 + r) + o->off;
      } else {
        float sx = (float)px_ * scale + o->off, sy = (float)py_ * scale + o->off;
        float ex = sx + (float)(w - sbw) * scale, ey = sy + (float)(h - sbh) * scale;
        float stx = cols == 1 ? 0.0f : (ex - sx) / (float)(cols - 1);
        float sty = rows == 1 ? 0.0f : (ey - sy) / (float)(rows - 1);
        gx[i] = cols == 1 ? ex : (c == cols - 1 ? ex : sx + (float)c * stx);
        gy[i] = rows == 1 ? ey : (r == rows - 1 ? ey : sy + (float)r * sty);
      }
    }
  const float mvX = (float)(mvh >> 4) + (float)(mvh & 15) / (float)16;
  const float mvY = (float)(mvv >> 4) + (float)(mvv & 15) / (float)16;
  const float cx = (float)px_ + ((float)w - 1) / 2.0f, cy = (float)py_ + ((float)h - 1) / 2.0f;
  const int zero = (mvX == 0 && mvY == 0);
  switch (model) {
    case 1: case 2: case 3: {
      float *ppx = fa(n), *ppy = fa(n);
      unsigned char* vip = (unsigned char*)malloc((size_t)n);
      if (!chroma) { /* modelMotionCached: cached perspective grid of the whole frame */
        const int fcols = o->W / 4;
        for (int c = 0; c < cols; c++)
          for (int r = 0; r < rows; r++) {
            int fi = (py_ / 4 + r) * fcols + px_ / 4 + c;
            ppx[c * rows + r] = o->mpa_px[model - 1][fi];
            ppy[c * rows + r] = o->mpa_py[model - 1][fi];
            vip[c * rows + r] = o->mpa_vip[model - 1][fi];
          }
      } else {
        mpa_to_perspective_arr(o, model, gx, gy, ppx, ppy, vip, n);
      }
      for (int i = 0; i < n; i++) {
        float sgn = vip[i] ? -1.0f : 1.0f;
        ppx[i] = ppx[i] + mvX * sgn;
        ppy[i] = ppy[i] + mvY * sgn;
      }
      mpa_to_projection_arr(o, model, ppx, ppy, vip, mx, my, n);
      free(ppx); free(ppy); free(vip);
    } break;
    case 4:
      if (zero) { memcpy(mx, gx, sizeof(float) * n); memcpy(my, gy, sizeof(float) * n); }
      else tan_model(o, gx, gy, n, mvX, mvY, cx, cy, mx, my);
      break;
    case 5:
      if (zero) { memcpy(mx, gx, sizeof(float) * n); memcpy(my, gy, sizeof(float) * n); }
      else t3d_model(o, gx, gy, n, mvX, mvY, cx, cy, mx, my);
      break;
    case 6:
      if (zero) { memcpy(mx, gx, sizeof(float) * n); memcpy(my, gy, sizeof(float) * n); }
      else rot_model(o, gx, gy, n, mvX, mvY, cx, cy, mx, my);
      break;
    case 7: case 8: case 9: case 10: {
      float e[3], Rm[9];
      if (model == 7) { e[0] = 1; e[1] = 0; e[2] = 0; }
      else if (model == 8) { e[0] = 0; e[1] = 1; e[2] = 0; }
      else if (model == 9) { e[0] = 0; e[1] = 0; e[2] = 1; }
      else if (find_epipole(o, cur, ref, e)) { free(gx); free(gy); free(mx); free(my); return MM_ERR_NOEPIPOLE; }
      ged_set_epipole(e, Rm);
      if (chroma && zero) { memcpy(mx, gx, sizeof(float) * n); memcpy(my, gy, sizeof(float) * n); }
      else ged_model(o, Rm, gx, gy, n, mvX, mvY, cx, cy, mx, my);
    } break;
    default:
      free(gx); free(gy); free(mx); free(my);
      return MM_ERR_MODEL;
  }
  for (int i = 0; i < n; i++) {
    float x = (isnan(mx[i]) || isnan(my[i])) ? gx[i] : mx[i];
    float y = (isnan(mx[i]) || isnan(my[i])) ? gy[i] : my[i];
    x = x - o->off;
    y = y - o->off;
    if (chroma) { x = x / scale; y = y / scale; }
#if MM_ROUND_MODE
    const int packet = n >= 4 && i < n - n % 4; /* pround = _mm_round_ps(x, 0): ties to even */
    float rx = packet ? rintf(x * (float)(1 << shift)) : roundf(x * (float)(1 << shift));
    float ry = packet ? rintf(y * (float)(1 << shift)) : roundf(y * (float)(1 << shift));
#else
    float rx = roundf(x * (float)(1 << shift)), ry = roundf(y * (float)(1 << shift));
#endif
    out[2 * i] = _mm_cvtt_ss2si(_mm_set_ss(rx));
    out[2 * i + 1] = _mm_cvtt_ss2si(_mm_set_ss(ry));
  }
  free(gx); free(gy); free(mx); free(my);
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * Integer pel pipeline (InterpolationFilter.cpp, Buffer.cpp) on padded planes
 * ------------------------------------------------------------------------------------------ */
static const int16_t LUMA[16][8] = {
    {0, 0, 0, 64, 0, 0, 0, 0},        {0, 1, -3, 63, 4, -2, 1, 0},      {-1, 2, -5, 62, 8, -3, 1, 0},
    {-1, 3, -8, 60, 13, -4, 1, 0},    {-1, 4, -10, 58, 17, -5, 1, 0},   {-1, 4, -11, 52, 26, -8, 3, -1},
    {-1, 3, -9, 47, 31, -10, 4, -1},  {-1, 4, -11, 45, 34, -10, 4, -1}, {-1, 4, -11, 40, 40, -11, 4, -1},
    {-1, 4, -10, 34, 45, -11, 4, -1}, {-1, 4, -10, 31, 47, -9, 3, -1},  {-1, 3, -8, 26, 52, -11, 4, -1},
    {0, 1, -5, 17, 58, -10, 4, -1},   {0, 1, -4, 13, 60, -8, 3, -1},    {0, 1, -3, 8, 62, -5, 2, -1},
    {0, 1, -2, 4, 63, -3, 1, 0}};
static const int16_t CHROMA[32][4] = {
    {0, 64, 0, 0},    {-1, 63, 2, 0},   {-2, 62, 4, 0},   {-2, 60, 7, -1},  {-2, 58, 10, -2}, {-3, 57, 12, -2},
    {-4, 56, 14, -2}, {-4, 55, 15, -2}, {-4, 54, 16, -2}, {-5, 53, 18, -2}, {-6, 52, 20, -2}, {-6, 49, 24, -3},
    {-6, 46, 28, -4}, {-5, 44, 29, -4}, {-4, 42, 30, -4}, {-4, 39, 33, -4}, {-4, 36, 36, -4}, {-4, 33, 39, -4},
    {-4, 30, 42, -4}, {-4, 29, 44, -5}, {-4, 28, 46, -6}, {-3, 24, 49, -6}, {-2, 20, 52, -6}, {-2, 18, 53, -5},
    {-2, 16, 54, -4}, {-2, 15, 55, -4}, {-2, 14, 56, -4}, {-2, 12, 57, -3}, {-2, 10, 58, -2}, {-1, 7, 60, -2},
    {0, 4, 62, -2},   {0, 2, 63, -1}};

static int frac_bits(int bd) { return (14 - bd) > 2 ? 14 - bd : 2; }
static int16_t clip_pel(int v, int bd) { int m = (1 << bd) - 1; return (int16_t)(v < 0 ? 0 : v > m ? m : v); }

/* InterpolationFilter::filterCopy<isFirst,isLast> (InterpolationFilter.cpp:392-514) */
static void filter_copy(int bd, const int16_t* src, ptrdiff_t ss, int16_t* dst, ptrdiff_t ds, int w, int h, int first,
                        int last) {
  for (int r = 0; r < h; r++, src += ss, dst += ds)
    for (int c = 0; c < w; c++) {
      if (first == last)
        dst[c] = src[c];
      else if (first) {
        int16_t val = (int16_t)(src[c] << frac_bits(bd));
        dst[c] = (int16_t)(val - (int16_t)8192);
      } else {
        int shift = frac_bits(bd);
        int16_t val = (int16_t)((src[c] + 8192 + (1 << (shift - 1))) >> shift);
        dst[c] = clip_pel(val, bd);
      }
    }
}

/* InterpolationFilter::filter<N,isVertical,isFirst,isLast> (InterpolationFilter.cpp:540-644) */
static void filter_n(int N, int vert, int first, int last, int bd, const int16_t* src, ptrdiff_t ss, int16_t* dst,
                     ptrdiff_t ds, int w, int h, const int16_t* coeff) {
  ptrdiff_t cs = vert ? ss : 1;
  src -= (N / 2 - 1) * cs;
  int headRoom = frac_bits(bd), shift = 6, offset;
  if (last) {
    shift += first ? 0 : headRoom;
    offset = 1 << (shift - 1);
    offset += first ? 0 : 8192 << 6;
  } else {
    shift -= first ? headRoom : 0;
    offset = first ? -8192 * (1 << shift) : 0;
  }
  for (int r = 0; r < h; r++, src += ss, dst += ds)
    for (int c = 0; c < w; c++) {
      int sum = 0;
      for (int k = 0; k < N; k++) sum += src[c + k * cs] * coeff[k];
      int16_t val = (int16_t)((sum + offset) >> shift);
      if (last) val = clip_pel(val, bd);
      dst[c] = val;
    }
}

/* public filterHor / filterVer (InterpolationFilter.cpp:675-809), FILTER_DEFAULT */
static void filter_hor(int comp, int bd, const int16_t* src, ptrdiff_t ss, int16_t* dst, ptrdiff_t ds, int w, int h,
                       int frac, int last) {
  if (frac == 0) filter_copy(bd, src, ss, dst, ds, w, h, 1, last);
  else if (comp == 0) filter_n(8, 0, 1, last, bd, src, ss, dst, ds, w, h, LUMA[frac]);
  else filter_n(4, 0, 1, last, bd, src, ss, dst, ds, w, h, CHROMA[frac]);
}
static void filter_ver(int comp, int bd, const int16_t* src, ptrdiff_t ss, int16_t* dst, ptrdiff_t ds, int w, int h,
                       int frac, int first, int last) {
  if (frac == 0) filter_copy(bd, src, ss, dst, ds, w, h, first, last);
  else if (comp == 0) filter_n(8, 1, first, last, bd, src, ss, dst, ds, w, h, LUMA[frac]);
  else filter_n(4, 1, first, last, bd, src, ss, dst, ds, w, h, CHROMA[frac]);
}

/* Picture with the reference's padded layout (margin = 2*(maxCU+16), extendPicBorder) */
typedef struct {
  int poc;
  int16_t* buf[3];
  int stride[3], margin[3], w[3], h[3];
} OPic;

static void pad_plane(const int16_t* src, ptrdiff_t sstride, int w, int h, int margin, int16_t** out, int* ostride) {
  int stride = w + 2 * margin;
  int16_t* b = (int16_t*)malloc(sizeof(int16_t) * (size_t)stride * (size_t)(h + 2 * margin));
  int16_t* org = b + (size_t)margin * stride + margin;
  for (int y = 0; y < h; y++) {
    memcpy(org + (size_t)y * stride, src + (size_t)y * sstride, sizeof(int16_t) * (size_t)w);
    for (int x = 0; x < margin; x++) {
      org[(size_t)y * stride - margin + x] = org[(size_t)y * stride];
      org[(size_t)y * stride + w + x] = org[(size_t)y * stride + w - 1];
    }
  }
  for (int y = 0; y < margin; y++) {
    memcpy(org + (size_t)(h + y) * stride - margin, org + (size_t)(h - 1) * stride - margin, sizeof(int16_t) * stride);
    memcpy(org - (size_t)(y + 1) * stride - margin, org - margin, sizeof(int16_t) * stride);
  }
  *out = b;
  *ostride = stride;
}

/* InterPrediction::xPredInterBlkMM (InterPrediction.cpp:683-856) for one component of one list,
 * and (enc = 1) its encoder twin InterSearch::xMVReprojectionInterpolation
 * (EncoderLib/InterSearch.cpp:6277-6385: luma, out-of-range margin maxCUWidth = 0 for both axes).
 * dst: w*h int16 (component units) */
static int pred_blk_mm_x(Orc* o, int comp, const OPic* ref, int x, int y, int w, int h, int mvh, int mvv, int model,
                         int bi, int cur_poc, int16_t* dst, int enc) {
  const int chroma = comp != 0;
  const int sbw = chroma ? 2 : 4, sbh = chroma ? 2 : 4;
  const int rows = h / sbh, cols = w / sbw;
  int32_t* fx = (int32_t*)malloc(sizeof(int32_t) * 2 * (size_t)(rows * cols));
  int rc = reproject(o, x, y, w, h, mvh, mvv, model, comp, cur_poc, ref->poc, fx);
  if (rc) { free(fx); return rc; }
  const int shiftH = 4 + chroma, mask = (1 << shiftH) - 1;
  const int rndRes = !bi;
  const int pi = chroma ? 1 : 0;
  const int refW = o->W >> chroma, refH = o->H >> chroma;
  const int maxCUw = enc ? 0 : o->maxcu_w >> chroma, maxCUh = enc ? 0 : o->maxcu_h >> chroma;
  const int16_t* org = ref->buf[pi] + (size_t)ref->margin[pi] * ref->stride[pi] + ref->margin[pi];
  const ptrdiff_t rs = ref->stride[pi];
  int16_t tmp[(4 + 7) * 4];
  for (int col = 0; col < cols; col++)
    for (int row = 0; row < rows; row++) {
      int i = col * rows + row;
      int xPos = fx[2 * i] >> shiftH, yPos = fx[2 * i + 1] >> shiftH;
      int xFrac = fx[2 * i] & mask, yFrac = fx[2 * i + 1] & mask;
      int16_t* d = dst + (size_t)row * sbh * w + col * sbw;
      if (xPos < -maxCUw || yPos < -maxCUh || xPos >= refW + maxCUw - sbw || yPos >= refH + maxCUh - sbh) {
        for (int r = 0; r < sbh; r++)
          for (int c = 0; c < sbw; c++) d[r * w + c] = 0;
        continue;
      }
      const int16_t* s = org + (ptrdiff_t)yPos * rs + xPos;
      if (yFrac == 0)
        filter_hor(comp, o->bd, s, rs, d, w, sbw, sbh, xFrac, rndRes);
      else if (xFrac == 0)
        filter_ver(comp, o->bd, s, rs, d, w, sbw, sbh, yFrac, 1, rndRes);
      else {
        int vfs = chroma ? 4 : 8;
        filter_hor(comp, o->bd, s - ((vfs >> 1) - 1) * rs, rs, tmp, sbw, sbw, sbh + vfs - 1, xFrac, 0);
        filter_ver(comp, o->bd, tmp + ((vfs >> 1) - 1) * sbw, sbw, d, w, sbw, sbh, yFrac, 0, rndRes);
      }
    }
  free(fx);
  return 0;
}

static int pred_blk_mm(Orc* o, int comp, const OPic* ref, int x, int y, int w, int h, int mvh, int mvv, int model,
                       int bi, int cur_poc, int16_t* dst) {
  return pred_blk_mm_x(o, comp, ref, x, y, w, h, mvh, mvv, model, bi, cur_poc, dst, 0);
}

/* ==========================================================================================
 * Exported oracle API (ctypes)
 * ========================================================================================== */
void* orc_create(const mm_seq_params* p) {
  Orc* o = (Orc*)calloc(1, sizeof(Orc));
  o->W = p->width;
  o->H = p->height;
  o->chroma = p->chroma_format == 1;
  o->Wc = p->width / 2;
  o->Hc = p->height / 2;
  o->bd = p->bit_depth;
  o->maxcu_w = p->max_cu_width;
  o->maxcu_h = p->max_cu_height;
  o->ged_flavor = p->ged_flavor;
  o->active = p->active_models;
  o->off = p->mm_offset4x4 == 4 ? 1.5f : (float)p->mm_offset4x4;
  o->focal = (float)(1. / tan(M_PI / p->height));
  o->res = (float)(M_PI / p->height);
  /* MVReprojection::fillCache + MotionPlaneAdaptiveMotionModel::fillCache on the frame grid
   * (Eigen column-major order: element (j, i) at i*rows + j) */
  const int cols = o->W / 4, rows = o->H / 4, n = cols * rows;
  for (int pl = 0; pl < 3; pl++) {
    if (!(o->active & (1u << (pl + 1)))) continue;
    float *gx = fa(n), *gy = fa(n), *px = fa(n), *py = fa(n);
    unsigned char* vip = (unsigned char*)malloc((size_t)n);
    for (int i = 0; i < cols; i++)
      for (int j = 0; j < rows; j++) {
        gx[i * rows + j] = 4.0f * (float)i + o->off;
        gy[i * rows + j] = 4.0f * (float)j + o->off;
      }
    mpa_to_perspective_arr(o, pl + 1, gx, gy, px, py, vip, n);
    o->mpa_px[pl] = fa(n);
    o->mpa_py[pl] = fa(n);
    o->mpa_vip[pl] = (unsigned char*)malloc((size_t)n);
    for (int i = 0; i < cols; i++)
      for (int j = 0; j < rows; j++) {
        o->mpa_px[pl][j * cols + i] = px[i * rows + j];
        o->mpa_py[pl][j * cols + i] = py[i * rows + j];
        o->mpa_vip[pl][j * cols + i] = vip[i * rows + j];
      }
    free(gx); free(gy); free(px); free(py); free(vip);
  }
  return o;
}

void orc_destroy(void* h) {
  Orc* o = (Orc*)h;
  if (!o) return;
  for (int pl = 0; pl < 3; pl++) { free(o->mpa_px[pl]); free(o->mpa_py[pl]); free(o->mpa_vip[pl]); }
  free(o);
}

int orc_set_epipole(void* h, int cur, int ref, const int32_t* q) {
  Orc* o = (Orc*)h;
  for (int i = 0; i < o->n_epi; i++)
    if (o->epi_key[i][0] == cur && o->epi_key[i][1] == ref) { memcpy(o->epi_q[i], q, 12); return 0; }
  if (o->n_epi >= 256) return MM_ERR_ARG;
  o->epi_key[o->n_epi][0] = cur;
  o->epi_key[o->n_epi][1] = ref;
  memcpy(o->epi_q[o->n_epi], q, 12);
  o->n_epi++;
  return 0;
}

/* mm_reproject twin */
int orc_reproject(void* h, const mm_block_desc* b, int n, int32_t* out) {
  Orc* o = (Orc*)h;
  size_t off = 0;
  for (int i = 0; i < n; i++) {
    int chroma = b[i].comp != 0, sb = chroma ? 2 : 4;
    int rc = reproject(o, b[i].x, b[i].y, b[i].w, b[i].h, b[i].mv_hor, b[i].mv_ver, b[i].model, b[i].comp,
                       b[i].cur_poc, b[i].ref_poc, out + 2 * off);
    if (rc) return rc;
    off += (size_t)(b[i].w / sb) * (size_t)(b[i].h / sb);
  }
  return 0;
}

/* mm_pred twin.  refs: n_refs pictures given as pocs[i] + planes (unpadded host planes). */
/* g_BcwWeights (Rom.cpp:203) and getBcwWeight (Rom.cpp:208-213): w1 = g_BcwWeights[idx], w0 = 8 - w1 */
static const int BCW_WEIGHTS[5] = {-2, 3, 4, 5, 10};

/* One PU: xPredInterUni per list (xPredInterBlkMM per component) + xWeightedAverage
 * (InterPrediction.cpp:1584-1679): addWeightedAvg when bcwIdx != BCW_DEFAULT (:1596-1600,
 * Buffer.cpp:398-424), else addAvg (Buffer.cpp:551-582); uni: copyClip.
 * only_list >= 0: mm_pred_list -- just that list's xPredInterBlkMM(bi = hp) output is written. */
static int pred_pu(Orc* o, const OPic* pics, int n_refs, const mm_pu_desc* u, int cur_poc, int16_t* pred[2][3],
                   int16_t* dy, ptrdiff_t sdy, int16_t* dcb, int16_t* dcr, ptrdiff_t sdc, int only_list, int hp) {
  int rc = 0;
  int bi = u->ref_poc[0] >= 0 && u->ref_poc[1] >= 0;
  if (only_list >= 0) {
    if (u->ref_poc[only_list] < 0) return MM_ERR_ARG;
    bi = hp;
  } else if (bi && (u->bcw_idx < 0 || u->bcw_idx > 4)) {
    return MM_ERR_ARG;
  }
  int ncomp = o->chroma ? 3 : 1;
  for (int l = 0; l < 2 && !rc; l++) {
    if (u->ref_poc[l] < 0 || (only_list >= 0 && l != only_list)) continue;
    const OPic* ref = NULL;
    for (int r = 0; r < n_refs; r++)
      if (pics[r].poc == u->ref_poc[l]) ref = &pics[r];
    if (!ref) return MM_ERR_NOREF;
    for (int c = 0; c < ncomp && !rc; c++) {
      int cs = c ? 1 : 0;
      OPic tmp = *ref;
      if (c == 2) { tmp.buf[1] = ref->buf[2]; tmp.stride[1] = ref->stride[2]; tmp.margin[1] = ref->margin[2]; }
      rc = pred_blk_mm(o, c, &tmp, u->x >> cs, u->y >> cs, u->w >> cs, u->h >> cs, u->mv[l][0], u->mv[l][1],
                       u->model[l], bi, cur_poc, pred[l][c]);
    }
  }
  for (int c = 0; c < ncomp && !rc; c++) {
    int cs = c ? 1 : 0, w = u->w >> cs, hh = u->h >> cs;
    int16_t* d = c == 0 ? dy : (c == 1 ? dcb : dcr);
    ptrdiff_t ds = c == 0 ? sdy : sdc;
    d += (ptrdiff_t)(u->y >> cs) * ds + (u->x >> cs);
    for (int y = 0; y < hh; y++)
      for (int x = 0; x < w; x++) {
        int k = y * w + x;
        if (only_list >= 0) { /* the PelUnitBuf xPredInterBlkMM wrote */
          d[y * ds + x] = pred[only_list][c][k];
        } else if (bi && u->bcw_idx != 2) { /* AreaBuf<Pel>::addWeightedAvg */
          int w1 = BCW_WEIGHTS[u->bcw_idx], w0 = 8 - w1;
          int shiftNum = frac_bits(o->bd) + 3, offset = (1 << (shiftNum - 1)) + (8192 << 3);
          d[y * ds + x] = clip_pel((pred[0][c][k] * w0 + pred[1][c][k] * w1 + offset) >> shiftNum, o->bd);
        } else if (bi) { /* AreaBuf<Pel>::addAvg */
          int shiftNum = frac_bits(o->bd) + 1, offset = (1 << (shiftNum - 1)) + 2 * 8192;
          d[y * ds + x] = clip_pel((pred[0][c][k] + pred[1][c][k] + offset) >> shiftNum, o->bd);
        } else { /* copyClip */
          int l = u->ref_poc[0] >= 0 ? 0 : 1;
          d[y * ds + x] = clip_pel(pred[l][c][k], o->bd);
        }
      }
  }
  return rc;
}

static OPic* pad_refs(Orc* o, int n_refs, const int32_t* pocs, const int16_t* const* ys, const int16_t* const* cbs,
                      const int16_t* const* crs, ptrdiff_t stride_y, ptrdiff_t stride_c) {
  OPic* pics = (OPic*)calloc((size_t)n_refs, sizeof(OPic));
  const int margin = 2 * (o->maxcu_w + 16);
  for (int r = 0; r < n_refs; r++) {
    pics[r].poc = pocs[r];
    pad_plane(ys[r], stride_y, o->W, o->H, margin, &pics[r].buf[0], &pics[r].stride[0]);
    pics[r].margin[0] = margin;
    if (o->chroma && cbs) {
      pad_plane(cbs[r], stride_c, o->Wc, o->Hc, margin / 2, &pics[r].buf[1], &pics[r].stride[1]);
      pad_plane(crs[r], stride_c, o->Wc, o->Hc, margin / 2, &pics[r].buf[2], &pics[r].stride[2]);
      pics[r].margin[1] = pics[r].margin[2] = margin / 2;
    }
  }
  return pics;
}

static void free_refs(OPic* pics, int n_refs) {
  for (int r = 0; r < n_refs; r++)
    for (int c = 0; c < 3; c++) free(pics[r].buf[c]);
  free(pics);
}

static int pred_list_all(void* h, int cur_poc, const mm_pu_desc* pus, int n, int n_refs, const int32_t* pocs,
                         const int16_t* const* ys, const int16_t* const* cbs, const int16_t* const* crs,
                         ptrdiff_t stride_y, ptrdiff_t stride_c, int16_t* dy, ptrdiff_t sdy, int16_t* dcb, int16_t* dcr,
                         ptrdiff_t sdc, int only_list, int hp) {
  Orc* o = (Orc*)h;
  OPic* pics = pad_refs(o, n_refs, pocs, ys, cbs, crs, stride_y, stride_c);
  int rc = 0;
  int16_t* pred[2][3];
  for (int l = 0; l < 2; l++)
    for (int c = 0; c < 3; c++) pred[l][c] = (int16_t*)malloc(sizeof(int16_t) * 128 * 128);
  for (int i = 0; i < n && !rc; i++)
    rc = pred_pu(o, pics, n_refs, &pus[i], cur_poc, pred, dy, sdy, dcb, dcr, sdc, only_list, hp);
  for (int l = 0; l < 2; l++)
    for (int c = 0; c < 3; c++) free(pred[l][c]);
  free_refs(pics, n_refs);
  return rc;
}

int orc_pred(void* h, int cur_poc, const mm_pu_desc* pus, int n, int n_refs, const int32_t* pocs,
             const int16_t* const* ys, const int16_t* const* cbs, const int16_t* const* crs, ptrdiff_t stride_y,
             ptrdiff_t stride_c, int16_t* dy, ptrdiff_t sdy, int16_t* dcb, int16_t* dcr, ptrdiff_t sdc) {
  return pred_list_all(h, cur_poc, pus, n, n_refs, pocs, ys, cbs, crs, stride_y, stride_c, dy, sdy, dcb, dcr, sdc, -1,
                       0);
}

/* mm_pred_list twin: xPredInterBlkMM (InterPrediction.cpp:683-856) of list `list` of every PU,
 * bi = hp (14-bit intermediate) or rounded + clipped. */
int orc_pred_list(void* h, int cur_poc, const mm_pu_desc* pus, int n, int list, int hp, int n_refs,
                  const int32_t* pocs, const int16_t* const* ys, const int16_t* const* cbs,
                  const int16_t* const* crs, ptrdiff_t stride_y, ptrdiff_t stride_c, int16_t* dy, ptrdiff_t sdy,
                  int16_t* dcb, int16_t* dcr, ptrdiff_t sdc) {
  return pred_list_all(h, cur_poc, pus, n, n_refs, pocs, ys, cbs, crs, stride_y, stride_c, dy, sdy, dcb, dcr, sdc,
                       list, hp);
}

/* ---- MM-DMVR: InterPrediction::xProcessDMVRProjected (InterPrediction.cpp:2442-2634) ---- */

/* xDMVRCost (:2147-2155): RdCost SAD with subShift 1 (even rows, sum <<= 1), then >> 1 */
static uint64_t dmvr_cost(const int16_t* p0, const int16_t* p1, int w, int h) {
  uint64_t sum = 0;
  for (int y = 0; y < h; y += 2)
    for (int x = 0; x < w; x++) {
      int d = p0[y * w + x] - p1[y * w + x];
      sum += (uint64_t)(d < 0 ? -d : d);
    }
  return (sum << 1) >> 1;
}

static int32_t div_for_maxq7(int64_t N, int64_t D) { /* :1958-1994 */
  int32_t sign = 0, q = 0;
  if (N < 0) { sign = 1; N = -N; }
  D = D << 3;
  if (N >= D) { N -= D; q++; }
  q = q << 1;
  D = D >> 1;
  if (N >= D) { N -= D; q++; }
  q = q << 1;
  if (N >= (D >> 1)) q++;
  return sign ? -q : q;
}

static void sub_pel_error_srfc(const uint64_t* sadBuffer, int32_t* deltaMv) { /* :1996-2048 */
  int64_t numerator, denominator;
  numerator = (int64_t)((sadBuffer[1] - sadBuffer[3]) << 4);
  denominator = (int64_t)((sadBuffer[1] + sadBuffer[3] - (sadBuffer[0] << 1)));
  if (0 != denominator) {
    if ((sadBuffer[1] != sadBuffer[0]) && (sadBuffer[3] != sadBuffer[0])) deltaMv[0] = div_for_maxq7(numerator, denominator);
    else deltaMv[0] = (sadBuffer[1] == sadBuffer[0]) ? -8 : 8;
  }
  numerator = (int64_t)((sadBuffer[2] - sadBuffer[4]) << 4);
  denominator = (int64_t)((sadBuffer[2] + sadBuffer[4] - (sadBuffer[0] << 1)));
  if (0 != denominator) {
    if ((sadBuffer[2] != sadBuffer[0]) && (sadBuffer[4] != sadBuffer[0])) deltaMv[1] = div_for_maxq7(numerator, denominator);
    else deltaMv[1] = (sadBuffer[2] == sadBuffer[0]) ? -8 : 8;
  }
}

static int clip_mv18(int v) { return v < -(1 << 17) ? -(1 << 17) : (v > (1 << 17) - 1 ? (1 << 17) - 1 : v); }

/* Branch trace of one sub-PU's decision (orc_pred_dmvr_trace; tests assert that every branch of
 * :2516-2531 and :1996-2048 is reached): bit 0 early exit (minCost < dx*dy, notZeroCost = false);
 * bits 1-5 the best offset index; bit 6 best on the window border (no error surface); bits 8-9 / 10-11
 * the horizontal / vertical error-surface case: 0 denominator 0 (no change), 1 div_for_maxq7,
 * 2 SAD tie on the -1 side (-8, half pel), 3 tie on the +1 side (+8).  The `!minCost` exit (:2528-2531)
 * is unreachable in the reference's single iteration: it follows the minCost >= dx*dy > 0 test. */
#define DMVR_TR_EARLY 1
#define DMVR_TR_BORDER 64
static int surface_case(const uint64_t* s, int a, int b) {
  const int64_t den = (int64_t)(s[a] + s[b] - (s[0] << 1));
  if (den == 0) return 0;
  if (s[a] != s[0] && s[b] != s[0]) return 1;
  return s[a] == s[0] ? 2 : 3;
}
static int pred_dmvr_impl(void* h, int cur_poc, const mm_pu_desc* pus, int n, int n_refs, const int32_t* pocs,
                          const int16_t* const* ys, const int16_t* const* cbs, const int16_t* const* crs,
                          ptrdiff_t stride_y, ptrdiff_t stride_c, int16_t* dy, ptrdiff_t sdy, int16_t* dcb,
                          int16_t* dcr, ptrdiff_t sdc, int32_t* mvd_out, int32_t* trace) {
  Orc* o = (Orc*)h;
  OPic* pics = pad_refs(o, n_refs, pocs, ys, cbs, crs, stride_y, stride_c);
  int rc = 0, k = 0;
  int16_t* pred[2][3];
  for (int l = 0; l < 2; l++)
    for (int c = 0; c < 3; c++) pred[l][c] = (int16_t*)malloc(sizeof(int16_t) * 128 * 128);
  int16_t* s0 = (int16_t*)malloc(sizeof(int16_t) * 16 * 16);
  int16_t* s1 = (int16_t*)malloc(sizeof(int16_t) * 16 * 16);
  for (int i = 0; i < n && !rc; i++) {
    const mm_pu_desc* u = &pus[i];
    const OPic *r0 = NULL, *r1 = NULL;
    for (int r = 0; r < n_refs; r++) {
      if (pics[r].poc == u->ref_poc[0]) r0 = &pics[r];
      if (pics[r].poc == u->ref_poc[1]) r1 = &pics[r];
    }
    if (!r0 || !r1) { rc = MM_ERR_NOREF; break; }
    if (u->bcw_idx != 2) { rc = MM_ERR_ARG; break; } /* checkDMVRCondition: BCW_DEFAULT (UnitTools.cpp:1719) */
    const int dxs = u->w < 16 ? u->w : 16, dys = u->h < 16 ? u->h : 16, model = u->model[0];
    for (int y = u->y; y < u->y + u->h && !rc; y += dys)
      for (int x = u->x; x < u->x + u->w && !rc; x += dxs) {
        uint64_t sads[25];
        for (int j = 0; j < 25; j++) sads[j] = UINT64_MAX;
        int tdx = 0, tdy = 0, notZeroCost = 1;
        rc = pred_blk_mm(o, 0, r0, x, y, dxs, dys, u->mv[0][0], u->mv[0][1], model, 1, cur_poc, s0);
        if (!rc) rc = pred_blk_mm(o, 0, r1, x, y, dxs, dys, u->mv[1][0], u->mv[1][1], model, 1, cur_poc, s1);
        uint64_t minCost = dmvr_cost(s0, s1, dxs, dys);
        minCost -= (minCost >> 2);
        if (minCost < (uint64_t)(dxs * dys)) notZeroCost = 0;
        int best = 12, tr = notZeroCost ? 0 : DMVR_TR_EARLY;
        if (notZeroCost) {
          sads[12] = minCost;
          for (int j = 0; j < 25 && !rc; j++) {
            const int ox = j % 5 - 2, oy = j / 5 - 2;
            rc = pred_blk_mm(o, 0, r0, x, y, dxs, dys, u->mv[0][0] + ox * 16, u->mv[0][1] + oy * 16, model, 1, cur_poc, s0);
            if (!rc) rc = pred_blk_mm(o, 0, r1, x, y, dxs, dys, u->mv[1][0] - ox * 16, u->mv[1][1] - oy * 16, model, 1, cur_poc, s1);
            if (sads[j] == UINT64_MAX) sads[j] = dmvr_cost(s0, s1, dxs, dys);
            if (sads[j] < minCost) { minCost = sads[j]; best = j; }
          }
          tdx = (best % 5 - 2) << 4;
          tdy = (best / 5 - 2) << 4;
          tr |= best << 1;
          if (abs(tdx) != 32 && abs(tdy) != 32) {
            uint64_t sb[5] = {sads[best], sads[best - 1], sads[best - 5], sads[best + 1], sads[best + 5]};
            int32_t d[2] = {0, 0};
            sub_pel_error_srfc(sb, d);
            tdx += d[0];
            tdy += d[1];
            tr |= surface_case(sb, 1, 3) << 8 | surface_case(sb, 2, 4) << 10;
          } else {
            tr |= DMVR_TR_BORDER;
          }
        }
        if (mvd_out) { mvd_out[2 * k] = tdx; mvd_out[2 * k + 1] = tdy; }
        if (trace) trace[k] = tr;
        k++;
        mm_pu_desc sp = *u;
        sp.x = x; sp.y = y; sp.w = dxs; sp.h = dys;
        sp.mv[0][0] = clip_mv18(u->mv[0][0] + tdx); sp.mv[0][1] = clip_mv18(u->mv[0][1] + tdy);
        sp.mv[1][0] = clip_mv18(u->mv[1][0] - tdx); sp.mv[1][1] = clip_mv18(u->mv[1][1] - tdy);
        if (!rc) rc = pred_pu(o, pics, n_refs, &sp, cur_poc, pred, dy, sdy, dcb, dcr, sdc, -1, 0);
      }
  }
  free(s0);
  free(s1);
  for (int l = 0; l < 2; l++)
    for (int c = 0; c < 3; c++) free(pred[l][c]);
  free_refs(pics, n_refs);
  return rc;
}

int orc_pred_dmvr(void* h, int cur_poc, const mm_pu_desc* pus, int n, int n_refs, const int32_t* pocs,
                  const int16_t* const* ys, const int16_t* const* cbs, const int16_t* const* crs, ptrdiff_t stride_y,
                  ptrdiff_t stride_c, int16_t* dy, ptrdiff_t sdy, int16_t* dcb, int16_t* dcr, ptrdiff_t sdc,
                  int32_t* mvd_out) {
  return pred_dmvr_impl(h, cur_poc, pus, n, n_refs, pocs, ys, cbs, crs, stride_y, stride_c, dy, sdy, dcb, dcr, sdc,
                        mvd_out, NULL);
}
int orc_pred_dmvr_trace(void* h, int cur_poc, const mm_pu_desc* pus, int n, int n_refs, const int32_t* pocs,
                        const int16_t* const* ys, const int16_t* const* cbs, const int16_t* const* crs,
                        ptrdiff_t stride_y, ptrdiff_t stride_c, int16_t* dy, ptrdiff_t sdy, int16_t* dcb, int16_t* dcr,
                        ptrdiff_t sdc, int32_t* mvd_out, int32_t* trace) {
  return pred_dmvr_impl(h, cur_poc, pus, n, n_refs, pocs, ys, cbs, crs, stride_y, stride_c, dy, sdy, dcb, dcr, sdc,
                        mvd_out, trace);
}

/* mm_filter twin: raw filterHor / filterVer on a host block with margin */
int orc_filter(int comp, int vertical, int bd, const int16_t* src, ptrdiff_t ss, int16_t* dst, ptrdiff_t ds, int w, int h,
               int frac, int first, int last) {
  if (vertical)
    filter_ver(comp, bd, src, ss, dst, ds, w, h, frac, first, last);
  else {
    if (!first) return MM_ERR_ARG; /* filterHor is always isFirst (InterpolationFilter.cpp:658) */
    filter_hor(comp, bd, src, ss, dst, ds, w, h, frac, last);
  }
  return 0;
}

/* Encoder candidate windows (mm_sad_window twin): for each block and candidate (i, j) in
 * [-range, range]^2, xMVReprojectionInterpolation with rndRes = true (InterSearch.h:555-566) and
 * RdCost::xGetSAD (RdCost.cpp:482-517: rows stepped by 1 << subShift, sum <<= subShift,
 * FULL_NBIT so no distortion shift; the early exit only truncates values above the running best
 * and is not modelled). */
int orc_sad_window(void* h, int cur_poc, const mm_me_block* blocks, int n, int range, int step, int n_refs,
                   const int32_t* pocs, const int16_t* const* ys, ptrdiff_t stride_y, const int16_t* org,
                   ptrdiff_t org_stride, uint32_t* sads) {
  Orc* o = (Orc*)h;
  OPic* pics = (OPic*)calloc((size_t)n_refs, sizeof(OPic));
  const int margin = 2 * (o->maxcu_w + 16);
  for (int r = 0; r < n_refs; r++) {
    pics[r].poc = pocs[r];
    pad_plane(ys[r], stride_y, o->W, o->H, margin, &pics[r].buf[0], &pics[r].stride[0]);
    pics[r].margin[0] = margin;
  }
  const int side = 2 * range + 1, C = side * side;
  int16_t* pred = (int16_t*)malloc(sizeof(int16_t) * 128 * 128);
  int rc = 0;
  for (int b = 0; b < n && !rc; b++) {
    const mm_me_block* k = &blocks[b];
    const OPic* ref = NULL;
    for (int r = 0; r < n_refs; r++)
      if (pics[r].poc == k->ref_poc) ref = &pics[r];
    if (!ref) { rc = MM_ERR_NOREF; break; }
    for (int c = 0; c < C && !rc; c++) {
      const int i = c % side - range, j = c / side - range;
      rc = pred_blk_mm_x(o, 0, ref, k->x, k->y, k->w, k->h, k->mv_hor + i * step, k->mv_ver + j * step, k->model, 0,
                         cur_poc, pred, 1);
      uint64_t sum = 0;
      const int sub = 1 << k->sub_shift;
      for (int y = 0; y < k->h; y += sub)
        for (int x = 0; x < k->w; x++) {
          int d = org[(ptrdiff_t)(k->y + y) * org_stride + k->x + x] - pred[y * k->w + x];
          sum += (uint64_t)(d < 0 ? -d : d);
        }
      sads[(size_t)b * C + c] = (uint32_t)(sum << k->sub_shift);
    }
  }
  free(pred);
  for (int r = 0; r < n_refs; r++) free(pics[r].buf[0]);
  free(pics);
  return rc;
}

/* ==========================================================================================
 * MM-MVP: MVReprojection::motionVectorInDesiredMotionModel (MVReprojection.cpp:168-217)
 * ========================================================================================== */

/* scalar EquirectangularProjection::fromSphere(Array3TCoord) (Projection.cpp, scalar overload) */
static void erp_from_sphere1(const Orc* o, float X, float Y, float Z, float* x, float* y) {
  float R, th, ph;
  c2s_scalar(X, Y, Z, &R, &th, &ph);
  ph = ph > 0 ? ph - 2.0f * PI_F : ph;
  *x = -(ph / (2.0f * PI_F)) * (float)o->W - 0.0f;
  *y = (th / PI_F) * (float)o->H - 0.0f;
}

/* scalar MotionPlaneAdaptiveMotionModel::toPerspective (:137-161) with the scalar
 * PerspectiveProjection::fromSphere (optical centre 0) */
static void mpa_to_perspective1(const Orc* o, int plane, float x, float y, float* px, float* py, int* vip) {
  float X, Y, Z;
  erp_to_sphere1(o, x, y, &X, &Y, &Z);
  float mx, my, mz;
  if (plane == 1) { mx = X; my = Y; mz = Z; }
  else if (plane == 2) { mx = Y; my = -X; mz = Z; }
  else { mx = -Z; my = Y; mz = X; }
  float R, th, ph;
  c2s_scalar(my, -mz, -mx, &R, &th, &ph);
  float polarR = o->focal * tanf(th);
  *px = polarR * cosf(ph) + 0.0f;
  *py = polarR * sinf(ph) + 0.0f;
  *vip = polarR < 0;
}

static void rot_apply(const float* M, float x, float y, float z, float* ox, float* oy, float* oz) {
  *ox = dot3(M[0], x, M[1], y, M[2], z);
  *oy = dot3(M[3], x, M[4], y, M[5], z);
  *oz = dot3(M[6], x, M[7], y, M[8], z);
}

/* <Model>::motionVectorForEquivalentPixelShiftAt, scalar code of each model file */
static void equivalent_mv(const Orc* o, int model, const float* Rm, float px, float py, float sx, float sy, float cx,
                          float cy, float* mvx, float* mvy) {
  float R, th, ph;
  switch (model) {
    case 0: *mvx = sx - px; *mvy = sy - py; return;
    case 1: case 2: case 3: {
      float ox, oy, qx, qy;
      int vo, vq;
      mpa_to_perspective1(o, model, px, py, &ox, &oy, &vo);
      mpa_to_perspective1(o, model, sx, sy, &qx, &qy, &vq);
      if (vo != vq) { *mvx = 0; *mvy = 0; return; }
      float sgn = vq ? -1.0f : 1.0f;
      *mvx = (qx - ox) * sgn;
      *mvy = (qy - oy) * sgn;
      return;
    }
    case 4: {
      float X, Y, Z, thc, phc;
      erp_to_sphere1(o, cx, cy, &X, &Y, &Z);
      c2s_scalar(X, Y, Z, &R, &thc, &phc);
      const float epsC = (float)M_PI_2 - thc, alphaC = phc;
      float xs[2], ys[2];
      float pts[2][2] = {{px, py}, {sx, sy}};
      for (int k = 0; k < 2; k++) {
        erp_to_sphere1(o, pts[k][0], pts[k][1], &X, &Y, &Z);
        c2s_scalar(X, Y, Z, &R, &th, &ph);
        float eps = (float)M_PI_2 - th, dA = ph - alphaC;
        float cosPsi = sinf(epsC) * sinf(eps) + cosf(epsC) * cosf(eps) * cosf(dA);
        ys[k] = (sinf(eps) * cosf(epsC) - sinf(epsC) * cosf(eps) * cosf(dA)) / cosPsi;
        xs[k] = (sinf(dA) * cosf(eps)) / cosPsi;
      }
      *mvx = (xs[0] - xs[1]) / o->res;
      *mvy = (ys[0] - ys[1]) / o->res;
      return;
    }
    case 5: {
      float Xc, Yc, Zc, X, Y, Z, Xm, Ym, Zm, ox, oy;
      erp_to_sphere1(o, cx, cy, &Xc, &Yc, &Zc);
      erp_to_sphere1(o, px, py, &X, &Y, &Z);
      erp_to_sphere1(o, sx, sy, &Xm, &Ym, &Zm);
      erp_from_sphere1(o, Xm - X + Xc, Ym - Y + Yc, Zm - Z + Zc, &ox, &oy);
      *mvx = ox - cx;
      *mvy = oy - cy;
      return;
    }
    case 6: {
      float X, Y, Z, thc, phc;
      erp_to_sphere1(o, cx, cy, &X, &Y, &Z);
      c2s_scalar(X, Y, Z, &R, &thc, &phc);
      const float uz[3] = {0, 0, 1}, uy[3] = {0, 1, 0};
      float uphi[9], uth[9], M[9];
      angle_axis(-phc, uz, uphi);
      angle_axis((float)(M_PI_2 - thc), uy, uth);
      matmul3(uth, uphi, M);
      float a[3], b[3], t1, p1, t2, p2;
      erp_to_sphere1(o, px, py, &X, &Y, &Z);
      rot_apply(M, X, Y, Z, &a[0], &a[1], &a[2]);
      erp_to_sphere1(o, sx, sy, &X, &Y, &Z);
      rot_apply(M, X, Y, Z, &b[0], &b[1], &b[2]);
      c2s_scalar(a[0], a[1], a[2], &R, &t1, &p1);
      c2s_scalar(b[0], b[1], b[2], &R, &t2, &p2);
      *mvx = (p1 - p2) / o->res;
      *mvy = (t2 - t1) / o->res;
      return;
    }
    default: { /* 7..10 geodesic */
      float X, Y, Z, a[3], t1, p1, t2, p2;
      erp_to_sphere1(o, px, py, &X, &Y, &Z);
      rot_apply(Rm, X, Y, Z, &a[0], &a[1], &a[2]);
      c2s_scalar(a[0], a[1], a[2], &R, &t1, &p1);
      erp_to_sphere1(o, sx, sy, &X, &Y, &Z);
      rot_apply(Rm, X, Y, Z, &a[0], &a[1], &a[2]);
      c2s_scalar(a[0], a[1], a[2], &R, &t2, &p2);
      if (o->ged_flavor == 0) {
        *mvx = (t2 - t1) / o->res;
      } else {
        float tc, pc;
        erp_to_sphere1(o, cx, cy, &X, &Y, &Z);
        rot_apply(Rm, X, Y, Z, &a[0], &a[1], &a[2]);
        c2s_scalar(a[0], a[1], a[2], &R, &tc, &pc);
        float dTheta = t2 - t1;
        float k = sinf(dTheta + t1) / sinf(dTheta);
        float dThetaC = atanf(sinf(tc) / (k - cosf(tc)));
        *mvx = dThetaC / o->res;
      }
      *mvy = (p2 - p1) / o->res;
      return;
    }
  }
}

int orc_mvp(void* h, const mm_mvp_query* qs, int n, int32_t* out) {
  Orc* o = (Orc*)h;
  for (int i = 0; i < n; i++) {
    const mm_mvp_query* q = &qs[i];
    int32_t* r = out + 2 * i;
    if (q->mv_hor == 0 && q->mv_ver == 0) { r[0] = r[1] = 0; continue; }
    float eo[3] = {0, 0, 0}, ed[3] = {0, 0, 0};
    int have_o = 0, have_d = 0;
    if (q->model_orig == 10) { if (find_epipole(o, q->cur_poc_orig, q->ref_poc_orig, eo)) return MM_ERR_NOEPIPOLE; have_o = 1; }
    if (q->model_desired == 10) { if (find_epipole(o, q->cur_poc_desired, q->ref_poc_desired, ed)) return MM_ERR_NOEPIPOLE; have_d = 1; }
    if (q->model_desired == q->model_orig &&
        (q->model_desired != 10 || (have_o && have_d && eo[0] == ed[0] && eo[1] == ed[1] && eo[2] == ed[2]))) {
      r[0] = q->mv_hor;
      r[1] = q->mv_ver;
      continue;
    }
    const float mvX = (float)(q->mv_hor >> q->shift_hor) + (float)(q->mv_hor & ((1 << q->shift_hor) - 1)) / (float)(1 << q->shift_hor);
    const float mvY = (float)(q->mv_ver >> q->shift_ver) + (float)(q->mv_ver & ((1 << q->shift_ver) - 1)) / (float)(1 << q->shift_ver);
    const float ccx = (float)q->cand_x + ((float)q->cand_w - 1) / 2.0f, ccy = (float)q->cand_y + ((float)q->cand_h - 1) / 2.0f;
    float gx = (float)q->pos_x, gy = (float)q->pos_y, sx, sy;
    float Rm[9];
    switch (q->model_orig) { /* the candidate's modelMotion on a 1x1 array */
      case 0: sx = gx + mvX; sy = gy + mvY; break;
      case 1: case 2: case 3: {
        float ppx, ppy;
        unsigned char vip;
        mpa_to_perspective_arr(o, q->model_orig, &gx, &gy, &ppx, &ppy, &vip, 1);
        float sgn = vip ? -1.0f : 1.0f;
        ppx = ppx + mvX * sgn;
        ppy = ppy + mvY * sgn;
        mpa_to_projection_arr(o, q->model_orig, &ppx, &ppy, &vip, &sx, &sy, 1);
      } break;
      case 4: tan_model(o, &gx, &gy, 1, mvX, mvY, ccx, ccy, &sx, &sy); break;
      case 5: t3d_model(o, &gx, &gy, 1, mvX, mvY, ccx, ccy, &sx, &sy); break;
      case 6: rot_model(o, &gx, &gy, 1, mvX, mvY, ccx, ccy, &sx, &sy); break;
      default: {
        float e[3] = {1, 0, 0};
        if (q->model_orig == 8) { e[0] = 0; e[1] = 1; }
        else if (q->model_orig == 9) { e[0] = 0; e[2] = 1; }
        else if (q->model_orig == 10) { e[0] = eo[0]; e[1] = eo[1]; e[2] = eo[2]; }
        ged_set_epipole(e, Rm);
        ged_model(o, Rm, &gx, &gy, 1, mvX, mvY, ccx, ccy, &sx, &sy);
      }
    }
    if (q->model_desired >= 7) {
      float e[3] = {1, 0, 0};
      if (q->model_desired == 8) { e[0] = 0; e[1] = 1; }
      else if (q->model_desired == 9) { e[0] = 0; e[2] = 1; }
      else if (q->model_desired == 10) { e[0] = ed[0]; e[1] = ed[1]; e[2] = ed[2]; }
      ged_set_epipole(e, Rm);
    }
    const float cx = (float)q->cur_x + ((float)q->cur_w - 1) / 2.0f, cy = (float)q->cur_y + ((float)q->cur_h - 1) / 2.0f;
    float ex, ey;
    equivalent_mv(o, q->model_desired, Rm, (float)q->pos_x, (float)q->pos_y, sx, sy, cx, cy, &ex, &ey);
    if (isnan(ex) || isnan(ey)) { r[0] = r[1] = 0; continue; }
    float rx = roundf(ex * (float)(1 << q->shift_hor)), ry = roundf(ey * (float)(1 << q->shift_ver));
    r[0] = _mm_cvtt_ss2si(_mm_set_ss(rx));
    r[1] = _mm_cvtt_ss2si(_mm_set_ss(ry));
  }
  return 0;
}

/* ==========================================================================================
 * EpipoleList (SRC/EpipoleList.{h,cpp}) -- entries kept sorted by (curPOC, refPOC) like the
 * reference's std::map; Q24 fixed point.
 * ========================================================================================== */
typedef struct {
  int n;
  int key[512][2];
  int32_t q[512][3];
  int avail[512];
} OEpi;

static int oepi_index(const OEpi* e, int cur, int ref) {
  for (int i = 0; i < e->n; i++)
    if (e->key[i][0] == cur && e->key[i][1] == ref) return i;
  return -1;
}

/* addEpipole (:8-11): m_epipoleMap[{curPOC, refPOC}] = entry */
int orc_epi_add(void* h, int cur, int ref, const int32_t* q, int make_available) {
  OEpi* e = (OEpi*)h;
  int i = oepi_index(e, cur, ref);
  if (i < 0) {
    if (e->n >= 512) return MM_ERR_ARG;
    i = e->n;
    while (i > 0 && (e->key[i - 1][0] > cur || (e->key[i - 1][0] == cur && e->key[i - 1][1] > ref))) {
      memcpy(e->key[i], e->key[i - 1], sizeof(e->key[i]));
      memcpy(e->q[i], e->q[i - 1], sizeof(e->q[i]));
      e->avail[i] = e->avail[i - 1];
      i--;
    }
    e->n++;
    e->key[i][0] = cur;
    e->key[i][1] = ref;
  }
  memcpy(e->q[i], q, 12);
  e->avail[i] = make_available != 0;
  return 0;
}

/* EpipoleList() : addEpipole({0, 0, 0}) -- global, not available (EpipoleList.h:15-17) */
void* orc_epi_create(void) {
  OEpi* e = (OEpi*)calloc(1, sizeof(OEpi));
  const int32_t z[3] = {0, 0, 0};
  orc_epi_add(e, -1, -1, z, 0);
  return e;
}
void orc_epi_destroy(void* h) { free(h); }

/* findEpipoleFixed (:19-36) */
int orc_epi_find(void* h, int cur, int ref, int32_t* out) {
  const OEpi* e = (const OEpi*)h;
  int i = oepi_index(e, cur, ref);
  if (i < 0 || !e->avail[i]) i = oepi_index(e, cur, -1);
  if (i >= 0 && !e->avail[i]) i = -1;
  if (i < 0) i = oepi_index(e, -1, -1);
  if (i < 0 || !e->avail[i]) return MM_ERR_NOEPIPOLE;
  memcpy(out, e->q[i], 12);
  return 0;
}

/* hasEpipole (:82-89) */
int orc_epi_has(void* h, int cur, int ref) {
  const OEpi* e = (const OEpi*)h;
  int i = oepi_index(e, cur, ref);
  return i >= 0 && e->avail[i];
}

/* makeAvailable (:91-99) */
void orc_epi_make_available(void* h, int cur) {
  OEpi* e = (OEpi*)h;
  for (int i = 0; i < e->n; i++)
    if (e->key[i][0] == cur) e->avail[i] = 1;
}

/* FloatingFixedConversion::fixedToFloating / floatingToFixed (Coordinate.cpp:70-92) */
static float fx2fl(int32_t v) { return (float)(v >> 24) + (float)(v & ((1 << 24) - 1)) / (float)(1 << 24); }
static int32_t fl2fx(float f) { return (int32_t)roundf(f * (float)(1 << 24)); }

/* derivePredictor (:38-80) + DecLib.cpp:3138 floatingToFixed */
int orc_epi_predictor(void* h, int cur, int32_t* out) {
  const OEpi* e = (const OEpi*)h;
  int g = oepi_index(e, -1, -1);
  if (g < 0 || !e->avail[g]) return MM_ERR_NOEPIPOLE; /* CHECK(!globalEpipoleEntry.isAvailable) */
  int minPOCDistances[2] = {INT_MAX, INT_MAX};
  int32_t predictors[2][3];
  memcpy(predictors[0], e->q[g], 12);
  memcpy(predictors[1], e->q[g], 12);
  for (int i = 0; i < e->n; i++) {
    if (!e->avail[i]) continue;
    int distance = abs(cur - e->key[i][0]);
    if (distance < minPOCDistances[0]) {
      minPOCDistances[0] = distance;
      memcpy(predictors[0], e->q[i], 12);
    } else if (distance < minPOCDistances[1]) {
      minPOCDistances[1] = distance;
      memcpy(predictors[1], e->q[i], 12);
    }
  }
  int32_t predictor[3];
  if (minPOCDistances[0] == minPOCDistances[1]) {
    for (int k = 0; k < 3; k++) predictor[k] = predictors[0][k] + predictors[1][k] / 2; /* as written (:71) */
  } else {
    if (minPOCDistances[0] > minPOCDistances[1]) return MM_ERR_ARG;
    memcpy(predictor, predictors[0], 12);
  }
  for (int k = 0; k < 3; k++) out[k] = fl2fx(fx2fl(predictor[k]));
  return 0;
}

int orc_epi_count(void* h) {
  const OEpi* e = (const OEpi*)h;
  int g = oepi_index(e, -1, -1);
  int def = g >= 0 && e->q[g][0] == 0 && e->q[g][1] == 0 && e->q[g][2] == 0;
  return e->n - def;
}

/* ==========================================================================================
 * InterPrediction::motionCompensation (InterPrediction.cpp:1681-1810) for MM PUs: the blocks it
 * hands to xPredInterBlkMM (via xPredInterUni / xPredInterBi) and the DMVR decision.
 * ========================================================================================== */
typedef struct {
  const mm_tool_flags* tools;
  mm_pu_desc *mc, *dmvr;
  int n_mc, n_dmvr, cap_mc, cap_dmvr;
} OEff;

/* PU::isBiPredFromDifferentDirEqDistPoc (UnitTools.cpp:4466-4487) */
static int o_bi_dd_eq(const mm_pu_desc* pu, int poc, unsigned flags) {
  if (pu->ref_poc[0] >= 0 && pu->ref_poc[1] >= 0) {
    if (flags & MM_PU_LONGTERM) return 0;
    const int poc0 = pu->ref_poc[0], poc1 = pu->ref_poc[1];
    if ((poc - poc0) * (poc - poc1) < 0)
      if (abs(poc - poc0) == abs(poc - poc1)) return 1;
  }
  return 0;
}

/* PU::checkDMVRCondition (UnitTools.cpp:1698-1726) */
static int o_check_dmvr(const OEff* x, const mm_pu_desc* pu, int poc, unsigned flags, int merge_type_default) {
  if (!x->tools->dmvr) return 0;
  return (flags & MM_PU_MERGE) && merge_type_default && !(flags & MM_PU_CIIP) && !(flags & MM_PU_MMVD) &&
         pu->model[0] == pu->model[1] && o_bi_dd_eq(pu, poc, flags) && pu->h >= 8 && pu->w >= 8 &&
         pu->h * pu->w >= 128 && pu->bcw_idx == 2 && !(flags & MM_PU_WEIGHTED) && !(flags & MM_PU_REF_SCALED);
}

static void o_emit(OEff* x, const mm_pu_desc* pu, int to_dmvr) {
  mm_pu_desc d = *pu;
  d.flags = 0;
  d.reserved[0] = d.reserved[1] = 0;
  if (to_dmvr) {
    if (x->n_dmvr < x->cap_dmvr) x->dmvr[x->n_dmvr] = d;
    x->n_dmvr++;
  } else {
    if (x->n_mc < x->cap_mc) x->mc[x->n_mc] = d;
    x->n_mc++;
  }
}

/* MotionInfo::operator== (MotionInfo.h:196-219) */
static int o_mi_equal(const mm_pu_desc* a, const mm_pu_desc* b) {
  int interDirA = (a->ref_poc[0] >= 0 ? 1 : 0) + (a->ref_poc[1] >= 0 ? 2 : 0);
  int interDirB = (b->ref_poc[0] >= 0 ? 1 : 0) + (b->ref_poc[1] >= 0 ? 2 : 0);
  if (interDirA != interDirB) return 0;
  if (interDirA != 2) {
    if (a->ref_poc[0] != b->ref_poc[0] || a->mv[0][0] != b->mv[0][0] || a->mv[0][1] != b->mv[0][1] ||
        a->model[0] != b->model[0])
      return 0;
  }
  if (interDirA != 1) {
    if (a->ref_poc[1] != b->ref_poc[1] || a->mv[1][0] != b->mv[1][0] || a->mv[1][1] != b->mv[1][1] ||
        a->model[1] != b->model[1])
      return 0;
  }
  return 1;
}

static int o_motion_compensation(OEff* x, const mm_pu_desc* pu, unsigned flags, int poc, int merge_type_default,
                                 int m_subPuMC, const mm_pu_desc* sub);

/* xSubPuBio (:361-453) */
static int o_sub_pu_bio(OEff* x, const mm_pu_desc* pu, unsigned flags, int poc) {
  int fstStep = pu->h < 16 ? pu->h : 16, secStep = pu->w < 16 ? pu->w : 16;
  for (int fstDim = pu->y; fstDim < pu->y + pu->h; fstDim += fstStep)
    for (int secDim = pu->x; secDim < pu->x + pu->w; secDim += secStep) {
      mm_pu_desc subPu = *pu;
      subPu.x = secDim;
      subPu.y = fstDim;
      subPu.w = secStep;
      subPu.h = fstStep;
      int rc = o_motion_compensation(x, &subPu, flags, poc, 1, 0, NULL);
      if (rc) return rc;
    }
  return 0;
}

/* xSubPuMC (:283-359) */
static int o_sub_pu_mc(OEff* x, const mm_pu_desc* pu, unsigned flags, int poc, const mm_pu_desc* sub) {
  int numPartLine = (pu->w >> 3) > 1 ? (pu->w >> 3) : 1;
  int numPartCol = (pu->h >> 3) > 1 ? (pu->h >> 3) : 1;
  int puHeight = numPartCol == 1 ? pu->h : 8;
  int puWidth = numPartLine == 1 ? pu->w : 8;
  int verMC = pu->h > pu->w;
  int fstStart = !verMC ? pu->y : pu->x, secStart = !verMC ? pu->x : pu->y;
  int fstEnd = !verMC ? pu->y + pu->h : pu->x + pu->w, secEnd = !verMC ? pu->x + pu->w : pu->y + pu->h;
  int fstStep = !verMC ? puHeight : puWidth, secStep = !verMC ? puWidth : puHeight;
  int scaled = (flags & MM_PU_REF_SCALED) != 0;
#define O_MI(X, Y) (&sub[(((Y) - pu->y) / puHeight) * numPartLine + ((X) - pu->x) / puWidth])
  for (int fstDim = fstStart; fstDim < fstEnd; fstDim += fstStep)
    for (int secDim = secStart; secDim < secEnd; secDim += secStep) {
      int xx = !verMC ? secDim : fstDim, yy = !verMC ? fstDim : secDim;
      const mm_pu_desc* curMi = O_MI(xx, yy);
      int length = secStep, later = secDim + secStep;
      while (later < secEnd) {
        const mm_pu_desc* laterMi = !verMC ? O_MI(later, fstDim) : O_MI(fstDim, later);
        if (!scaled && o_mi_equal(laterMi, curMi))
          length += secStep;
        else
          break;
        later += secStep;
      }
      mm_pu_desc subPu = *curMi;
      subPu.x = xx;
      subPu.y = yy;
      subPu.w = !verMC ? length : puWidth;
      subPu.h = !verMC ? puHeight : length;
      subPu.bcw_idx = pu->bcw_idx;
      if (subPu.ref_poc[0] < 0 && subPu.ref_poc[1] < 0) return MM_ERR_ARG;
      int rc = o_motion_compensation(x, &subPu, flags & ~(unsigned)(MM_PU_MVREFINE | MM_PU_SUBPU), poc, 1, 1, NULL);
      if (rc) return rc;
      secDim = later - secStep;
    }
#undef O_MI
  return 0;
}

static int o_motion_compensation(OEff* x, const mm_pu_desc* pu, unsigned flags, int poc, int merge_type_default,
                                 int m_subPuMC, const mm_pu_desc* sub) {
  if (pu->ref_poc[0] >= 0 && pu->ref_poc[1] >= 0 && pu->w + pu->h == 12) return MM_ERR_ARG;
  int bioApplied = 0;
  if (x->tools->bdof) {
    if (m_subPuMC) {
      bioApplied = 0;
    } else {
      if (!(flags & MM_PU_WEIGHTED) && o_bi_dd_eq(pu, poc, flags) && pu->h >= 8 && pu->w >= 8 && pu->h * pu->w >= 128)
        bioApplied = 1;
    }
    if (bioApplied && (flags & MM_PU_CIIP)) bioApplied = 0;
    if (bioApplied && (flags & MM_PU_SMVD)) bioApplied = 0;
    if (x->tools->bcw && bioApplied && pu->bcw_idx != 2) bioApplied = 0;
    if (flags & MM_PU_MMVD_ENC2) bioApplied = 0;
  }
  if (flags & MM_PU_REF_SCALED) bioApplied = 0;
  int dmvrApplied = (flags & MM_PU_MVREFINE) && o_check_dmvr(x, pu, poc, flags, merge_type_default);
  if ((pu->w > 16 || pu->h > 16) && merge_type_default && (bioApplied && !dmvrApplied))
    return o_sub_pu_bio(x, pu, flags, poc);
  if (!merge_type_default) return o_sub_pu_mc(x, pu, flags, poc, sub);
  /* xCheckIdenticalMotion (:248-281) */
  if (!x->tools->wp_bi && pu->ref_poc[0] >= 0 && pu->ref_poc[1] >= 0 && pu->ref_poc[0] == pu->ref_poc[1] &&
      pu->mv[0][0] == pu->mv[1][0] && pu->mv[0][1] == pu->mv[1][1]) {
    mm_pu_desc u = *pu;
    u.ref_poc[1] = -1;
    u.mv[1][0] = u.mv[1][1] = 0;
    u.model[1] = 0;
    o_emit(x, &u, 0);
    return 0;
  }
  o_emit(x, pu, dmvrApplied); /* xPredInterBi: DMVR inside when dmvrApplied */
  return 0;
}

int orc_effective(const mm_tool_flags* tools, const mm_pu_motion* pus, int n, const mm_pu_desc* sub, mm_pu_desc* out_mc,
                  int cap_mc, int* n_mc, mm_pu_desc* out_dmvr, int cap_dmvr, int* n_dmvr) {
  OEff x = {tools, out_mc, out_dmvr, 0, 0, cap_mc, cap_dmvr};
  for (int i = 0; i < n; i++) {
    const mm_pu_motion* m = &pus[i];
    const mm_pu_desc* pu = &m->pu;
    if (pu->w < 4 || pu->h < 4 || (pu->w & 3) || (pu->h & 3) || (pu->ref_poc[0] < 0 && pu->ref_poc[1] < 0))
      return MM_ERR_ARG;
    int rc = o_motion_compensation(&x, pu, m->flags, m->cur_poc, !(m->flags & MM_PU_SUBPU), 0,
                                   (m->flags & MM_PU_SUBPU) ? sub + m->sub_motion : NULL);
    if (rc) return rc;
  }
  *n_mc = x.n_mc;
  *n_dmvr = x.n_dmvr;
  return (x.n_mc > cap_mc || x.n_dmvr > cap_dmvr) ? MM_ERR_ARG : 0;
}

/* ==========================================================================================
 * CPU baseline helpers (bench.py cpu_baseline leg): reference pictures padded once, then the
 * picture's PUs predicted on n_threads host threads (PU-parallel: PUs write disjoint samples;
 * the Orc state is read-only during prediction).  The per-PU arithmetic is pred_pu's.
 * ========================================================================================== */
#include <pthread.h>

typedef struct {
  int n;
  OPic* pics;
} ORefs;

void* orc_refs_create(void* h, int n_refs, const int32_t* pocs, const int16_t* const* ys, const int16_t* const* cbs,
                      const int16_t* const* crs, ptrdiff_t stride_y, ptrdiff_t stride_c) {
  ORefs* r = (ORefs*)calloc(1, sizeof(ORefs));
  r->n = n_refs;
  r->pics = pad_refs((Orc*)h, n_refs, pocs, ys, cbs, crs, stride_y, stride_c);
  return r;
}

void orc_refs_destroy(void* p) {
  ORefs* r = (ORefs*)p;
  if (!r) return;
  free_refs(r->pics, r->n);
  free(r);
}

typedef struct {
  Orc* o;
  const ORefs* refs;
  int cur_poc;
  const mm_pu_desc* pus;
  int begin, end;
  int16_t *dy, *dcb, *dcr;
  ptrdiff_t sdy, sdc;
  int rc;
} OJob;

static void* pred_range(void* arg) {
  OJob* j = (OJob*)arg;
  int16_t* pred[2][3];
  for (int l = 0; l < 2; l++)
    for (int c = 0; c < 3; c++) pred[l][c] = (int16_t*)malloc(sizeof(int16_t) * 128 * 128);
  j->rc = 0;
  for (int i = j->begin; i < j->end && !j->rc; i++)
    j->rc = pred_pu(j->o, j->refs->pics, j->refs->n, &j->pus[i], j->cur_poc, pred, j->dy, j->sdy, j->dcb, j->dcr, j->sdc,
                    -1, 0);
  for (int l = 0; l < 2; l++)
    for (int c = 0; c < 3; c++) free(pred[l][c]);
  return NULL;
}

int orc_pred_padded(void* h, void* refs, int cur_poc, const mm_pu_desc* pus, int n, int16_t* dy, ptrdiff_t sdy,
                    int16_t* dcb, int16_t* dcr, ptrdiff_t sdc, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  OJob jobs[256];
  pthread_t th[256];
  for (int t = 0; t < n_threads; t++) {
    /* interleaved chunks of 64 PUs would balance better; contiguous ranges keep it simple and the
       PU list is raster-ordered with a uniform mix of models */
    OJob jb = {(Orc*)h, (const ORefs*)refs, cur_poc, pus, (int)((long)n * t / n_threads),
               (int)((long)n * (t + 1) / n_threads), dy, dcb, dcr, sdy, sdc, 0};
    jobs[t] = jb;
  }
  if (n_threads == 1) {
    pred_range(&jobs[0]);
    return jobs[0].rc;
  }
  for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, pred_range, &jobs[t]);
  int rc = 0;
  for (int t = 0; t < n_threads; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc && !rc) rc = jobs[t].rc;
  }
  return rc;
}

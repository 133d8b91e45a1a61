// Cost of the bit-exact float primitives k_reproj is made of (glibc / Eigen restatements in
// mm_numerics.h), on wave-coherent inputs (neighbouring lanes get neighbouring arguments, as the
// elements of one reprojection job do).  Prints ns per element and VALU-issue cycles per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../vvc-extension-mm_amd/csrc/mm_numerics.h"

using namespace mmnum;
constexpr int N = 1 << 22;
constexpr int REP = 8;

#define PRIM(NAME, LO, HI, EXPR)                                                              \
  __global__ void k_##NAME(float* out) {                                                      \
    const int i = blockIdx.x * blockDim.x + threadIdx.x;                                      \
    float acc = 0.0f;                                                                         \
    for (int r = 0; r < REP; r++) {                                                           \
      const float x = (LO) + ((HI) - (LO)) * (float)((i * 7 + r * 977) & (N - 1)) / (float)N; \
      acc += (EXPR);                                                                          \
    }                                                                                         \
    out[i] = acc;                                                                             \
  }

PRIM(empty, 0.1f, 0.9f, x)
PRIM(div, 0.1f, 0.9f, 1.0f / (x + 3.0f))
PRIM(sqrtf, 0.1f, 0.9f, sqrtf_(x))
PRIM(psqrt, 0.1f, 0.9f, e_psqrt(x))
PRIM(g_sinf, -3.0f, 3.0f, g_sinf(x))
PRIM(g_cosf, -3.0f, 3.0f, g_cosf(x))
PRIM(psin, -3.0f, 3.0f, e_psin(x))
PRIM(pcos, -3.0f, 3.0f, e_pcos(x))
PRIM(sin_dbl, -3.0f, 3.0f, sinf_via_double(x))
PRIM(g_atanf, -4.0f, 4.0f, g_atanf(x))
PRIM(g_atan2f, -1.0f, 1.0f, g_atan2f(x, 0.7f - x))
PRIM(g_acosf, -0.99f, 0.99f, g_acosf(x))
PRIM(g_asinf, -0.99f, 0.99f, g_asinf(x))
PRIM(g_tanf, -1.5f, 1.5f, g_tanf(x))
PRIM(psincos, -3.0f, 3.0f, e_psin(x) + e_pcos(x))
PRIM(g_sincos, -3.0f, 3.0f, g_sinf(x) + g_cosf(x))
PRIM(div_y_x, -1.0f, 1.0f, x / (0.7f - x))

int main() {
  float* out;
  hipMalloc(&out, N * sizeof(float));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipDeviceProp_t pr;
  hipGetDeviceProperties(&pr, 0);
  const double simds = 4.0 * pr.multiProcessorCount;
  struct K {
    const char* name;
    void (*f)(float*);
  } ks[] = {{"empty", k_empty},   {"div", k_div},       {"sqrtf", k_sqrtf},       {"psqrt", k_psqrt},
            {"g_sinf", k_g_sinf}, {"g_cosf", k_g_cosf}, {"psin", k_psin},         {"pcos", k_pcos},
            {"sin_dbl", k_sin_dbl}, {"g_atanf", k_g_atanf}, {"g_atan2f", k_g_atan2f}, {"g_acosf", k_g_acosf},
            {"g_asinf", k_g_asinf}, {"g_tanf", k_g_tanf}, {"psincos", k_psincos}, {"g_sincos", k_g_sincos},
            {"div_y_x", k_div_y_x}};
  float base = 0.0f;
  for (const K& k : ks) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k.f, dim3(N / 256), dim3(256), 0, 0, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    if (k.f == k_empty) base = best;
    const double calls = (double)N * REP;
    const double cyc_per_wave = (best - base) * 1e-3 * 2.4e9 * simds / (calls / 64);
    printf("%-10s %8.3f ms  %7.1f issue-cycles per wave-call (net of the empty loop)\n", k.name, best, cyc_per_wave);
  }
  return 0;
}

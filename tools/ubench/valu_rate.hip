// Throughput of the integer / float VALU forms usable by the 8-tap filter (gfx950), many waves
// per SIMD, 8 independent accumulation chains per lane.   hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
#define N_ITER 4096
template <int OP>
__global__ void __launch_bounds__(256) k(const unsigned* in, unsigned* out) {
  unsigned a[8];
  for (int i = 0; i < 8; i++) a[i] = in[threadIdx.x + i];
  unsigned b = in[threadIdx.x + 9], c = in[threadIdx.x + 10];
  float f[8];
  for (int i = 0; i < 8; i++) f[i] = __uint_as_float(a[i] & 0x3fffffff);
  float fb = __uint_as_float(b & 0x3fffffff);
  for (int it = 0; it < N_ITER; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (OP == 0) a[i] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, b), __builtin_bit_cast(s2, c), (int)a[i], false);
      if (OP == 1) f[i] = __builtin_fmaf(f[i], fb, fb);
      if (OP == 2) a[i] = __mul24((int)a[i], (int)b) + (int)c;
      if (OP == 3) a[i] = a[i] * b + c;
      if (OP == 4) { b += a[i]; a[i] = __builtin_amdgcn_perm(a[i], b, 0x05040100u); }
      if (OP == 5) a[i] = __builtin_amdgcn_sdot4((int)b, (int)c, (int)a[i], false);
      if (OP == 6) f[i] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, b), __builtin_bit_cast(h2, c), f[i], false);
      if (OP == 7) a[i] = a[i] >> 2;
      if (OP == 8) f[i] = __builtin_floorf(f[i] * fb);
    }
  }
  unsigned s = 0;
  for (int i = 0; i < 8; i++) s += a[i] + __float_as_uint(f[i]);
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int OP>
void run(const char* name, const unsigned* din, unsigned* dout) {
  const int blocks = 256 * 4 * 8 / 4;  // 8 waves per SIMD
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, din, dout);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, din, dout);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double waves = blocks * 4.0, instrs = waves * N_ITER * 8;
  const double per_simd = instrs / 1024.0;
  printf("%-10s %.3f ms  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", name, ms,
         ms * 1e-3 * 2.4e9 / per_simd);
}
int main() {
  unsigned *din, *dout;
  hipMalloc(&din, 4096 * 4);
  hipMemset(din, 1, 4096 * 4);
  hipMalloc(&dout, 256 * 4 * 8 / 4 * 256 * 4);
  run<0>("dot2_i16", din, dout);
  run<1>("fma_f32", din, dout);
  run<2>("mad_i24", din, dout);
  run<3>("mul_lo+add", din, dout);
  run<4>("add+perm", din, dout);
  run<5>("sdot4_i8", din, dout);
  run<6>("fdot2_f16", din, dout);
  run<7>("ashr", din, dout);
  run<8>("mul+floor", din, dout);
  return 0;
}

// Issue rate of packed FP32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) against scalar FP32 and FP64
// on gfx950, many waves per SIMD, 8 independent chains per lane: does a packed instruction (two
// lanes' worth of f32 math) issue at the scalar rate?   hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
#define N_ITER 4096
template <int OP>
__global__ void __launch_bounds__(256) k(const unsigned* in, unsigned* out) {
  float f[8];
  f2 v[8];
  double d[8];
  for (int i = 0; i < 8; i++) {
    f[i] = __uint_as_float(in[threadIdx.x + i] & 0x3fffffff);
    v[i] = f2{f[i], f[i] * 0.5f};
    d[i] = f[i];
  }
  const float fb = __uint_as_float(in[threadIdx.x + 9] & 0x3fffffff);
  const f2 vb = f2{fb, fb * 0.25f};
  const double db = fb;
  for (int it = 0; it < N_ITER; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (OP == 0) f[i] = __builtin_fmaf(f[i], fb, fb);
      if (OP == 1) v[i] = __builtin_elementwise_fma(v[i], vb, vb);
      if (OP == 2) v[i] = v[i] * vb;
      if (OP == 3) v[i] = v[i] + vb;
      if (OP == 4) d[i] = __builtin_fma(d[i], db, db);
      if (OP == 5) f[i] = f[i] * fb;
    }
  }
  float s = 0.0f;
  for (int i = 0; i < 8; i++) s += f[i] + v[i].x + v[i].y + (float)d[i];
  out[blockIdx.x * 256 + threadIdx.x] = __float_as_uint(s);
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
  printf("%-12s %.3f ms  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", name, ms,
         ms * 1e-3 * 2.4e9 / (instrs / 1024.0));
}
int main() {
  unsigned *din, *dout;
  hipMalloc(&din, 4096 * 4);
  hipMemset(din, 1, 4096 * 4);
  hipMalloc(&dout, 256 * 4 * 8 / 4 * 256 * 4);
  run<0>("fma_f32", din, dout);
  run<1>("pk_fma_f32", din, dout);
  run<2>("pk_mul_f32", din, dout);
  run<3>("pk_add_f32", din, dout);
  run<4>("fma_f64", din, dout);
  run<5>("mul_f32", din, dout);
  return 0;
}

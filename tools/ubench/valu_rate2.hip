// Issue rate of packed / 64-bit VALU forms on gfx950 (k_mc design questions): v_pk_fma_f32 vs
// v_fma_f32 vs v_dot2_i32_i16, packed int16 math, v_lshl_add_u64, v_cvt_f32_i32 with word select.
// 8 waves per SIMD, 8 independent chains per lane.   hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
#define N_ITER 2048
template <int OP>
__global__ void __launch_bounds__(256) k(const unsigned* in, unsigned* out) {
  unsigned a[8];
  f2 p[8];
  unsigned long long q[8];
  for (int i = 0; i < 8; i++) {
    a[i] = in[threadIdx.x + i];
    p[i] = f2{__uint_as_float(a[i] & 0x3f7fffff), __uint_as_float(a[i] & 0x3e7fffff)};
    q[i] = a[i];
  }
  unsigned b = in[threadIdx.x + 9], c = in[threadIdx.x + 10];
  f2 pb = f2{__uint_as_float(b & 0x3f7fffff), __uint_as_float(c & 0x3f7fffff)};
  float fb = __uint_as_float(b & 0x3f7fffff);
  for (int it = 0; it < N_ITER; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (OP == 0) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(pb), "v"(pb));
      if (OP == 1) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(fb), "v"(fb));
      if (OP == 2) asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c));
      if (OP == 3) asm volatile("v_pk_add_u16 %0, %1, %0" : "+v"(a[i]) : "v"(b));
      if (OP == 4) asm volatile("v_pk_mad_i16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c));
      if (OP == 5) asm volatile("v_lshl_add_u64 %0, %1, 1, %0" : "+v"(q[i]) : "v"(q[(i + 1) & 7]));
      if (OP == 6) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
      if (OP == 7) asm volatile("v_cvt_f32_i32_sdwa %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "+v"(a[i]));
      if (OP == 8) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p[i]) : "v"(pb));
      if (OP == 9) asm volatile("v_med3_i32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c));
      if (OP == 10) asm volatile("v_cvt_flr_i32_f32 %0, %0" : "+v"(a[i]));
      if (OP == 11) asm volatile("v_ashrrev_i32 %0, 2, %0" : "+v"(a[i]));
      if (OP == 12) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      if (OP == 13) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c));
    }
  }
  unsigned s = 0;
  for (int i = 0; i < 8; i++) s += a[i] + __float_as_uint(p[i].x) + __float_as_uint(p[i].y) + (unsigned)q[i];
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
  printf("%-12s %.3f ms  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", name, ms,
         ms * 1e-3 * 2.4e9 / per_simd);
}
int main() {
  unsigned *din, *dout;
  hipMalloc(&din, 4096 * 4);
  hipMemset(din, 1, 4096 * 4);
  hipMalloc(&dout, 256 * 4 * 8 / 4 * 256 * 4);
  run<1>("fma_f32", din, dout);
  run<0>("pk_fma_f32", din, dout);
  run<8>("pk_mul_f32", din, dout);
  run<2>("dot2_i32_i16", din, dout);
  run<3>("pk_add_u16", din, dout);
  run<4>("pk_mad_i16", din, dout);
  run<5>("lshl_add_u64", din, dout);
  run<6>("add_u32", din, dout);
  run<7>("cvt_f32_sdwa", din, dout);
  run<9>("med3_i32", din, dout);
  run<10>("cvt_flr_i32", din, dout);
  run<11>("ashr_i32", din, dout);
  run<12>("perm_b32", din, dout);
  run<13>("mad_u32_u24", din, dout);
  return 0;
}

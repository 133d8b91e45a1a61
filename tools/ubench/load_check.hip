// Correctness of the load forms a faster k_mc would use (gfx950): dwordx4 loads from 2-byte-aligned
// addresses (global and raw buffer), and buffer loads with an SGPR row offset + a per-lane VGPR
// offset.  Prints mismatches (0 expected) and exits non-zero on any.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned u4a2 __attribute__((ext_vector_type(4), aligned(2)));
typedef int i4 __attribute__((ext_vector_type(4)));

__global__ void k(const short* p, int n, unsigned* out_g, unsigned* out_b) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t + 8 > n) return;
  u4a2 v = *reinterpret_cast<const u4a2*>(p + t);  // 2-byte aligned for odd t
  out_g[4 * t + 0] = v.x;
  out_g[4 * t + 1] = v.y;
  out_g[4 * t + 2] = v.z;
  out_g[4 * t + 3] = v.w;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, n * 2, 0x00020000);
  const int row = (t / 64) * 128;  // uniform per wave: SGPR offset
  const int lane_off = (t - (t / 64) * 64) * 2;
  i4 w = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off, row, 0);
  out_b[4 * t + 0] = w.x;
  out_b[4 * t + 1] = w.y;
  out_b[4 * t + 2] = w.z;
  out_b[4 * t + 3] = w.w;
}

int main() {
  const int n = 1 << 16;
  std::vector<short> h(n);
  for (int i = 0; i < n; i++) h[i] = (short)(i * 2654435761u >> 16);
  short* d;
  unsigned *og, *ob;
  hipMalloc(&d, n * 2);
  hipMalloc(&og, (size_t)n * 16);
  hipMalloc(&ob, (size_t)n * 16);
  hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d, n, og, ob);
  std::vector<unsigned> g((size_t)n * 4), b((size_t)n * 4);
  hipMemcpy(g.data(), og, (size_t)n * 16, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), ob, (size_t)n * 16, hipMemcpyDeviceToHost);
  long bad_g = 0, bad_b = 0;
  for (int t = 0; t + 8 <= n; t++) {
    for (int k = 0; k < 4; k++) {
      unsigned want = (unsigned short)h[t + 2 * k] | ((unsigned)(unsigned short)h[t + 2 * k + 1] << 16);
      bad_g += g[4 * t + k] != want;
      const int bt = (t / 64) * 64 + (t - (t / 64) * 64);  // byte offset row + lane_off -> element
      const int e = (t / 64) * 64 + (t - (t / 64) * 64);
      (void)bt;
      unsigned wb = (unsigned short)h[e + 2 * k] | ((unsigned)(unsigned short)h[e + 2 * k + 1] << 16);
      bad_b += b[4 * t + k] != wb;
    }
  }
  printf("unaligned global dwordx4 mismatches %ld, buffer (sgpr row + vgpr lane) mismatches %ld\n", bad_g, bad_b);
  return (bad_g || bad_b) ? 1 : 0;
}

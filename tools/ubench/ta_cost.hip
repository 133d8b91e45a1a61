// Texture-address (TA) cost of one vector-memory wave-instruction on gfx950 by access shape, L2-warm:
// how k_mc's window gathers should be shaped.  Every lane issues ITER loads of the pattern; the
// table (2 MiB) stays in L2.  Prints ns per wave-instruction per CU for each pattern.
//   pattern  bytes/lane  lanes per distinct 128-B line group
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 256;
constexpr int TABLE = 1 << 20;  // shorts (2 MiB)

template <int BYTES>
struct V;
template <>
struct V<16> {
  typedef unsigned T __attribute__((ext_vector_type(4)));
};
template <>
struct V<8> {
  typedef unsigned T __attribute__((ext_vector_type(2)));
};
template <>
struct V<4> {
  typedef unsigned T;
};

// lanes_per_row: consecutive lanes reading consecutive BYTES-wide pieces of one row; rows are
// `row_stride` bytes apart (distinct lines), rotated per iteration
template <int BYTES>
__global__ void k(const char* __restrict__ tab, int lanes_per_row, int row_stride, unsigned* out) {
  typedef typename V<BYTES>::T T;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int row = lane / lanes_per_row, col = lane % lanes_per_row;
  unsigned acc = 0;
  const int lane_off = row * row_stride + col * BYTES;
  unsigned base = (unsigned)(wave * 977 % 4096) * 256;
#pragma unroll 8
  for (int i = 0; i < ITER; i++) {
    const T v = *reinterpret_cast<const T*>(tab + (base & ((1u << 20) - 1)) + lane_off);
    if constexpr (BYTES == 4)
      acc += v;
    else if constexpr (BYTES == 8)
      acc += v.x ^ v.y;
    else
      acc += v.x ^ v.y ^ v.z ^ v.w;
    base += 4096 + 128;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  char* tab;
  unsigned* out;
  hipMalloc(&tab, 2 * TABLE);
  hipMemset(tab, 1, 2 * TABLE);
  hipMalloc(&out, 64);
  hipDeviceProp_t pr;
  hipGetDeviceProperties(&pr, 0);
  const int cus = pr.multiProcessorCount;
  const int blocks = cus * 8, threads = 256;  // 32 waves per CU
  const long waves = (long)blocks * threads / 64;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct P {
    int bytes, lanes_per_row, stride;
    const char* name;
  } ps[] = {{16, 64, 0, "x4 contiguous 1 KB"},
            {16, 4, 2048, "x4 16 rows x 64 B"},
            {16, 2, 2048, "x4 32 rows x 32 B"},
            {16, 1, 2048, "x4 64 rows x 16 B"},
            {8, 64, 0, "x2 contiguous 512 B"},
            {8, 4, 2048, "x2 16 rows x 32 B"},
            {8, 1, 2048, "x2 64 rows x 8 B"},
            {4, 64, 0, "x1 contiguous 256 B"},
            {4, 1, 2048, "x1 64 rows x 4 B"}};
  for (const P& p : ps) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      hipEventRecord(a);
      if (p.bytes == 16)
        hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(threads), 0, 0, tab, p.lanes_per_row, p.stride, out);
      else if (p.bytes == 8)
        hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(threads), 0, 0, tab, p.lanes_per_row, p.stride, out);
      else
        hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(threads), 0, 0, tab, p.lanes_per_row, p.stride, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    const double per_cu_instr = (double)waves * ITER / cus;
    printf("%-24s %8.3f ms  %6.2f ns per wave-instruction per CU (%5.1f cycles at 2.4 GHz)\n", p.name, best,
           best * 1e6 / per_cu_instr, best * 1e6 / per_cu_instr * 2.4);
  }
  return 0;
}

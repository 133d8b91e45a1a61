// Does hipFree wait for unrelated work queued on another stream?  A bounded busy kernel (~100-200 ms)
// runs on a non-blocking stream; the host then frees an unrelated buffer and times the call.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void busy(float* out, int iters) {
  float a = threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; i++) a = a * 0.999999f + 1e-7f;  // bounded: every wave exits
  if (a == 12345.0f) out[threadIdx.x] = a;
}

int main() {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  float *out = nullptr, *victim = nullptr, *victim2 = nullptr;
  if (hipMalloc(&out, 1024 * sizeof(float)) != hipSuccess) return 1;
  if (hipMalloc(&victim, 64 << 20) != hipSuccess) return 1;
  if (hipMalloc(&victim2, 64 << 20) != hipSuccess) return 1;
  // calibrate the busy kernel alone
  auto t0 = std::chrono::steady_clock::now();
  hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, out, 20000000);
  if (hipStreamSynchronize(s) != hipSuccess) return 1;
  auto t1 = std::chrono::steady_clock::now();
  const double kern_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  // hipFree while the kernel runs on the other stream
  hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, out, 20000000);
  auto t2 = std::chrono::steady_clock::now();
  if (hipFree(victim) != hipSuccess) return 1;
  auto t3 = std::chrono::steady_clock::now();
  if (hipStreamSynchronize(s) != hipSuccess) return 1;
  // hipMalloc while the kernel runs
  hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, out, 20000000);
  auto t4 = std::chrono::steady_clock::now();
  float* fresh = nullptr;
  if (hipMalloc(&fresh, 64 << 20) != hipSuccess) return 1;
  auto t5 = std::chrono::steady_clock::now();
  if (hipStreamSynchronize(s) != hipSuccess) return 1;
  printf("busy kernel alone %.1f ms; hipFree during it %.1f ms; hipMalloc during it %.1f ms\n", kern_ms,
         std::chrono::duration<double, std::milli>(t3 - t2).count(),
         std::chrono::duration<double, std::milli>(t5 - t4).count());
  // stream-ordered: hipMallocAsync / hipFreeAsync on a second stream while the kernel runs
  hipStream_t s2;
  if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess) return 1;
  float* pooled = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&pooled), 64 << 20, s2) != hipSuccess) return 1;
  if (hipStreamSynchronize(s2) != hipSuccess) return 1;
  hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, out, 20000000);
  auto t6 = std::chrono::steady_clock::now();
  hipError_t ef = hipFreeAsync(pooled, s2);
  auto t7 = std::chrono::steady_clock::now();
  hipError_t es = hipStreamSynchronize(s2);
  auto t8 = std::chrono::steady_clock::now();
  // hipFreeAsync of a hipMalloc'd pointer
  float* plain = nullptr;
  if (hipMalloc(&plain, 64 << 20) != hipSuccess) return 1;
  hipError_t ef2 = hipFreeAsync(plain, s2);
  hipError_t es2 = hipStreamSynchronize(s2);
  auto t9 = std::chrono::steady_clock::now();
  if (hipStreamSynchronize(s) != hipSuccess) return 1;
  printf("hipFreeAsync (pool) call %.2f ms rc %d, its stream done after %.1f ms rc %d; hipFreeAsync of a hipMalloc "
         "pointer rc %d / %d (%.1f ms)\n",
         std::chrono::duration<double, std::milli>(t7 - t6).count(), (int)ef,
         std::chrono::duration<double, std::milli>(t8 - t6).count(), (int)es, (int)ef2, (int)es2,
         std::chrono::duration<double, std::milli>(t9 - t8).count());
  (void)hipStreamDestroy(s2);
  (void)hipFree(fresh);
  (void)hipFree(victim2);
  (void)hipFree(out);
  (void)hipStreamDestroy(s);
  return 0;
}

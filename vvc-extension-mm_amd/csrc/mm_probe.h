// mm_probe.h -- the MM_RACE_PROBE diagnostic build (never the product library).
//
// Every LDS word that one thread stores and other waves of the workgroup read goes through
// lds_put().  In the product build that is the plain store.  With -DMM_RACE_PROBE the storing
// thread first writes a poison value to the word, then sleeps ~7 us, then stores the real value:
// a reader that is correctly ordered behind a __syncthreads() sees the real value, a reader whose
// barrier is missing reads the poison (or, for counters, its atomics are overwritten by the late
// initialisation), so the missing barrier shows up as a wrong picture in the GPU suite instead of a
// timing-dependent fault.  Poison values are chosen so that a racing reader computes wrong results
// without leaving its buffers: pool offsets point at the pool's last slot, indices and counts are 0,
// positions are out of range.  tools/race_probe.sh builds the variant and runs the GPU suite on it.
#pragma once

#if defined(__HIP__)
#if defined(MM_RACE_PROBE) && defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void mm_probe_delay() {
#pragma unroll 1
  for (int i = 0; i < 2; i++) __builtin_amdgcn_s_sleep(127);  // 2 x 127 x 64 cycles
}
template <class T>
__device__ __forceinline__ void lds_put(T& dst, const T& v, const T& poison) {
  dst = poison;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the poison is in LDS before the delay
  mm_probe_delay();
  asm volatile("" ::: "memory");
  dst = v;
}
#else
template <class T>
__device__ __forceinline__ void lds_put(T& dst, const T& v, const T&) {
  dst = v;
}
#endif
#endif

// sit_occupy.hip — test utility (not part of libsit.so): a kernel that holds wave slots and registers on
// the CUs for a bounded time, so that a step kernel launched beside it on another stream is placed on
// SIMDs it would not get alone (tests/test_gpu_placement.py).  Each wave spins on the 100 MHz real-time
// counter with s_sleep until its own deadline and exits: every wave reaches the exit condition, so the
// grid always drains.  "heavy" waves reserve 256 VGPRs (a clobber of v255), so that a SIMD holding one
// has room for one 192-VGPR step wave, not two.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

template <bool HEAVY>
__global__ __launch_bounds__(256) void k_occupy(uint64_t ticks, uint32_t* started) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (HEAVY) asm volatile("s_nop 0" ::: "v255");
  if ((threadIdx.x & 63) == 0) atomicAdd(started, 1u);
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

}  // namespace

extern "C" {

// blocks x threads / 64 waves of the occupier for `ms` milliseconds (at most 2 s) on `stream`; `started`
// (a device uint32) counts the waves that began.  Returns 0 when launched.
int sit_test_occupy(int32_t blocks, int32_t threads, int32_t heavy, double ms, uint32_t* started, void* stream) {
  if (blocks <= 0 || threads <= 0 || threads > 256 || threads % 64 != 0 || !started || ms <= 0 || ms > 2000) return -1;
  const uint64_t ticks = (uint64_t)(ms * 1e5);   // 100 MHz
  if (heavy)
    hipLaunchKernelGGL(k_occupy<true>, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, ticks, started);
  else
    hipLaunchKernelGGL(k_occupy<false>, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, ticks, started);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}

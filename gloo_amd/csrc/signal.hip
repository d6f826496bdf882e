// signal.hip — see gloo_amd/signal.h.
#include <hip/hip_runtime.h>

#include "gloo_amd/signal.h"

namespace gloo_amd {
namespace {

__global__ __launch_bounds__(64) void signal_kernel(uint64_t* flag, uint64_t value) {
  if (threadIdx.x == 0) {
    // every write that precedes this kernel on the stream (the chunk copy,
    // the reduction that consumed an inbox) is performed at system scope
    // before the flag can be observed
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(64) void wait_kernel(const uint64_t* flag, uint64_t target, uint64_t timeout_ticks,
                                                  uint32_t* err) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  // relaxed polls, ONE acquire after the match (an acquire per poll would
  // invalidate the caches on every iteration)
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
    __builtin_amdgcn_s_sleep(8);
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

}  // namespace

hipError_t launchSignal(uint64_t* flag, uint64_t value, hipStream_t stream) {
  signal_kernel<<<1, 64, 0, stream>>>(flag, value);
  return hipGetLastError();
}

hipError_t launchWait(const uint64_t* flag, uint64_t target, uint64_t timeoutTicks, uint32_t* err,
                      hipStream_t stream) {
  wait_kernel<<<1, 64, 0, stream>>>(flag, target, timeoutTicks, err);
  return hipGetLastError();
}

}  // namespace gloo_amd

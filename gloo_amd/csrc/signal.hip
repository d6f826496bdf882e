// signal.hip — see gloo_amd/signal.h.
#include <hip/hip_runtime.h>

#include "gloo_amd/signal.h"

namespace gloo_amd {
namespace {

__device__ __forceinline__ uint64_t seqValue(uint64_t base, uint64_t perRun, const uint64_t* epoch) {
  return epoch ? base + *epoch * perRun : base;
}

__global__ __launch_bounds__(64) void epoch_kernel(uint64_t* epoch, int set, uint64_t value) {
  if (threadIdx.x == 0) *epoch = set ? value : *epoch + 1;
}

__global__ __launch_bounds__(64) void signal_kernel(uint64_t* flag, uint64_t base, uint64_t perRun,
                                                    const uint64_t* epoch) {
  if (threadIdx.x == 0) {
    // every write that precedes this kernel on the stream (the chunk copy,
    // the reduction that consumed an inbox) is performed at system scope
    // before the flag can be observed
    const uint64_t v = seqValue(base, perRun, epoch);
    // one release, then a relaxed flag store (a release store would write the
    // L2 back a second time); the wait keeps the flag behind the write-back
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(64) void wait_kernel(const uint64_t* flag, uint64_t base, uint64_t perRun,
                                                  const uint64_t* epoch, uint64_t timeout_ticks, uint32_t* err) {
  if (threadIdx.x != 0) return;
  const uint64_t target = seqValue(base, perRun, epoch);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  // relaxed polls, ONE acquire after the match (an acquire per poll would
  // invalidate the caches on every iteration)
  // signed difference: a target "below" the counter is already satisfied
  while ((int64_t)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
    __builtin_amdgcn_s_sleep(8);
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

struct WaitList {
  int n;
  const uint64_t* flag[kMaxWaitEntries];
  Seq target[kMaxWaitEntries];
};

__global__ __launch_bounds__(64) void wait_multi_kernel(WaitList w, const uint64_t* epoch, uint64_t timeout_ticks,
                                                        uint32_t* err) {
  const int j = threadIdx.x;
  if (j < w.n) {
    const uint64_t target = seqValue(w.target[j].base, w.target[j].perRun, epoch);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int64_t)(__hip_atomic_load(w.flag[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
      __builtin_amdgcn_s_sleep(8);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// Diagnosis of IPC mappings: the first word behind `p` read four ways.
__global__ __launch_bounds__(64) void probe_kernel(const uint64_t* p, uint64_t* out) {
  if (threadIdx.x == 0) {
    out[0] = *reinterpret_cast<const volatile uint64_t*>(p);
    out[1] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    out[2] = __builtin_nontemporal_load(p);
    out[3] = *reinterpret_cast<const volatile uint64_t*>(p);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
}

}  // namespace

hipError_t launchProbe(const uint64_t* p, uint64_t* out, hipStream_t stream) {
  probe_kernel<<<1, 64, 0, stream>>>(p, out);
  return hipGetLastError();
}

hipError_t launchWaitMulti(const uint64_t* const* flags, const Seq* targets, int n, const uint64_t* epoch,
                           uint64_t timeoutTicks, uint32_t* err, hipStream_t stream) {
  for (int i = 0; i < n; i += kMaxWaitEntries) {
    WaitList w;
    w.n = n - i < kMaxWaitEntries ? n - i : kMaxWaitEntries;
    for (int j = 0; j < w.n; j++) {
      w.flag[j] = flags[i + j];
      w.target[j] = targets[i + j];
    }
    wait_multi_kernel<<<1, 64, 0, stream>>>(w, epoch, timeoutTicks, err);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launchEpochBump(uint64_t* epoch, hipStream_t stream) {
  epoch_kernel<<<1, 64, 0, stream>>>(epoch, 0, 0);
  return hipGetLastError();
}

hipError_t launchEpochSet(uint64_t* epoch, uint64_t value, hipStream_t stream) {
  epoch_kernel<<<1, 64, 0, stream>>>(epoch, 1, value);
  return hipGetLastError();
}

hipError_t launchSignal(uint64_t* flag, Seq value, const uint64_t* epoch, hipStream_t stream) {
  signal_kernel<<<1, 64, 0, stream>>>(flag, value.base, value.perRun, epoch);
  return hipGetLastError();
}

hipError_t launchWait(const uint64_t* flag, Seq target, const uint64_t* epoch, uint64_t timeoutTicks,
                      uint32_t* err, hipStream_t stream) {
  wait_kernel<<<1, 64, 0, stream>>>(flag, target.base, target.perRun, epoch, timeoutTicks, err);
  return hipGetLastError();
}

}  // namespace gloo_amd

// test_kernels.hip — TEST HELPERS for tests/bridge/bridge_test.cc (built into
// tests/bridge/libbridge_kernels.so by gloo_amd/Makefile).
//
//   bt_spin     the reference's waitClocks / cudaSleep test helper
//               (gloo/test/cuda_base_test.cu:15-27): one lane spins on the
//               GPU's 100 MHz constant clock for `ticks`, delaying the work
//               queued behind it on `stream` (MultiPointerAsync,
//               gloo/test/cuda_base_test.h:60-75).  Bounded: it always ends.
//   bt_add_i32  a caller-supplied device reduction (dst[i] += src[i] on
//               int32), the device function of a HipReductionFunction<int>
//               with ReductionType CUSTOM; counts its host-side calls.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>

namespace {

__global__ void spin_kernel(unsigned long long ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}

__global__ void add_i32_kernel(int32_t* dst, const int32_t* src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = (int32_t)((uint32_t)dst[i] + (uint32_t)src[i]);
}

std::atomic<long> g_calls{0};

}  // namespace

extern "C" int bt_spin(hipStream_t stream, unsigned long long ticks) {
  spin_kernel<<<1, 64, 0, stream>>>(ticks);
  return (int)hipGetLastError();
}

extern "C" void bt_add_i32(int32_t* dst, const int32_t* src, size_t n, hipStream_t stream) {
  g_calls++;
  if (n == 0) return;
  const unsigned blocks = (unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
  add_i32_kernel<<<blocks, 256, 0, stream>>>(dst, src, n);
}

extern "C" long bt_add_i32_calls(void) { return g_calls.load(); }

// xor_op.hip — TEST HELPER: a caller-supplied device reduction for the
// custom-op path (gloo_hip_register_op; the reference's
// ReductionType::CUSTOM, gloo/algorithm.h:49-95).  Bytewise XOR: not one of
// the built-in ops, exact and order-independent, so every schedule's result
// is the XOR of all ranks' inputs.  `user` points at the element size.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
__global__ void xor_kernel(uint8_t* c, const uint8_t* a, const uint8_t* b, size_t nbytes) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nbytes; i += (size_t)gridDim.x * blockDim.x)
    c[i] = a[i] ^ b[i];
}
unsigned long long g_calls = 0;
}  // namespace

extern "C" {
void xor_op_fn(void* user, void* c, const void* a, const void* b, size_t n, void* stream) {
  const size_t nbytes = n * (user ? *static_cast<const int*>(user) : 1);
  size_t grid = (nbytes + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid == 0) return;
  xor_kernel<<<(unsigned)grid, 256, 0, static_cast<hipStream_t>(stream)>>>(
      static_cast<uint8_t*>(c), static_cast<const uint8_t*>(a), static_cast<const uint8_t*>(b), nbytes);
  __atomic_add_fetch(&g_calls, 1, __ATOMIC_RELAXED);
}
unsigned long long xor_op_calls() { return g_calls; }
int xor_elem_size_4 = 4;
}

// staged.cc — the host-staged chunk reduction: chunks that
// start and end in host memory (a transport's receive buffer on a socket or
// NIC) reduced on the GPU.  The reference's CudaHostWorkspace path
// (gloo/cuda_collectives_host.h:22-136) copies device data to the host and
// reduces on the CPU; here the data goes the other way and the reduction
// stays the HIP kernel.
//
// Zero-copy (piece_elems == 0, both host buffers pinned and mapped into the
// device's address space): ONE kernel reads both operands over PCIe and
// writes the result back in place, with no staging copies — the fastest way
// measured (74.2 GiB/s algorithmic on a 64 MiB fp32 chunk, BENCH_r05
// host_staged).
//
// Otherwise the chunk is staged through the caller's device scratch in one
// pass on the caller's stream: H2D dst, H2D src, the kernel, D2H dst (51.6
// GiB/s).  Rounds 2-5 pipelined that pass in pieces over three streams so
// that copies of different pieces overlapped; on MI355X the pipeline lost to
// the one pass at every piece size from 4 to 32 MiB (35.4-38.1 against 51.6
// GiB/s, BENCH_r05), so it is gone and piece_elems only chooses staging over
// zero-copy.
#include <hip/hip_runtime_api.h>

#include "gloo_amd.h"
#include "gloo_amd/common.h"
#include "gloo_amd/errors.h"
#include "gloo_amd/signal.h"

extern "C" int gloo_hip_reduce_staged(int op, int dtype, void* host_dst, const void* host_src, size_t n,
                                      void* dev_dst, void* dev_src, size_t piece_elems,
                                      gloo_hip_stream_t stream) {
  using namespace gloo_amd;
  try {
    const size_t es = gloo_hip_dtype_size(dtype);
    if (es == 0) return setError(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
    gloo_hip_custom_fn cfn;
    void* cuser;
    if (!isBuiltinOp(op) && !customOp(op, &cfn, &cuser)) return setError(GLOO_HIP_EINVAL_OP, "unknown reduction op");
    if (n == 0) return GLOO_HIP_OK;
    if (!host_dst || !host_src || !dev_dst || !dev_src) return setError(GLOO_HIP_EINVAL_PTR, "null buffer pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (piece_elems == 0) {
      void* mdst = nullptr;
      void* msrc = nullptr;
      const bool mapped = hipHostGetDevicePointer(&mdst, host_dst, 0) == hipSuccess &&
                          hipHostGetDevicePointer(&msrc, const_cast<void*>(host_src), 0) == hipSuccess &&
                          mdst && msrc;
      (void)hipGetLastError();  // a buffer that is not mapped is not an error here
      if (mapped) return gloo_hip_reduce(op, dtype, mdst, msrc, n, s);
    }
    const size_t bytes = n * es;
    GLOO_AMD_HIP_CHECK(hipMemcpyAsync(dev_dst, host_dst, bytes, hipMemcpyHostToDevice, s));
    GLOO_AMD_HIP_CHECK(hipMemcpyAsync(dev_src, host_src, bytes, hipMemcpyHostToDevice, s));
    const int rc = gloo_hip_reduce(op, dtype, dev_dst, dev_src, n, s);
    if (rc != GLOO_HIP_OK) return rc;
    GLOO_AMD_HIP_CHECK(hipMemcpyAsync(host_dst, dev_dst, bytes, hipMemcpyDeviceToHost, s));
    return GLOO_HIP_OK;
  } catch (const std::exception& e) {
    return setError(GLOO_HIP_EINVAL_ARG, e.what());
  }
}

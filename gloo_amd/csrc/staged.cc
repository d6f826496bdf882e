// staged.cc — the host-staged chunk reduction: chunks that
// start and end in host memory (a transport's receive buffer on a socket or
// NIC) reduced on the GPU.  The reference's CudaHostWorkspace path
// (gloo/cuda_collectives_host.h:22-136) copies device data to the host and
// reduces on the CPU; here the data goes the other way and the reduction
// stays the HIP kernel:
//
//   piece k:  H2D dst_k, H2D src_k  (copy-in stream)
//             kernel dst_k op= src_k (compute stream = the caller's)
//             D2H dst_k              (copy-out stream)
//
// Pieces are independent, so the copy-in of piece k+1, the kernel of piece k
// and the copy-out of piece k-1 overlap: PCIe is full duplex, so the H2D and
// D2H directions run at the same time on separate DMA engines, and the
// whole chunk costs about max(H2D bytes, D2H bytes) / link rate instead of
// their sum.  Streams and events are per thread and device, created once.
//
// Zero-copy (piece_elems == 0, both host buffers pinned and mapped into the
// device's address space): ONE kernel reads both operands over PCIe and
// writes the result back in place, with no staging copies.  The same 192 MiB
// cross the link, but as one stream of 16-B accesses: a 64 MiB fp32 chunk
// takes 2.54-2.59 ms against 2.96-3.01 ms pipelined in 16 MiB pieces
// (profiles/round3/r3aa_/r3ai_bench_n1*.json host_staged).  A buffer that is
// pinned but not mapped, or an explicit piece size, keeps the pipeline.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <map>
#include <vector>

#include "gloo_amd.h"
#include "gloo_amd/common.h"
#include "gloo_amd/errors.h"
#include "gloo_amd/signal.h"

namespace gloo_amd {
namespace {

struct StagingStreams {
  hipStream_t in = nullptr, out = nullptr;
  std::vector<hipEvent_t> inDone, redDone, outDone;
  hipEvent_t event(std::vector<hipEvent_t>& v, size_t k) {
    while (v.size() <= k) {
      hipEvent_t e;
      GLOO_AMD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      v.push_back(e);
    }
    return v[k];
  }
};

StagingStreams& streamsFor(int device) {
  thread_local std::map<int, StagingStreams> m;
  StagingStreams& s = m[device];
  if (!s.in) {
    GLOO_AMD_HIP_CHECK(hipStreamCreateWithFlags(&s.in, hipStreamNonBlocking));
    GLOO_AMD_HIP_CHECK(hipStreamCreateWithFlags(&s.out, hipStreamNonBlocking));
  }
  return s;
}

}  // namespace
}  // namespace gloo_amd

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
    int device = 0;
    GLOO_AMD_HIP_CHECK(hipGetDevice(&device));
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
    StagingStreams& st = streamsFor(device);
    // default: 16 MiB pieces (one MI355X: a 64 MiB fp32 chunk took 3.05 ms
    // in 16 MiB pieces against 5.2-5.8 ms in 4-8 MiB ones and 3.64 ms
    // unpipelined; profiles/round2/r2c_bench_n1.json host_staged)
    const size_t piece = piece_elems ? piece_elems : std::max<size_t>(1, (size_t)(16u << 20) / es);
    char* hd = static_cast<char*>(host_dst);
    const char* hs = static_cast<const char*>(host_src);
    char* dd = static_cast<char*>(dev_dst);
    char* ds = static_cast<char*>(dev_src);
    // the copy-in may not overwrite device scratch an earlier call on `s`
    // still uses, nor start before work the caller queued on `s`
    hipEvent_t start = st.event(st.outDone, 0);
    GLOO_AMD_HIP_CHECK(hipEventRecord(start, s));
    GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(st.in, start, 0));
    size_t k = 0;
    for (size_t off = 0; off < n; off += piece, k++) {
      const size_t len = std::min(piece, n - off);
      const size_t b = off * es, bytes = len * es;
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(dd + b, hd + b, bytes, hipMemcpyHostToDevice, st.in));
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(ds + b, hs + b, bytes, hipMemcpyHostToDevice, st.in));
      hipEvent_t in = st.event(st.inDone, k);
      GLOO_AMD_HIP_CHECK(hipEventRecord(in, st.in));
      GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(s, in, 0));
      const int rc = gloo_hip_reduce(op, dtype, dd + b, ds + b, len, s);
      if (rc != GLOO_HIP_OK) return rc;
      hipEvent_t red = st.event(st.redDone, k);
      GLOO_AMD_HIP_CHECK(hipEventRecord(red, s));
      GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(st.out, red, 0));
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(hd + b, dd + b, bytes, hipMemcpyDeviceToHost, st.out));
    }
    // the caller's stream covers the whole chunk, copy-out included
    hipEvent_t done = st.event(st.outDone, 1);
    GLOO_AMD_HIP_CHECK(hipEventRecord(done, st.out));
    GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(s, done, 0));
    return GLOO_HIP_OK;
  } catch (const std::exception& e) {
    return setError(GLOO_HIP_EINVAL_ARG, e.what());
  }
}

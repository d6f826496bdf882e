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
// Otherwise the chunk is staged through the caller's device scratch in
// pieces of at least 16 MiB:
//
//   piece k:  H2D dst_k, H2D src_k  (copy-in stream)
//             kernel dst_k op= src_k (the caller's stream)
//             D2H dst_k              (copy-out stream)
//
// so the copy-in of piece k+1, the kernel of piece k and the copy-out of
// piece k-1 overlap (PCIe is full duplex).  On one MI355X (BENCH_r05, 64 MiB
// fp32): 16 MiB pieces 62.5 GiB/s and 32 MiB 58.9 against 51.6 for one
// unpipelined pass, but 4 and 8 MiB pieces 35.4 and 38.1 (their per-piece
// event and copy overheads outweigh the overlap).  So a piece size below
// 16 MiB is raised to 16 MiB, and a chunk of at most one piece is staged in
// one pass on the caller's stream.  Streams and events are per thread and
// device, created once.
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

constexpr size_t kMinPieceBytes = size_t(16) << 20;

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
    const size_t minPiece = std::max<size_t>(1, kMinPieceBytes / es);
    const size_t piece = std::max(piece_elems, minPiece);
    char* hd = static_cast<char*>(host_dst);
    const char* hs = static_cast<const char*>(host_src);
    char* dd = static_cast<char*>(dev_dst);
    char* ds = static_cast<char*>(dev_src);
    if (n <= piece) {  // one pass on the caller's stream
      const size_t bytes = n * es;
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(dd, hd, bytes, hipMemcpyHostToDevice, s));
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(ds, hs, bytes, hipMemcpyHostToDevice, s));
      const int rc = gloo_hip_reduce(op, dtype, dd, ds, n, s);
      if (rc != GLOO_HIP_OK) return rc;
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(hd, dd, bytes, hipMemcpyDeviceToHost, s));
      return GLOO_HIP_OK;
    }
    int device = 0;
    GLOO_AMD_HIP_CHECK(hipGetDevice(&device));
    StagingStreams& st = streamsFor(device);
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

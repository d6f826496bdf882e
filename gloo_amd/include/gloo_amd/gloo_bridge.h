// gloo_bridge.h — the MI355X-native GPU algorithms behind Gloo's own
// gloo::Context / gloo::Algorithm surface.  HEADER-ONLY and compiled on the
// GLOO side: it includes the reference's headers and links against the
// user's libgloo plus libgloo_amd.so, while libgloo_amd.so itself never
// links (or includes) Gloo — everything below crosses the C-ABI of
// include/gloo_amd.h.
//
//   gloo::CudaAllreduceRingChunked<T, W>     -> gloo::HipAllreduceRingChunked<T, W>
//        (gloo/cuda_allreduce_ring_chunked.h:19-26)
//   gloo::CudaAllreduceHalvingDoubling<T, W> -> gloo::HipAllreduceHalvingDoubling<T, W>
//        (gloo/cuda_allreduce_halving_doubling.h:22-30)
//   gloo::CudaAllreduceRing<T, W>            -> gloo::HipAllreduceRing<T, W>
//        (gloo/cuda_allreduce_ring.h:20-24)
//   gloo::CudaAllreduceLocal<T, W>           -> gloo::HipAllreduceLocal<T, W>
//        (gloo/cuda_allreduce_local.h:19-23)
//   gloo::ReduceScatterHalvingDoubling<T>    -> gloo::HipReduceScatterHalvingDoubling<T, W>
//        (gloo/reduce_scatter.h:112-117; CPU-only in the reference)
//   gloo::CudaHostWorkspace / CudaDeviceWorkspace -> gloo::HipHostWorkspace / HipDeviceWorkspace
//        (gloo/cuda_workspace.h:20-31)
//
// Every class derives from gloo::Algorithm (gloo/algorithm.h:20-38) and is
// constructed from the program's existing std::shared_ptr<gloo::Context>,
// device pointers, `int count` and (optionally) one hipStream_t per pointer,
// exactly like the CUDA classes.  There is no second rendezvous: the
// library's own context (inbox arenas, their dma-buf references, signal mailboxes) is
// bootstrapped by gloo_hip_context_create_ex with gloo::allgather over the
// gloo::Context's pairs (gloo/allgather.h) as its only exchange.  Like the
// reference's algorithms, construction and destruction are collective:
// every rank constructs (and destroys) its algorithms in the same order.
//
// Errors follow the reference: a peer that does not answer within the
// context timeout raises gloo::IoException (gloo/common/error.h:42-48),
// anything else gloo::EnforceNotMet (gloo/common/logging.h:32-59).
//
// Stream semantics (docs/cuda.md:6-13 of the reference): without streams,
// run() returns with the outputs complete; with one stream per pointer
// (gloo/cuda_allreduce_ring_chunked.cc:55-67), run() orders its use of
// ptrs[i] after the work already queued on streams[i], and every streams[i]
// is ordered after the collective, so the caller synchronises with them.
//
// Element types: the reference's CUDA instantiations (gloo/cuda.cu:265-272),
// plus c10::BFloat16 when built with GLOO_USE_TORCH_DTYPES (cuda.cu:394-401).
// Reductions: the built-in ReductionType values run the library's kernels; a
// CUSTOM reduction is a gloo::HipReductionFunction<T> carrying a device
// function (the device half of CudaReductionFunction, gloo/cuda.h:286-358).
#pragma once

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "gloo/algorithm.h"
#include "gloo/allgather.h"
#include "gloo/common/error.h"
#include "gloo/common/logging.h"
#include "gloo/context.h"
#include "gloo/types.h"
#include "gloo_amd.h"
#include "gloo_amd/gloo_transport.h"

#if GLOO_USE_TORCH_DTYPES
#include <c10/util/BFloat16.h>
#endif

#include <map>
#include <mutex>

namespace gloo {

// Where the inboxes (the transport's receive buffers) live.
template <typename T>
struct HipDeviceWorkspace {
  static constexpr int kind = GLOO_HIP_WORKSPACE_DEVICE;
};
template <typename T>
struct HipHostWorkspace {
  static constexpr int kind = GLOO_HIP_WORKSPACE_HOST;
};

namespace hip_bridge {

template <typename T>
struct DType;
template <> struct DType<int8_t> { static constexpr int value = GLOO_HIP_I8; };
template <> struct DType<uint8_t> { static constexpr int value = GLOO_HIP_U8; };
template <> struct DType<int32_t> { static constexpr int value = GLOO_HIP_I32; };
template <> struct DType<uint32_t> { static constexpr int value = GLOO_HIP_U32; };
template <> struct DType<int64_t> { static constexpr int value = GLOO_HIP_I64; };
template <> struct DType<uint64_t> { static constexpr int value = GLOO_HIP_U64; };
template <> struct DType<float16> { static constexpr int value = GLOO_HIP_F16; };
template <> struct DType<float> { static constexpr int value = GLOO_HIP_F32; };
template <> struct DType<double> { static constexpr int value = GLOO_HIP_F64; };
#if GLOO_USE_TORCH_DTYPES
template <> struct DType<c10::BFloat16> { static constexpr int value = GLOO_HIP_BF16; };
#endif

// CUSTOM reductions: ReductionFunction<T> has no virtual members, so a
// HipReductionFunction<T> records its library op code here, keyed by its
// address, for as long as it lives.
struct CustomOps {
  std::mutex m;
  std::map<const void*, int> ops;
  static CustomOps& get() {
    static CustomOps* c = new CustomOps();
    return *c;
  }
};

// gloo::ReductionType (gloo/algorithm.h:49-57) -> gloo_hip_op_t (same values
// for the built-ins; a registered code >= GLOO_HIP_CUSTOM for CUSTOM).
template <typename T>
inline int opOf(const ReductionFunction<T>* fn) {
  GLOO_ENFORCE(fn != nullptr, "null reduction function");
  const ReductionType t = fn->type();
  if (t == SUM || t == PRODUCT || t == MAX || t == MIN) return static_cast<int>(t);
  GLOO_ENFORCE(t == CUSTOM, "unknown reduction type ", static_cast<int>(t));
  CustomOps& c = CustomOps::get();
  std::lock_guard<std::mutex> lk(c.m);
  auto it = c.ops.find(fn);
  GLOO_ENFORCE(it != c.ops.end(),
               "a CUSTOM reduction on device memory needs a device function: pass a gloo::HipReductionFunction<T>");
  return it->second;
}

inline void check(int rc, const char* what) {
  if (rc == GLOO_HIP_OK) return;
  const std::string msg = std::string(what) + ": " + gloo_hip_last_error();
  if (rc == GLOO_HIP_EIO) throw ::gloo::IoException(msg);  // timed out waiting for a peer
  GLOO_ENFORCE(false, msg);
}

inline int deviceOf(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) == hipSuccess && attr.device >= 0) return attr.device;
  (void)hipGetLastError();
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}

// The library context of one algorithm, bootstrapped over the gloo::Context:
// its only exchange is gloo::allgather of fixed records on a tag of its own
// (Slot::build(kAllgatherSlotPrefix, tag) — no context slot is consumed).
class BootstrapContext {
 public:
  static constexpr uint32_t kTag = 0x6e617664;  // distinct from a user's default tag 0

  BootstrapContext(const std::shared_ptr<Context>& context, int device) : context_(context) {
    check(gloo_hip_context_create_ex(context->rank, context->size, device,
                                     (int)context->getTimeout().count(), &BootstrapContext::allgather, this,
                                     &handle_),
          "gloo_hip_context_create_ex");
  }
  ~BootstrapContext() {
    if (handle_) (void)gloo_hip_context_destroy(handle_);
  }
  BootstrapContext(const BootstrapContext&) = delete;
  BootstrapContext& operator=(const BootstrapContext&) = delete;
  gloo_hip_context_t handle() const { return handle_; }

 private:
  static int allgather(void* user, const void* in, void* out, size_t block) {
    auto* self = static_cast<BootstrapContext*>(user);
    if (self->context_->size == 1) {  // nothing to exchange (a size-1 context may have no transport)
      std::memcpy(out, in, block);
      return 0;
    }
    try {
      // A gloo::Context on the xGMI transport (gloo_transport.h) already
      // sits on a library context: exchange through that context's store
      // rather than moving host records through the transport's own
      // unbound buffers.
      const int peer = self->context_->rank == 0 ? 1 : 0;
      if (auto* hp = dynamic_cast<transport::hip::Pair*>(self->context_->getPair(peer).get()))
        return hp->hipContext()->allgather(in, out, block);
      AllgatherOptions opts(self->context_);
      opts.setInput(const_cast<uint8_t*>(static_cast<const uint8_t*>(in)), block);
      opts.setOutput(static_cast<uint8_t*>(out), block * (size_t)self->context_->size);
      opts.setTag(kTag);
      ::gloo::allgather(opts);
      return 0;
    } catch (const std::exception&) {
      return 1;  // the library raises IoException for the failed exchange
    }
  }

  std::shared_ptr<Context> context_;
  gloo_hip_context_t handle_ = nullptr;
};

}  // namespace hip_bridge

// A CUSTOM reduction for the device path: the device half of
// CudaReductionFunction<T> (gloo/cuda.h:286-358), whose device function
// enqueues dst[i] = dst[i] op src[i] on a stream (cuda.h:288-290), with the
// host function the reference's ReductionFunction<T> calls (algorithm.h:59-95;
// optional: the device path never calls it).  The device function must not
// allocate or synchronise, as the reference requires of its device
// functions.  Pass it where a const ReductionFunction<T>* is taken; it must
// outlive the algorithms built with it.
template <typename T>
class HipReductionFunction : public ReductionFunction<T> {
 public:
  using DeviceFunction = void(T* dst, const T* src, size_t n, hipStream_t stream);

  explicit HipReductionFunction(DeviceFunction* dev, typename ReductionFunction<T>::Function* host = nullptr)
      : ReductionFunction<T>(CUSTOM, host ? host : &HipReductionFunction::noHost), dev_(dev) {
    GLOO_ENFORCE(dev != nullptr, "null device function");
    hip_bridge::check(gloo_hip_register_op(&HipReductionFunction::trampoline, this, &op_), "gloo_hip_register_op");
    auto& c = hip_bridge::CustomOps::get();
    std::lock_guard<std::mutex> lk(c.m);
    c.ops[this] = op_;
  }
  ~HipReductionFunction() {
    auto& c = hip_bridge::CustomOps::get();
    std::lock_guard<std::mutex> lk(c.m);
    c.ops.erase(this);
  }
  HipReductionFunction(const HipReductionFunction&) = delete;
  HipReductionFunction& operator=(const HipReductionFunction&) = delete;

  int op() const { return op_; }
  void callDevice(T* dst, const T* src, size_t n, hipStream_t stream) const { dev_(dst, src, n, stream); }

 private:
  // the library's custom op is three-operand (c = a op b, c may alias a)
  static void trampoline(void* user, void* c, const void* a, const void* b, size_t n, gloo_hip_stream_t s) {
    auto* self = static_cast<HipReductionFunction*>(user);
    hipStream_t stream = static_cast<hipStream_t>(s);
    if (c != a) (void)hipMemcpyAsync(c, a, n * sizeof(T), hipMemcpyDeviceToDevice, stream);
    self->dev_(static_cast<T*>(c), static_cast<const T*>(b), n, stream);
  }
  static void noHost(T*, const T*, size_t) {
    GLOO_ENFORCE(false, "this HipReductionFunction has no host function");
  }
  DeviceFunction* dev_;
  int op_ = 0;
};

// One of the library's schedule executors as a gloo::Algorithm.
template <typename T, int ALGO, typename W>
class HipPlanAlgorithm : public Algorithm {
 public:
  HipPlanAlgorithm(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, int count,
                   const std::vector<int>& recvElems, const std::vector<hipStream_t>& streams,
                   const ReductionFunction<T>* fn)
      : Algorithm(context) {
    GLOO_ENFORCE(!ptrs.empty(), "need at least one pointer");
    // gloo/cuda_allreduce_ring_chunked.cc:55-58
    GLOO_ENFORCE(streams.empty() || streams.size() == ptrs.size(), "one stream per pointer, or none");
    const int op = hip_bridge::opOf(fn);
    boot_.reset(new hip_bridge::BootstrapContext(context, hip_bridge::deviceOf(ptrs[0])));
    std::vector<void*> p(ptrs.begin(), ptrs.end());
    std::vector<gloo_hip_stream_t> s(streams.begin(), streams.end());
    hip_bridge::check(
        gloo_hip_algorithm_create_streams(boot_->handle(), ALGO, op, hip_bridge::DType<T>::value, p.data(),
                                          (int)p.size(), (size_t)(count > 0 ? count : 0),
                                          recvElems.empty() ? nullptr : recvElems.data(),
                                          s.empty() ? nullptr : s.data(), (int)s.size(), W::kind, &algo_),
        "gloo_hip_algorithm_create");
  }

  ~HipPlanAlgorithm() override {
    if (algo_) (void)gloo_hip_algorithm_destroy(algo_);  // collective: a tear-down barrier
  }

  void run() override { hip_bridge::check(gloo_hip_algorithm_run(algo_), "run"); }

 protected:
  std::unique_ptr<hip_bridge::BootstrapContext> boot_;
  gloo_hip_algorithm_t algo_ = nullptr;
};

template <typename T, typename W = HipDeviceWorkspace<T>>
class HipAllreduceRingChunked : public HipPlanAlgorithm<T, GLOO_HIP_ALGO_RING_CHUNKED, W> {
 public:
  HipAllreduceRingChunked(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, const int count,
                          const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                          const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : HipPlanAlgorithm<T, GLOO_HIP_ALGO_RING_CHUNKED, W>(context, ptrs, count, {}, streams, fn) {}
};

template <typename T, typename W = HipDeviceWorkspace<T>>
class HipAllreduceHalvingDoubling : public HipPlanAlgorithm<T, GLOO_HIP_ALGO_HALVING_DOUBLING, W> {
 public:
  // pipelineBroadcastAndReduce (gloo/cuda_allreduce_halving_doubling.h:29)
  // overlaps the reference's per-chunk local reduce / broadcast with the
  // exchange; here a rank's pointers are folded in one fused pass before the
  // exchange and broadcast in one pass after it, so the flag changes no
  // result and is accepted for source compatibility (DESIGN.md §8 round 6,
  // "Multi-pointer local passes").
  HipAllreduceHalvingDoubling(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, const int count,
                              const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                              bool /*pipelineBroadcastAndReduce*/ = false,
                              const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : HipPlanAlgorithm<T, GLOO_HIP_ALGO_HALVING_DOUBLING, W>(context, ptrs, count, {}, streams, fn) {}
};

// gloo::CudaAllreduceHalvingDoublingPipelined
// (gloo/cuda_allreduce_halving_doubling_pipelined.h:13-28).
template <typename T, typename W = HipDeviceWorkspace<T>>
class HipAllreduceHalvingDoublingPipelined : public HipAllreduceHalvingDoubling<T, W> {
 public:
  HipAllreduceHalvingDoublingPipelined(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                                       const int count,
                                       const std::vector<hipStream_t>& streams = std::vector<hipStream_t>())
      : HipAllreduceHalvingDoubling<T, W>(context, ptrs, count, streams, true) {}
};

// gloo::CudaAllreduceBcube (gloo/cuda_allreduce_bcube.h:50-58): groups of the
// program's context->base ranks (0 = 2, gloo/cuda_allreduce_bcube.cc:57).
template <typename T, typename W = HipDeviceWorkspace<T>>
class HipAllreduceBcube : public HipPlanAlgorithm<T, GLOO_HIP_ALGO_BCUBE, W> {
 public:
  HipAllreduceBcube(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, const int count,
                    const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                    const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : HipPlanAlgorithm<T, GLOO_HIP_ALGO_BCUBE, W>(context, ptrs, count, {context->base ? context->base : 2},
                                                    streams, fn) {}
};

template <typename T, typename W = HipDeviceWorkspace<T>>
class HipAllreduceRing : public HipPlanAlgorithm<T, GLOO_HIP_ALGO_RING, W> {
 public:
  HipAllreduceRing(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, const int count,
                   const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                   const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : HipPlanAlgorithm<T, GLOO_HIP_ALGO_RING, W>(context, ptrs, count, {}, streams, fn) {}
};

template <typename T, typename W = HipDeviceWorkspace<T>>
class HipAllreduceLocal : public HipPlanAlgorithm<T, GLOO_HIP_ALGO_LOCAL, W> {
 public:
  HipAllreduceLocal(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, const int count,
                    const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                    const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : HipPlanAlgorithm<T, GLOO_HIP_ALGO_LOCAL, W>(context, ptrs, count, {}, streams, fn) {}
};

template <typename T, typename W = HipDeviceWorkspace<T>>
class HipReduceScatterHalvingDoubling : public HipPlanAlgorithm<T, GLOO_HIP_ALGO_REDUCE_SCATTER, W> {
 public:
  HipReduceScatterHalvingDoubling(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                                  const int count, const std::vector<int>& recvElems,
                                  const ReductionFunction<T>* fn = ReductionFunction<T>::sum,
                                  const std::vector<hipStream_t>& streams = std::vector<hipStream_t>())
      : HipPlanAlgorithm<T, GLOO_HIP_ALGO_REDUCE_SCATTER, W>(context, ptrs, count, recvElems, streams, fn) {
    GLOO_ENFORCE_EQ((int)recvElems.size(), context->size, "recvElems needs one entry per rank");
  }
};

}  // namespace gloo

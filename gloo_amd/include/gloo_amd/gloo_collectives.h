// gloo_collectives.h — the reference's new-style collectives, called the way a
// Gloo program calls them, run on the MI355X path.
//
// HEADER-ONLY and compiled on the GLOO side (like gloo_bridge.h): it reads
// the reference's option objects and crosses into libgloo_amd.so only
// through the C-ABI of include/gloo_amd.h.
//
//   gloo::allreduce(const gloo::AllreduceOptions&)  (gloo/allreduce.h:89-193,
//        gloo/allreduce.cc:97-145)  ->  gloo::hip::allreduce(opts[, stream])
//   gloo::reduce(gloo::ReduceOptions&)               (gloo/reduce.h:19-110,
//        gloo/reduce.cc:21-247)     ->  gloo::hip::reduce(opts[, stream])
//
// The caller fills the SAME option object it would hand to gloo::allreduce /
// gloo::reduce: setInput(s) / setOutput(s) with DEVICE pointers (the
// context's createUnboundBuffer only records pointer and size; nothing is
// sent through it), setReduceFunction, setAlgorithm (RING, BCUBE), setTag,
// setMaxSegmentSize, setRoot.  The options are read through pointers to
// their protected members (taken in a derived class, so no layout is
// assumed).  Results are the reference's bits: the schedules are the
// reference's (RING and BCUBE segment geometry, reduce's ring + gather),
// verified against its outputs (tests/golden/newstyle_golden.npz).
//
// The element type and operation come from the reduce function, which is
// untyped in the options (gloo/allreduce.h:36): the reference's own
// gloo::sum / product / max / min<T> (gloo/math.h:15-73) map to the
// library's kernels for every instantiated T (+ c10::BFloat16 under
// GLOO_USE_TORCH_DTYPES); any other function must be registered with a
// device implementation (registerReduction, ReductionType CUSTOM), because
// a host function cannot run on device memory.
//
// Streams (docs/cuda.md:6-13): without one, the outputs are complete on
// return; with one, the work is ordered on it and the caller synchronises.
//
// The library context behind a gloo::Context is created by the first call on
// it (a collective exchange over gloo::allgather, as for gloo_bridge.h's
// algorithms) and kept, with the cached schedules, until releaseContext —
// a collective call every rank makes while the gloo::Context is alive.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "gloo/allreduce.h"
#include "gloo/math.h"
#include "gloo/reduce.h"
#include "gloo_amd/gloo_bridge.h"

namespace gloo {
namespace hip {

namespace detail {

using ReduceFn = void (*)(void*, const void*, const void*, size_t);

struct Reduction {
  int op = 0;
  int dtype = -1;
  size_t elementSize = 0;
};

struct Registry {
  std::mutex m;
  std::vector<std::pair<ReduceFn, Reduction>> fns;
  template <typename T>
  void builtins() {
    const int dt = ::gloo::hip_bridge::DType<T>::value;
    fns.push_back({static_cast<ReduceFn>(&::gloo::sum<T>), {GLOO_HIP_SUM, dt, sizeof(T)}});
    fns.push_back({static_cast<ReduceFn>(&::gloo::product<T>), {GLOO_HIP_PRODUCT, dt, sizeof(T)}});
    fns.push_back({static_cast<ReduceFn>(&::gloo::max<T>), {GLOO_HIP_MAX, dt, sizeof(T)}});
    fns.push_back({static_cast<ReduceFn>(&::gloo::min<T>), {GLOO_HIP_MIN, dt, sizeof(T)}});
  }
  static Registry& get() {
    static Registry* r = [] {
      auto* x = new Registry();
      x->builtins<int8_t>();
      x->builtins<uint8_t>();
      x->builtins<int32_t>();
      x->builtins<uint32_t>();
      x->builtins<int64_t>();
      x->builtins<uint64_t>();
      x->builtins<::gloo::float16>();
      x->builtins<float>();
      x->builtins<double>();
#if GLOO_USE_TORCH_DTYPES
      x->builtins<c10::BFloat16>();
#endif
      return x;
    }();
    return *r;
  }
};

// The operation and element type of an options object's reduce function.
inline Reduction classify(const std::function<void(void*, const void*, const void*, size_t)>& f,
                          size_t elementSize) {
  GLOO_ENFORCE(f, "no reduce function set (setReduceFunction)");
  const ReduceFn* target = f.target<ReduceFn>();
  GLOO_ENFORCE(target != nullptr,
               "the device path needs the reduce function as a plain function pointer: one of "
               "gloo::sum/product/max/min<T> or a function registered with gloo::hip::registerReduction");
  Registry& r = Registry::get();
  std::lock_guard<std::mutex> lk(r.m);
  for (const auto& e : r.fns)
    if (e.first == *target) {
      GLOO_ENFORCE_EQ(e.second.elementSize, elementSize, "the reduce function's element size differs from the "
                                                         "buffers' (setInput<T> / setOutput<T>)");
      return e.second;
    }
  GLOO_ENFORCE(false, "unknown reduce function: register its device implementation with "
                      "gloo::hip::registerReduction");
  return {};
}

// The library context of one gloo::Context (kept until releaseContext).
struct Contexts {
  std::mutex m;
  std::map<const ::gloo::Context*, std::pair<std::shared_ptr<::gloo::Context>,
                                             std::unique_ptr<::gloo::hip_bridge::BootstrapContext>>> byContext;
  static Contexts& get() {
    static Contexts* c = new Contexts();  // never destroyed: tear-down is collective (releaseContext)
    return *c;
  }
};

inline gloo_hip_context_t contextFor(const std::shared_ptr<::gloo::Context>& c, const void* anyDevicePtr) {
  Contexts& cs = Contexts::get();
  {
    std::lock_guard<std::mutex> lk(cs.m);
    auto it = cs.byContext.find(c.get());
    if (it != cs.byContext.end()) return it->second.second->handle();
  }
  // The bootstrap is collective: never under the registry's lock, which the
  // other ranks of this process (threads) need for their own contexts.
  std::unique_ptr<::gloo::hip_bridge::BootstrapContext> boot(
      new ::gloo::hip_bridge::BootstrapContext(c, ::gloo::hip_bridge::deviceOf(anyDevicePtr)));
  std::lock_guard<std::mutex> lk(cs.m);
  auto& e = cs.byContext[c.get()];
  e.first = c;
  e.second = std::move(boot);
  return e.second->handle();
}

// Read access to the options' protected state: pointers to members named
// in a derived class (no object of the derived type is ever formed).
struct AllreduceAccess : ::gloo::AllreduceOptions {
  static const ::gloo::detail::AllreduceOptionsImpl& impl(const ::gloo::AllreduceOptions& o) {
    return o.*(&AllreduceAccess::impl_);
  }
};
struct ReduceAccess : ::gloo::ReduceOptions {
  static const std::shared_ptr<::gloo::Context>& get_context(const ::gloo::ReduceOptions& o) {
    return o.*(&ReduceAccess::context);
  }
  static const std::unique_ptr<::gloo::transport::UnboundBuffer>& get_in(const ::gloo::ReduceOptions& o) {
    return o.*(&ReduceAccess::in);
  }
  static const std::unique_ptr<::gloo::transport::UnboundBuffer>& get_out(const ::gloo::ReduceOptions& o) {
    return o.*(&ReduceAccess::out);
  }
  static size_t get_elements(const ::gloo::ReduceOptions& o) { return o.*(&ReduceAccess::elements); }
  static size_t get_elementSize(const ::gloo::ReduceOptions& o) { return o.*(&ReduceAccess::elementSize); }
  static int get_root(const ::gloo::ReduceOptions& o) { return o.*(&ReduceAccess::root); }
  static const Func& get_reduce(const ::gloo::ReduceOptions& o) { return o.*(&ReduceAccess::reduce); }
  static uint32_t get_tag(const ::gloo::ReduceOptions& o) { return o.*(&ReduceAccess::tag); }
  static size_t get_maxSegmentSize(const ::gloo::ReduceOptions& o) { return o.*(&ReduceAccess::maxSegmentSize); }
};

}  // namespace detail

// A CUSTOM reduce function for the new-style calls: `host` is what the
// caller passes to setReduceFunction (the reference calls it on host
// memory), `device` its device implementation (gloo_bridge.h), which must
// outlive every call that uses it.
template <typename T>
void registerReduction(detail::ReduceFn host, const ::gloo::HipReductionFunction<T>& device) {
  GLOO_ENFORCE(host != nullptr, "null host function");
  detail::Registry& r = detail::Registry::get();
  std::lock_guard<std::mutex> lk(r.m);
  for (auto& e : r.fns)
    if (e.first == host) {
      e.second = {device.op(), ::gloo::hip_bridge::DType<T>::value, sizeof(T)};
      return;
    }
  r.fns.push_back({host, {device.op(), ::gloo::hip_bridge::DType<T>::value, sizeof(T)}});
}

// gloo::allreduce(opts) (gloo/allreduce.cc:97-145) on device buffers.
inline void allreduce(const ::gloo::AllreduceOptions& opts, hipStream_t stream = nullptr) {
  const auto& o = detail::AllreduceAccess::impl(opts);
  GLOO_ENFORCE(o.out.size() > 0, "no output buffer");  // gloo/allreduce.cc:102
  if (o.elements == 0) return;                          // gloo/allreduce.cc:98-100
  const detail::Reduction red = detail::classify(o.reduce, o.elementSize);
  std::vector<void*> ins, outs;
  for (const auto& b : o.in) {
    GLOO_ENFORCE_GE(b->size, o.elements * o.elementSize, "input buffer too small");
    ins.push_back(b->ptr);
  }
  for (const auto& b : o.out) {
    GLOO_ENFORCE_GE(b->size, o.elements * o.elementSize, "output buffer too small");
    outs.push_back(b->ptr);
  }
  GLOO_ENFORCE(o.algorithm == ::gloo::detail::AllreduceOptionsImpl::UNSPECIFIED ||
                   o.algorithm == ::gloo::detail::AllreduceOptionsImpl::RING ||
                   o.algorithm == ::gloo::detail::AllreduceOptionsImpl::BCUBE,
               "Algorithm not handled.");  // gloo/allreduce.cc:142-143
  gloo_hip_context_t ctx = detail::contextFor(o.context, outs[0]);
  gloo_hip_allreduce_options_t a;
  a.algorithm = o.algorithm == ::gloo::detail::AllreduceOptionsImpl::BCUBE ? GLOO_HIP_ALLREDUCE_BCUBE
                                                                            : GLOO_HIP_ALLREDUCE_RING;
  a.op = red.op;
  a.dtype = red.dtype;
  a.inputs = ins.empty() ? nullptr : ins.data();
  a.ninputs = (int)ins.size();
  a.outputs = outs.data();
  a.noutputs = (int)outs.size();
  a.elements = o.elements;
  a.max_segment_bytes = o.maxSegmentSize;
  a.tag = o.tag;
  a.stream = stream;
  ::gloo::hip_bridge::check(gloo_hip_allreduce(ctx, &a), "gloo::hip::allreduce");
}

// gloo::reduce(opts) (gloo/reduce.cc:21-247) on device buffers: only the
// root's output holds the result, as in the reference.
inline void reduce(::gloo::ReduceOptions& opts, hipStream_t stream = nullptr) {
  using A = detail::ReduceAccess;
  const auto& ctxp = A::get_context(opts);
  const size_t elements = A::get_elements(opts);
  if (elements == 0) return;  // gloo/reduce.cc:22-24
  GLOO_ENFORCE(A::get_out(opts), "no output buffer");
  const int root = A::get_root(opts);
  GLOO_ENFORCE(root >= 0 && root < ctxp->size, "invalid root ", root);  // gloo/reduce.cc:31-32
  const detail::Reduction red = detail::classify(A::get_reduce(opts), A::get_elementSize(opts));
  void* out = A::get_out(opts)->ptr;
  void* in = A::get_in(opts) ? A::get_in(opts)->ptr : nullptr;
  gloo_hip_context_t ctx = detail::contextFor(ctxp, out);
  gloo_hip_reduce_options_t r;
  r.op = red.op;
  r.dtype = red.dtype;
  r.input = in;
  r.output = out;
  r.elements = elements;
  r.root = root;
  r.max_segment_bytes = A::get_maxSegmentSize(opts);
  r.tag = A::get_tag(opts);
  r.stream = stream;
  ::gloo::hip_bridge::check(gloo_hip_reduce_to_root(ctx, &r), "gloo::hip::reduce");
}

// Collective: tears down the library context (and its cached schedules)
// behind `context`; every rank calls it, in the same order relative to its
// other collectives, while the gloo::Context is alive.
inline void releaseContext(const std::shared_ptr<::gloo::Context>& context) {
  detail::Contexts& cs = detail::Contexts::get();
  std::unique_ptr<::gloo::hip_bridge::BootstrapContext> boot;
  {
    std::lock_guard<std::mutex> lk(cs.m);
    auto it = cs.byContext.find(context.get());
    if (it == cs.byContext.end()) return;
    boot = std::move(it->second.second);
    cs.byContext.erase(it);
  }
  boot.reset();
}

}  // namespace hip
}  // namespace gloo

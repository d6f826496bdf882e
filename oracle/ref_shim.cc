// ref_shim.cc — ORACLE / TEST INFRASTRUCTURE ONLY.  Never linked into the
// product (gloo_amd/), never on a measured path except bench.py's
// `cpu_baseline` leg.
//
// A thin extern "C" driver around the UNMODIFIED reference, compiled from the
// sources under /root/reference by oracle/Makefile into oracle/_ref/.  It lets
// Python tests and the golden-vector generator call:
//   * gloo::sum/product/max/min<T>(c, a, b, n)       gloo/math.h:15-73
//     (float16 through the F16C specialisations of gloo/math.cc:17-97)
//   * AllreduceRingChunked<T>                        gloo/allreduce_ring_chunked.h
//   * AllreduceHalvingDoubling<T>                    gloo/allreduce_halving_doubling.h
//   * AllreduceRing<T>                               gloo/allreduce_ring.h
//   * AllreduceBcube<T>                              gloo/allreduce_bcube.h
//   * ReduceScatterHalvingDoubling<T>                gloo/reduce_scatter.h
//   * AllreduceLocal<T>                              gloo/allreduce_local.{h,cc}
// with P ranks as threads in one process over the reference's own TCP
// transport on localhost and an in-memory HashStore — the pattern of the
// reference's own tests (gloo/test/base_test.h:107-152).
//
// bf16 uses c10::BFloat16 from the installed PyTorch headers, the type the
// reference's CUDA bf16 instantiations name (gloo/cuda.cu:394-401).

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <c10/util/BFloat16.h>

#include "gloo/allreduce.h"
#include "gloo/allreduce_bcube.h"
#include "gloo/allreduce_halving_doubling.h"
#include "gloo/allreduce_local.h"
#include "gloo/allreduce_ring.h"
#include "gloo/allreduce_ring_chunked.h"
#include "gloo/math.h"
#include "gloo/reduce.h"
#include "gloo/reduce_scatter.h"
#include "gloo/rendezvous/context.h"
#include "gloo/rendezvous/hash_store.h"
#include "gloo/transport/tcp/device.h"
#include "gloo/types.h"

namespace {

thread_local std::string g_err;

// dtype / op codes identical to include/gloo_amd.h
enum { I8, U8, I32, U32, I64, U64, F16, BF16, F32, F64 };
enum { SUM = 1, PRODUCT = 2, MAX = 3, MIN = 4 };

template <typename T>
using Fn3 = void (*)(void*, const void*, const void*, size_t);

template <typename T>
Fn3<T> pick3(int op) {
  switch (op) {
    case SUM: return &gloo::sum<T>;
    case PRODUCT: return &gloo::product<T>;
    case MAX: return &gloo::max<T>;
    case MIN: return &gloo::min<T>;
  }
  return nullptr;
}

template <typename T>
const gloo::ReductionFunction<T>* pickFn(int op) {
  switch (op) {
    case SUM: return gloo::ReductionFunction<T>::sum;
    case PRODUCT: return gloo::ReductionFunction<T>::product;
    case MAX: return gloo::ReductionFunction<T>::max;
    case MIN: return gloo::ReductionFunction<T>::min;
  }
  return nullptr;
}

template <typename T>
int reduce3(int op, void* c, const void* a, const void* b, size_t n) {
  auto fn = pick3<T>(op);
  if (!fn) return -1;
  fn(c, a, b, n);
  return 0;
}

// Route every fp16 element through the F16C body (gloo/math.cc:24-31): pad to
// a multiple of 8 so the scalar `leftovers` loop, which goes through the
// defective float16::operator=, never runs.
int reduce3_f16_vector_only(int op, void* c, const void* a, const void* b, size_t n) {
  const size_t np = (n + 7) / 8 * 8;
  std::vector<gloo::float16> pa(np), pb(np), pc(np);
  std::memcpy(pa.data(), a, n * 2);
  std::memcpy(pb.data(), b, n * 2);
  int rc = reduce3<gloo::float16>(op, pc.data(), pa.data(), pb.data(), np);
  std::memcpy(c, pc.data(), n * 2);
  return rc;
}

class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    const int gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      gen_++;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen != gen_; });
    }
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0, gen_ = 0;
};

// Spawn P ranks as threads, connect a full mesh over TCP localhost, run fn.
int spawn(int P, const std::function<void(std::shared_ptr<gloo::Context>)>& fn, int base = 2) {
  auto store = std::make_shared<gloo::rendezvous::HashStore>();
  Barrier barrier(P);
  std::vector<std::thread> threads;
  std::mutex em;
  std::string first_error;
  for (int rank = 0; rank < P; rank++) {
    threads.emplace_back([&, rank] {
      try {
        auto ctx = std::make_shared<gloo::rendezvous::Context>(rank, P, base);
        ctx->setTimeout(std::chrono::seconds(60));
        if (P > 1) {
          gloo::transport::tcp::attr attr("localhost");
          auto dev = gloo::transport::tcp::CreateDevice(attr);
          ctx->connectFullMesh(store, dev);
        }
        fn(ctx);
        barrier.wait();
        if (P > 1) ctx->closeConnections();
      } catch (std::exception& e) {
        std::lock_guard<std::mutex> lk(em);
        if (first_error.empty()) first_error = e.what();
        barrier.wait();
      }
    });
  }
  for (auto& t : threads) t.join();
  if (!first_error.empty()) {
    g_err = first_error;
    return -10;
  }
  return 0;
}

// AllreduceLocal is only instantiated for the types of
// gloo/allreduce_local.cc:42-51; the others get no local algorithm.
template <typename T>
void run_local(std::shared_ptr<gloo::Context> ctx, std::vector<T*>& ptrs, int count,
               const gloo::ReductionFunction<T>* fn) {
  constexpr bool ok = std::is_same<T, int8_t>::value || std::is_same<T, uint8_t>::value ||
                      std::is_same<T, int32_t>::value || std::is_same<T, int64_t>::value ||
                      std::is_same<T, uint64_t>::value || std::is_same<T, float>::value ||
                      std::is_same<T, double>::value || std::is_same<T, gloo::float16>::value;
  if constexpr (ok) {
    gloo::AllreduceLocal<T> a(ctx, ptrs, count, fn);
    a.run();
  } else {
    throw std::runtime_error("AllreduceLocal not instantiated for this type");
  }
}

enum { ALGO_RING_CHUNKED = 0, ALGO_HALVING_DOUBLING = 1, ALGO_RING = 2, ALGO_LOCAL = 3 };

template <typename T>
int allreduce(int algo, int op, int P, int k, size_t n, const void* in, void* out) {
  const auto* fn = pickFn<T>(op);
  if (!fn) return -1;
  const T* src = static_cast<const T*>(in);
  T* dst = static_cast<T*>(out);
  std::memcpy(dst, src, sizeof(T) * (size_t)P * k * n);
  return spawn(P, [&](std::shared_ptr<gloo::Context> ctx) {
    std::vector<T*> ptrs;
    for (int j = 0; j < k; j++) ptrs.push_back(dst + ((size_t)ctx->rank * k + j) * n);
    const int count = (int)n;
    if (algo == ALGO_RING_CHUNKED) {
      gloo::AllreduceRingChunked<T> a(ctx, ptrs, count, fn);
      a.run();
    } else if (algo == ALGO_HALVING_DOUBLING) {
      gloo::AllreduceHalvingDoubling<T> a(ctx, ptrs, count, fn);
      a.run();
    } else if (algo == ALGO_RING) {
      gloo::AllreduceRing<T> a(ctx, ptrs, count, fn);
      a.run();
    } else {
      run_local<T>(ctx, ptrs, count, fn);
    }
  });
}

template <typename T>
int reduce_scatter(int op, int P, size_t n, const int* recvElems, const void* in, void* out) {
  const auto* fn = pickFn<T>(op);
  if (!fn) return -1;
  T* dst = static_cast<T*>(out);
  std::memcpy(dst, in, sizeof(T) * (size_t)P * n);
  std::vector<int> re(recvElems, recvElems + P);
  return spawn(P, [&](std::shared_ptr<gloo::Context> ctx) {
    std::vector<T*> ptrs{dst + (size_t)ctx->rank * n};
    gloo::ReduceScatterHalvingDoubling<T> a(ctx, ptrs, (int)n, re, fn);
    a.run();
  });
}

// AllreduceBcube<T> (gloo/allreduce_bcube.h) on a context of the given base
// (gloo/context.h:28).  in/out laid out [P][k][n].
template <typename T>
int allreduce_bcube(int op, int P, int base, int k, size_t n, const void* in, void* out) {
  const auto* fn = pickFn<T>(op);
  if (!fn) return -1;
  T* dst = static_cast<T*>(out);
  std::memcpy(dst, in, sizeof(T) * (size_t)P * k * n);
  return spawn(
      P,
      [&](std::shared_ptr<gloo::Context> ctx) {
        std::vector<T*> ptrs;
        for (int j = 0; j < k; j++) ptrs.push_back(dst + ((size_t)ctx->rank * k + j) * n);
        gloo::AllreduceBcube<T> a(ctx, ptrs, (int)n, fn);
        a.run();
      },
      base);
}

// New-style gloo::allreduce(opts), RING (gloo/allreduce.cc:147-392) or BCUBE
// (:428-669), as `algorithm` (AllreduceOptions::Algorithm, gloo/allreduce.h:38-42).
// in: [P][nin][n] (nin may be 0: outputs are the inputs); out: [P][nout][n].
template <typename T>
int allreduce_new(int algorithm, int op, int P, int nin, int nout, size_t n, size_t maxSeg, const void* in,
                  void* out) {
  Fn3<T> fn = pick3<T>(op);
  if (!fn) return -1;
  std::vector<T> inputs((size_t)P * nin * n);
  if (nin) std::memcpy(inputs.data(), in, inputs.size() * sizeof(T));
  T* o = static_cast<T*>(out);
  return spawn(P, [&](std::shared_ptr<gloo::Context> ctx) {
    gloo::AllreduceOptions opts(ctx);
    std::vector<T*> ip, op_;
    for (int j = 0; j < nin; j++) ip.push_back(inputs.data() + ((size_t)ctx->rank * nin + j) * n);
    for (int j = 0; j < nout; j++) op_.push_back(o + ((size_t)ctx->rank * nout + j) * n);
    if (nin) opts.setInputs(ip, n);
    opts.setOutputs(op_, n);
    opts.setAlgorithm(algorithm == 2 ? gloo::AllreduceOptions::Algorithm::BCUBE
                                     : gloo::AllreduceOptions::Algorithm::RING);
    opts.setReduceFunction(fn);
    if (maxSeg) opts.setMaxSegmentSize(maxSeg);
    gloo::allreduce(opts);
  });
}

// New-style gloo::reduce(opts) (gloo/reduce.cc:21-247).  in: [P][n] (used
// when has_input); out: [P][n] initial outputs, every rank's output after.
template <typename T>
int reduce_new(int op, int P, int has_input, size_t n, size_t maxSeg, int root, const void* in, void* out) {
  Fn3<T> fn = pick3<T>(op);
  if (!fn) return -1;
  std::vector<T> inputs(has_input ? (size_t)P * n : 0);
  if (has_input) std::memcpy(inputs.data(), in, inputs.size() * sizeof(T));
  T* o = static_cast<T*>(out);
  return spawn(P, [&](std::shared_ptr<gloo::Context> ctx) {
    gloo::ReduceOptions opts(ctx);
    if (has_input) opts.setInput(inputs.data() + (size_t)ctx->rank * n, n);
    opts.setOutput(o + (size_t)ctx->rank * n, n);
    opts.setRoot(root);
    opts.setReduceFunction(fn);
    if (maxSeg) opts.setMaxSegmentSize(maxSeg);
    gloo::reduce(opts);
  });
}

#define DISPATCH(dtype, CALL)                     \
  switch (dtype) {                                \
    case I8: { using T = int8_t; return CALL; }   \
    case U8: { using T = uint8_t; return CALL; }  \
    case I32: { using T = int32_t; return CALL; } \
    case U32: { using T = uint32_t; return CALL; } \
    case I64: { using T = int64_t; return CALL; } \
    case U64: { using T = uint64_t; return CALL; } \
    case F16: { using T = gloo::float16; return CALL; } \
    case BF16: { using T = c10::BFloat16; return CALL; } \
    case F32: { using T = float; return CALL; }   \
    case F64: { using T = double; return CALL; }  \
    default: return -2;                           \
  }

}  // namespace

extern "C" {

// gloo::<op><T>(c, a, b, n).  fp16 goes through the F16C vector body only.
int ref_reduce3(int op, int dtype, void* c, const void* a, const void* b, size_t n) {
  if (dtype == F16) return reduce3_f16_vector_only(op, c, a, b, n);
  DISPATCH(dtype, reduce3<T>(op, c, a, b, n));
}

// The scalar float16 path exactly as it ships when GLOO_USE_AVX is off
// (gloo/types.h:96-204), kept to pin the App. A.1 defect in a test.
int ref_reduce3_f16_scalar(int op, void* c, const void* a, const void* b, size_t n) {
  gloo::float16* pc = static_cast<gloo::float16*>(c);
  const gloo::float16* pa = static_cast<const gloo::float16*>(a);
  const gloo::float16* pb = static_cast<const gloo::float16*>(b);
  for (size_t i = 0; i < n; i++) {
    if (op == SUM) pc[i] = pa[i] + pb[i];
    else if (op == PRODUCT) pc[i] = pa[i] * pb[i];
    else if (op == MAX) pc[i] = std::max(pa[i], pb[i]);
    else pc[i] = std::min(pa[i], pb[i]);
  }
  return 0;
}

// P ranks x k pointers x n elements, in/out laid out [P][k][n].
int ref_allreduce(int algo, int op, int dtype, int P, int k, size_t n, const void* in,
                  void* out) {
  DISPATCH(dtype, allreduce<T>(algo, op, P, k, n, in, out));
}

// AllreduceBcube over P ranks of context base `base`, k pointers each.
int ref_allreduce_bcube(int op, int dtype, int P, int base, int k, size_t n, const void* in, void* out) {
  DISPATCH(dtype, allreduce_bcube<T>(op, P, base, k, n, in, out));
}

// New-style allreduce; out holds the initial outputs and receives the result.
int ref_allreduce_new(int op, int dtype, int P, int nin, int nout, size_t n, size_t maxSeg,
                      const void* in, void* out) {
  DISPATCH(dtype, allreduce_new<T>(1, op, P, nin, nout, n, maxSeg, in, out));
}

// The same with the algorithm chosen: 1 = RING, 2 = BCUBE.
int ref_allreduce_new_algo(int algorithm, int op, int dtype, int P, int nin, int nout, size_t n, size_t maxSeg,
                           const void* in, void* out) {
  DISPATCH(dtype, allreduce_new<T>(algorithm, op, P, nin, nout, n, maxSeg, in, out));
}

// New-style reduce; out holds the initial outputs and receives every rank's output.
int ref_reduce_new(int op, int dtype, int P, int has_input, size_t n, size_t maxSeg, int root, const void* in,
                   void* out) {
  DISPATCH(dtype, reduce_new<T>(op, P, has_input, n, maxSeg, root, in, out));
}

// P ranks x n elements; rank r's reduced block lands at out[r][0:recvElems[r]].
int ref_reduce_scatter(int op, int dtype, int P, size_t n, const int* recvElems,
                       const void* in, void* out) {
  DISPATCH(dtype, reduce_scatter<T>(op, P, n, recvElems, in, out));
}

// BASELINE config 1 timing: construct the reference algorithm once per rank,
// then time `iters` run() calls (threads over TCP localhost, the reference's
// own benchmark shape, gloo/benchmark/runner.cc:279-366).  Returns the
// slowest rank's mean seconds per run in *sec.
int ref_allreduce_timed(int algo, int P, size_t n, int iters, double* sec) {
  std::vector<float> data((size_t)P * n, 1.0f);
  std::vector<double> per(P, 0.0);
  const auto* fn = gloo::ReductionFunction<float>::sum;
  int rc = spawn(P, [&](std::shared_ptr<gloo::Context> ctx) {
    std::vector<float*> ptrs{data.data() + (size_t)ctx->rank * n};
    std::unique_ptr<gloo::Algorithm> a;
    if (algo == ALGO_RING_CHUNKED) a.reset(new gloo::AllreduceRingChunked<float>(ctx, ptrs, (int)n, fn));
    else a.reset(new gloo::AllreduceHalvingDoubling<float>(ctx, ptrs, (int)n, fn));
    a->run();  // warmup
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++) a->run();
    per[ctx->rank] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
  });
  double m = 0;
  for (double v : per) m = v > m ? v : m;
  *sec = m;
  return rc;
}

// BASELINE config 1 with the reference benchmark's methodology
// (gloo/benchmark/runner.cc:311-363): `warmup` untimed-for-the-result runs,
// an iteration count from the warmup median so one batch lasts about
// `min_seconds`, batches grown x2 until a batch's per-rank time exceeds
// `min_seconds` (rank 0 decides, every rank follows), and every iteration of
// every rank of the last batch kept as a latency sample (seconds).  At most
// `max_samples` are written; *count receives how many.
int ref_allreduce_samples(int algo, int P, size_t n, int warmup, double min_seconds, double* samples,
                          int max_samples, int* count) {
  std::vector<float> data((size_t)P * n, 1.0f);
  const auto* fn = gloo::ReductionFunction<float>::sum;
  Barrier bar(P);
  std::atomic<long> iterations{0};
  std::atomic<int> done{0};
  std::vector<std::vector<double>> per(P);
  int rc = spawn(P, [&](std::shared_ptr<gloo::Context> ctx) {
    const int r = ctx->rank;
    std::vector<float*> ptrs{data.data() + (size_t)r * n};
    std::unique_ptr<gloo::Algorithm> a;
    if (algo == ALGO_RING_CHUNKED) a.reset(new gloo::AllreduceRingChunked<float>(ctx, ptrs, (int)n, fn));
    else a.reset(new gloo::AllreduceHalvingDoubling<float>(ctx, ptrs, (int)n, fn));
    auto timeOne = [&] {
      const auto t0 = std::chrono::steady_clock::now();
      a->run();
      return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    std::vector<double> w;
    for (int i = 0; i < std::max(1, warmup); i++) w.push_back(timeOne());
    std::sort(w.begin(), w.end());
    if (r == 0) iterations = std::max(1L, (long)(min_seconds / std::max(1e-9, w[w.size() / 2])));
    bar.wait();
    for (;;) {
      const long it = iterations.load();
      std::vector<double> s;
      for (long i = 0; i < it; i++) s.push_back(timeOne());
      double total = 0;
      for (double v : s) total += v;
      per[r] = std::move(s);
      if (r == 0) {
        const bool enough = total > min_seconds || it >= 1000000;
        done = enough ? 1 : 0;
        if (!enough) iterations = std::max(it + 1, (long)(it * 2));
      }
      bar.wait();
      if (done.load()) break;
      bar.wait();  // nobody re-reads `done` before rank 0 rewrites it
    }
  });
  int k = 0;
  for (auto& s : per)
    for (double v : s)
      if (k < max_samples) samples[k++] = v;
  *count = k;
  return rc;
}

const char* ref_last_error() { return g_err.c_str(); }

}  // extern "C"

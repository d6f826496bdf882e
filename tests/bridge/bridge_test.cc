// bridge_test.cc — TEST PROGRAM (built by oracle/Makefile where the reference
// sources exist; the binary travels to the GPU box, the reference does not).
//
// A Gloo program that uses the MI355X-native algorithms through Gloo's own
// surface (gloo_amd/include/gloo_amd/gloo_bridge.h): ranks are threads with
// a gloo::rendezvous::Context each, connected over the reference's TCP
// transport (gloo/test/base_test.h:107-152); every rank hands its
// std::shared_ptr<gloo::Context> to gloo::HipAllreduce*<T>, which derives from
// gloo::Algorithm.  Mirrors gloo/test/cuda_allreduce_test.cc:60-349:
// SinglePointer / MultiPointer / MultiPointerAsync (user streams) across
// ring, ring-chunked, halving-doubling (+ pipelined), bcube, fp16, plus the
// reduce-scatter, the host workspace and the IoException on a silent peer.
// Expected values: the closed form of gloo/test/base_test.h:184-236.
//
// Usage: bridge_test [case-filter]   (prints one line per case, exit 0 = ok)
#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gloo/rendezvous/context.h"
#include "gloo/rendezvous/hash_store.h"
#include "gloo/transport/tcp/device.h"
#include "gloo_amd/gloo_bridge.h"

// tests/bridge/libbridge_kernels.so (test_kernels.hip)
extern "C" int bt_spin(hipStream_t stream, unsigned long long ticks);
extern "C" void bt_add_i32(int32_t* dst, const int32_t* src, size_t n, hipStream_t stream);
extern "C" long bt_add_i32_calls(void);

namespace {

#define HIPOK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

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

// P ranks as threads; each gets a connected gloo::Context (timeout `ms`).
// base: gloo::Context::base (gloo/context.h:28), AllreduceBcube's group size.
std::string spawn(int P, int ms, const std::function<void(std::shared_ptr<gloo::Context>)>& fn, bool gpu = true,
                  int base = 2) {
  auto store = std::make_shared<gloo::rendezvous::HashStore>();
  Barrier barrier(P);
  std::vector<std::thread> ts;
  std::mutex em;
  std::string err;
  for (int rank = 0; rank < P; rank++) {
    ts.emplace_back([&, rank] {
      try {
        if (gpu) HIPOK(hipSetDevice(0));
        auto ctx = std::make_shared<gloo::rendezvous::Context>(rank, P, base);
        ctx->setTimeout(std::chrono::milliseconds(ms));
        if (P > 1) {
          gloo::transport::tcp::attr attr("localhost");
          auto dev = gloo::transport::tcp::CreateDevice(attr);
          ctx->connectFullMesh(store, dev);
        }
        fn(ctx);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(em);
        if (err.empty()) err = "rank " + std::to_string(rank) + ": " + e.what();
      }
      barrier.wait();
    });
  }
  for (auto& t : ts) t.join();
  return err;
}

template <typename T>
T fromDouble(double v) { return T(v); }
template <>
gloo::float16 fromDouble<gloo::float16>(double v) { return gloo::cpu_float2half_rn((float)v); }
template <typename T>
double toDouble(T v) { return (double)v; }
template <>
double toDouble<gloo::float16>(gloo::float16 v) { return gloo::cpu_half2float(v); }
#if GLOO_USE_TORCH_DTYPES
template <>
c10::BFloat16 fromDouble<c10::BFloat16>(double v) { return c10::BFloat16((float)v); }
template <>
double toDouble<c10::BFloat16>(c10::BFloat16 v) { return (double)(float)v; }
#endif

// How a case hands its inputs to the algorithm and reads its outputs.
enum class Inputs {
  kSync,       // hipMemcpy before run(), no streams
  kStreams,    // hipMemcpy before run(), one user stream per pointer
  kAsyncSpin,  // MultiPointerAsync (gloo/test/cuda_allreduce_test.cc:196-220,
               // gloo/test/cuda_base_test.h:60-75): per pointer, a spin
               // kernel then an async H2D copy of its input on ITS stream,
               // run() at once, then an async D2H copy of each output on its
               // stream before the streams are synchronised
};

using Make = std::function<std::unique_ptr<gloo::Algorithm>(std::shared_ptr<gloo::Context>&, std::vector<void*>&,
                                                            int, std::vector<hipStream_t>&)>;

// Fixture<T>::assignValues / checkAllreduceResult (gloo/test/base_test.h:184-236)
// on k device buffers per rank: element j of pointer i on rank r holds
// (j % mod) * P * k + r * k + i (mod 0: j), so the sum is known in closed form
// (mod keeps 16-bit sums exact).
template <typename T>
std::string allreduceCase(int P, int k, int count, Inputs inputs, int runs, const Make& make, int mod = 0,
                          int base = 2) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    const size_t stride = (size_t)P * k;
    std::vector<void*> ptrs(k);
    std::vector<hipStream_t> streams;
    // pinned, so the async copies are really asynchronous; inputs and
    // outputs apart (an input copy may still be queued behind its spin)
    std::vector<T*> host(k), out(k);
    auto jj = [&](int j) { return (size_t)(mod ? j % mod : j); };
    auto fill = [&](int i) {
      const size_t val = (size_t)ctx->rank * k + i;
      for (int j = 0; j < count; j++) host[i][j] = fromDouble<T>((double)(jj(j) * stride + val));
    };
    for (int i = 0; i < k; i++) {
      HIPOK(hipMalloc(&ptrs[i], std::max<size_t>(1, count * sizeof(T))));
      HIPOK(hipHostMalloc(reinterpret_cast<void**>(&host[i]), std::max<size_t>(1, count * sizeof(T)), 0));
      HIPOK(hipHostMalloc(reinterpret_cast<void**>(&out[i]), std::max<size_t>(1, count * sizeof(T)), 0));
      if (inputs != Inputs::kSync) {
        hipStream_t s;
        HIPOK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        streams.push_back(s);
      }
    }
    auto load = [&] {
      for (int i = 0; i < k; i++) {
        fill(i);
        if (inputs == Inputs::kAsyncSpin) {
          // 2 ms on the GPU clock ahead of the copy: without the stream
          // contract, run() would read stale inputs
          HIPOK((hipError_t)bt_spin(streams[i], 200000));
          HIPOK(hipMemcpyAsync(ptrs[i], host[i], count * sizeof(T), hipMemcpyHostToDevice, streams[i]));
        } else {
          HIPOK(hipMemcpy(ptrs[i], host[i], count * sizeof(T), hipMemcpyHostToDevice));
        }
      }
    };
    {
      auto a = make(ctx, ptrs, count, streams);
      for (int r = 0; r < runs; r++) {
        load();  // (re)set the inputs
        a->run();
        for (int i = 0; i < k; i++) {
          std::memset(out[i], 0xA5, count * sizeof(T));
          if (inputs == Inputs::kAsyncSpin)  // ordered after the collective on ITS stream
            HIPOK(hipMemcpyAsync(out[i], ptrs[i], count * sizeof(T), hipMemcpyDeviceToHost, streams[i]));
        }
        for (auto s : streams) HIPOK(hipStreamSynchronize(s));
        for (int i = 0; i < k; i++) {
          if (inputs != Inputs::kAsyncSpin)
            HIPOK(hipMemcpy(out[i], ptrs[i], count * sizeof(T), hipMemcpyDeviceToHost));
          for (int j = 0; j < count; j++) {
            const double want = (double)jj(j) * stride * stride + stride * (stride - 1) / 2.0;
            if (toDouble<T>(fromDouble<T>(want)) != toDouble<T>(out[i][j]))
              throw std::runtime_error("mismatch in ptr " + std::to_string(i) + " element " + std::to_string(j) +
                                       " run " + std::to_string(r) + ": " + std::to_string(toDouble<T>(out[i][j])) +
                                       " != " + std::to_string(want));
          }
        }
      }
    }
    for (auto s : streams) HIPOK(hipStreamDestroy(s));
    for (void* p : ptrs) HIPOK(hipFree(p));
    for (T* h : host) HIPOK(hipHostFree(h));
    for (T* h : out) HIPOK(hipHostFree(h));
  }, true, base);
}

template <typename T>
Make ringChunked() {
  return [](std::shared_ptr<gloo::Context>& c, std::vector<void*>& p, int n, std::vector<hipStream_t>& s) {
    std::vector<T*> tp;
    for (void* x : p) tp.push_back(static_cast<T*>(x));
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceRingChunked<T>(c, tp, n, s));
  };
}
template <typename T>
Make ringChunkedHost() {
  return [](std::shared_ptr<gloo::Context>& c, std::vector<void*>& p, int n, std::vector<hipStream_t>& s) {
    std::vector<T*> tp;
    for (void* x : p) tp.push_back(static_cast<T*>(x));
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceRingChunked<T, gloo::HipHostWorkspace<T>>(c, tp, n, s));
  };
}
template <typename T>
Make ring() {
  return [](std::shared_ptr<gloo::Context>& c, std::vector<void*>& p, int n, std::vector<hipStream_t>& s) {
    std::vector<T*> tp;
    for (void* x : p) tp.push_back(static_cast<T*>(x));
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceRing<T>(c, tp, n, s));
  };
}
template <typename T>
Make halvingDoubling(bool pipelined) {
  return [pipelined](std::shared_ptr<gloo::Context>& c, std::vector<void*>& p, int n, std::vector<hipStream_t>& s) {
    std::vector<T*> tp;
    for (void* x : p) tp.push_back(static_cast<T*>(x));
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceHalvingDoubling<T>(c, tp, n, s, pipelined));
  };
}
template <typename T>
Make halvingDoublingPipelined() {  // gloo::CudaAllreduceHalvingDoublingPipelined's twin
  return [](std::shared_ptr<gloo::Context>& c, std::vector<void*>& p, int n, std::vector<hipStream_t>& s) {
    std::vector<T*> tp;
    for (void* x : p) tp.push_back(static_cast<T*>(x));
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceHalvingDoublingPipelined<T>(c, tp, n, s));
  };
}
template <typename T, typename W = gloo::HipDeviceWorkspace<T>>
Make bcube() {  // gloo::CudaAllreduceBcube's twin: groups of the context's base
  return [](std::shared_ptr<gloo::Context>& c, std::vector<void*>& p, int n, std::vector<hipStream_t>& s) {
    std::vector<T*> tp;
    for (void* x : p) tp.push_back(static_cast<T*>(x));
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceBcube<T, W>(c, tp, n, s));
  };
}

// ReductionType CUSTOM: a HipReductionFunction<int32_t> whose device function
// is bt_add_i32 (the library calls it for every chunk reduction).
gloo::HipReductionFunction<int32_t>& customAdd() {
  static auto* f = new gloo::HipReductionFunction<int32_t>(&bt_add_i32);
  return *f;
}
Make ringChunkedCustom() {
  return [](std::shared_ptr<gloo::Context>& c, std::vector<void*>& p, int n, std::vector<hipStream_t>& s) {
    std::vector<int32_t*> tp;
    for (void* x : p) tp.push_back(static_cast<int32_t*>(x));
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceRingChunked<int32_t>(c, tp, n, s, &customAdd()));
  };
}
Make halvingDoublingCustom() {
  return [](std::shared_ptr<gloo::Context>& c, std::vector<void*>& p, int n, std::vector<hipStream_t>& s) {
    std::vector<int32_t*> tp;
    for (void* x : p) tp.push_back(static_cast<int32_t*>(x));
    return std::unique_ptr<gloo::Algorithm>(
        new gloo::HipAllreduceHalvingDoubling<int32_t>(c, tp, n, s, false, &customAdd()));
  };
}
// The case must really run the device function.
std::string customCase(int P, int count, const Make& make) {
  const long before = bt_add_i32_calls();
  std::string e = allreduceCase<int32_t>(P, 1, count, Inputs::kSync, 2, make);
  if (e.empty() && bt_add_i32_calls() == before) e = "the custom device function was never called";
  return e;
}
// A CUSTOM ReductionFunction without a device function is refused.
std::string customHostOnlyCase() {
  return spawn(2, 10000, [&](std::shared_ptr<gloo::Context> ctx) {
    static const gloo::ReductionFunction<float> hostOnly(gloo::CUSTOM, &gloo::sum<float>);
    float* d = nullptr;
    HIPOK(hipMalloc(&d, 1024 * sizeof(float)));
    bool refused = false;
    try {
      gloo::HipAllreduceRingChunked<float> a(ctx, {d}, 1024, {}, &hostOnly);
    } catch (const gloo::EnforceNotMet& e) {
      refused = std::string(e.what()).find("device function") != std::string::npos;
    }
    HIPOK(hipFree(d));
    if (!refused) throw std::runtime_error("a host-only CUSTOM reduction was accepted");
  });
}

// ReduceScatterHalvingDoubling (gloo/test/reduce_scatter_test.cc:79-196):
// rank r's block [off_r, off_r + recvElems[r]) lands at the start of its buffer.
std::string reduceScatterCase(int P, int count) {
  std::vector<int> recv;
  for (int r = 0, rem = count, chunk = (count + P - 1) / P; r < P; r++) {
    recv.push_back(std::min(chunk, rem));
    rem = rem > chunk ? rem - chunk : 0;
  }
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    std::vector<float> host(count);
    for (int j = 0; j < count; j++) host[j] = (float)(j * P + ctx->rank);
    float* d = nullptr;
    HIPOK(hipMalloc(&d, count * sizeof(float)));
    HIPOK(hipMemcpy(d, host.data(), count * sizeof(float), hipMemcpyHostToDevice));
    {
      gloo::HipReduceScatterHalvingDoubling<float> a(ctx, {d}, count, recv);
      a.run();
    }
    HIPOK(hipMemcpy(host.data(), d, count * sizeof(float), hipMemcpyDeviceToHost));
    int off = 0;
    for (int r = 0; r < ctx->rank; r++) off += recv[r];
    for (int j = 0; j < recv[ctx->rank]; j++) {
      const double want = (double)(off + j) * P * P + P * (P - 1) / 2.0;
      if (want != (double)host[j])
        throw std::runtime_error("reduce-scatter mismatch at " + std::to_string(j));
    }
    HIPOK(hipFree(d));
  });
}

// A peer that never runs: run() must raise gloo::IoException after the
// context timeout (gloo/common/error.h:42-48), and tear-down still completes.
std::string silentPeerCase() {
  std::string seen;
  std::mutex m;
  std::string err = spawn(2, 2000, [&](std::shared_ptr<gloo::Context> ctx) {
    float* d = nullptr;
    HIPOK(hipMalloc(&d, 4096 * sizeof(float)));
    {
      gloo::HipAllreduceRingChunked<float> a(ctx, {d}, 4096);
      if (ctx->rank == 0) {
        try {
          a.run();
        } catch (const gloo::IoException& e) {
          std::lock_guard<std::mutex> lk(m);
          seen = e.what();
        }
      }
    }
    HIPOK(hipFree(d));
  });
  if (!err.empty()) return err;
  return seen.empty() ? std::string("no IoException from a silent peer") : std::string();
}

// CPU only (no HIP call): the library context bootstrapped over the
// gloo::Context's all-gather, created and destroyed twice per rank.
std::string bootstrapCase(int P) {
  return spawn(P, 10000, [&](std::shared_ptr<gloo::Context> ctx) {
    for (int i = 0; i < 2; i++) gloo::hip_bridge::BootstrapContext b(ctx, 0);
  }, false);
}

}  // namespace

int main(int argc, char** argv) {
  const std::string filter = argc > 1 ? argv[1] : "";
  struct Case {
    std::string name;
    std::function<std::string()> fn;
  };
  std::vector<Case> cases;
  for (int P : {1, 2, 3, 5})
    cases.push_back({"bootstrap_cpu/P" + std::to_string(P), [=] { return bootstrapCase(P); }});
  for (int P : {1, 2, 3, 4, 5}) {
    for (int n : {1, 1000, 100003}) {
      cases.push_back({"ring_chunked/P" + std::to_string(P) + "/n" + std::to_string(n),
                       [=] { return allreduceCase<float>(P, 1, n, Inputs::kSync, 2, ringChunked<float>()); }});
      cases.push_back({"halving_doubling/P" + std::to_string(P) + "/n" + std::to_string(n),
                       [=] { return allreduceCase<float>(P, 1, n, Inputs::kSync, 2, halvingDoubling<float>(false)); }});
    }
    cases.push_back({"ring/P" + std::to_string(P) + "/n1000",
                     [=] { return allreduceCase<float>(P, 1, 1000, Inputs::kSync, 1, ring<float>()); }});
  }
  cases.push_back({"halving_doubling_pipelined/P4/n4099",
                   [] { return allreduceCase<float>(4, 1, 4099, Inputs::kSync, 1, halvingDoubling<float>(true)); }});
  cases.push_back({"halving_doubling_pipelined_class/P4/k2/n4099",
                   [] { return allreduceCase<float>(4, 2, 4099, Inputs::kSync, 2, halvingDoublingPipelined<float>()); }});
  // CudaAllreduceBcube (gloo/test/cuda_allreduce_test.cc:311-339: P = base^k)
  for (auto pb : {std::make_pair(2, 2), std::make_pair(4, 2), std::make_pair(8, 2), std::make_pair(3, 3),
                  std::make_pair(9, 3), std::make_pair(4, 4), std::make_pair(16, 4)}) {
    for (int n : {1, 64, 1000}) {
      const int P = pb.first, base = pb.second;
      cases.push_back({"bcube/P" + std::to_string(P) + "/b" + std::to_string(base) + "/n" + std::to_string(n),
                       [=] { return allreduceCase<float>(P, 1, n, Inputs::kSync, 2, bcube<float>(), 0, base); }});
    }
  }
  cases.push_back({"host_workspace/bcube/P4/b2/n10007",  // CudaAllreduceBcube's default workspace is the host's
                   [] { return allreduceCase<float>(4, 1, 10007, Inputs::kSync, 2,
                                                    bcube<float, gloo::HipHostWorkspace<float>>(), 0, 2); }});
  cases.push_back({"multi_pointer_async/bcube/P4/k2/n4099",
                   [] { return allreduceCase<float>(4, 2, 4099, Inputs::kAsyncSpin, 2, bcube<float>(), 0, 2); }});
  cases.push_back({"multi_pointer/ring_chunked/P3/k2/n1000",
                   [] { return allreduceCase<float>(3, 2, 1000, Inputs::kSync, 1, ringChunked<float>()); }});
  cases.push_back({"multi_pointer_streams/ring_chunked/P2/k2/n10007",
                   [] { return allreduceCase<float>(2, 2, 10007, Inputs::kStreams, 3, ringChunked<float>()); }});
  cases.push_back({"multi_pointer_streams/halving_doubling/P4/k2/n1000",
                   [] { return allreduceCase<float>(4, 2, 1000, Inputs::kStreams, 2, halvingDoubling<float>(false)); }});
  // MultiPointerAsync proper: spin + async input copies on each pointer's stream
  for (int k : {2, 3}) {
    const std::string ks = "/k" + std::to_string(k);
    cases.push_back({"multi_pointer_async/ring_chunked/P2" + ks + "/n100003",
                     [=] { return allreduceCase<float>(2, k, 100003, Inputs::kAsyncSpin, 3, ringChunked<float>()); }});
    cases.push_back({"multi_pointer_async/ring/P3" + ks + "/n1000",
                     [=] { return allreduceCase<float>(3, k, 1000, Inputs::kAsyncSpin, 2, ring<float>()); }});
    cases.push_back({"multi_pointer_async/halving_doubling/P4" + ks + "/n4099",
                     [=] { return allreduceCase<float>(4, k, 4099, Inputs::kAsyncSpin, 2, halvingDoubling<float>(false)); }});
  }
  cases.push_back({"multi_pointer_async/ring_chunked/P1/k2/n1000",  // local only: no transport at all
                   [] { return allreduceCase<float>(1, 2, 1000, Inputs::kAsyncSpin, 2, ringChunked<float>()); }});
  cases.push_back({"single_pointer_async/ring_chunked/P3/k1/n100003",
                   [] { return allreduceCase<float>(3, 1, 100003, Inputs::kAsyncSpin, 2, ringChunked<float>()); }});
  cases.push_back({"half/ring_chunked/P4/n128",  // cuda_allreduce_test.cc HalfPrecision shape
                   [] { return allreduceCase<gloo::float16>(4, 1, 128, Inputs::kSync, 1, ringChunked<gloo::float16>()); }});
  cases.push_back({"half/halving_doubling/P4/n128",
                   [] { return allreduceCase<gloo::float16>(4, 1, 128, Inputs::kSync, 1, halvingDoubling<gloo::float16>(false)); }});
#if GLOO_USE_TORCH_DTYPES
  // c10::BFloat16 (gloo/cuda.cu:394-401); inputs mod 16 keep every sum exact in bf16
  cases.push_back({"bf16/ring_chunked/P4/n4099",
                   [] { return allreduceCase<c10::BFloat16>(4, 1, 4099, Inputs::kSync, 2, ringChunked<c10::BFloat16>(), 16); }});
  cases.push_back({"bf16/halving_doubling/P3/n1000",
                   [] { return allreduceCase<c10::BFloat16>(3, 1, 1000, Inputs::kSync, 2, halvingDoubling<c10::BFloat16>(false), 16); }});
  cases.push_back({"bf16/ring/P2/k2/n777",
                   [] { return allreduceCase<c10::BFloat16>(2, 2, 777, Inputs::kAsyncSpin, 2, ring<c10::BFloat16>(), 16); }});
#endif
  cases.push_back({"custom/ring_chunked/P3/n1000", [] { return customCase(3, 1000, ringChunkedCustom()); }});
  cases.push_back({"custom/halving_doubling/P4/n4099", [] { return customCase(4, 4099, halvingDoublingCustom()); }});
  cases.push_back({"custom/host_only_refused", [] { return customHostOnlyCase(); }});
  cases.push_back({"host_workspace/ring_chunked/P3/n10007",
                   [] { return allreduceCase<float>(3, 1, 10007, Inputs::kSync, 2, ringChunkedHost<float>()); }});
  cases.push_back({"reduce_scatter/P4/n1000", [] { return reduceScatterCase(4, 1000); }});
  cases.push_back({"reduce_scatter/P5/n10007", [] { return reduceScatterCase(5, 10007); }});
  cases.push_back({"io_exception/silent_peer", [] { return silentPeerCase(); }});
  int failed = 0, ran = 0;
  for (auto& c : cases) {
    if (!filter.empty() && c.name.find(filter) == std::string::npos) continue;
    ran++;
    std::string e;
    try {
      e = c.fn();
    } catch (const std::exception& ex) {
      e = ex.what();
    }
    std::printf("%s %s%s%s\n", e.empty() ? "ok  " : "FAIL", c.name.c_str(), e.empty() ? "" : ": ", e.c_str());
    std::fflush(stdout);
    failed += !e.empty();
  }
  std::printf("%d cases, %d failed\n", ran, failed);
  return failed ? 1 : 0;
}

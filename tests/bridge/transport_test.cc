// transport_test.cc — TEST PROGRAM (built by oracle/Makefile where the reference
// sources exist; the binary travels to the GPU box, the reference does not).
//
// The xGMI transport as a gloo::transport::Device
// (gloo_amd/include/gloo_amd/gloo_transport.h) inside a Gloo program built
// against the reference's own headers and objects:
//   connect/P*            gloo::rendezvous::Context::connectFullMesh(store,
//                         hip::CreateDevice(...)) (gloo/rendezvous/context.cc:25-35);
//   device_ring_chunked   a gloo::Algorithm on device memory in the shape of
//                         CudaAllreduceRingChunked<T, CudaDeviceWorkspace<T>>:
//                         device inboxes as receive buffers on getLeftPair()
//                         (gloo/cuda_allreduce_ring_chunked.cc:333-352), the
//                         reference's ring-chunked schedule
//                         (gloo/allreduce_ring_chunked.h:83-212), per-chunk HIP
//                         reduction + stream wait (.cc:185-190);
//   bridge_*              gloo::HipAllreduce* (gloo_bridge.h) on a context
//                         whose pairs are this transport;
//   ref_*_host            the reference's own AllreduceRingChunked /
//                         AllreduceHalvingDoubling templates, unmodified, on
//                         host buffers over this transport (thread ranks);
//   context_factory       the reference's rendezvous::ContextFactory
//                         (gloo/rendezvous/context.cc:37-162) bootstrapping a
//                         TCP context over this transport's bound buffers;
//   io_exception          a receive that never arrives raises gloo::IoException;
//   unbound_refused       createUnboundBuffer raises InvalidOperationException.
// Expected values: the closed form of gloo/test/base_test.h:184-236.
//
// Usage: transport_test [case-filter]             ranks as threads (exit 0 = ok)
//        transport_test proc RANK P STORE_DIR N   one rank of device_ring_chunked
//                                                 as a process (gloo::rendezvous::FileStore;
//                                                 receive buffers over HIP IPC)
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "gloo/allreduce_halving_doubling.h"
#include "gloo/allreduce_ring_chunked.h"
#include "gloo/rendezvous/context.h"
#include "gloo/rendezvous/file_store.h"
#include "gloo/rendezvous/hash_store.h"
#include "gloo/transport/tcp/device.h"
#include "gloo_amd/gloo_bridge.h"
#include "gloo_amd/gloo_transport.h"

namespace {

#define HIPOK(x)                                                                                    \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
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

std::shared_ptr<gloo::rendezvous::Context> connectHip(int rank, int P, int ms,
                                                      std::shared_ptr<gloo::rendezvous::Store> store) {
  HIPOK(hipSetDevice(0));
  auto ctx = std::make_shared<gloo::rendezvous::Context>(rank, P);
  ctx->setTimeout(std::chrono::milliseconds(ms));
  gloo::transport::hip::attr a;
  a.device = 0;
  auto dev = gloo::transport::hip::CreateDevice(a);
  ctx->connectFullMesh(store, dev);
  return ctx;
}

// P ranks as threads, each with a gloo::Context on the hip transport.
std::string spawn(int P, int ms, const std::function<void(std::shared_ptr<gloo::Context>)>& fn) {
  auto store = std::make_shared<gloo::rendezvous::HashStore>();
  Barrier barrier(P);
  std::vector<std::thread> ts;
  std::mutex em;
  std::string err;
  for (int rank = 0; rank < P; rank++) {
    ts.emplace_back([&, rank] {
      try {
        auto ctx = connectHip(rank, P, ms, store);
        fn(ctx);
        barrier.wait();  // the context (and its pairs) outlive every peer's use
      } catch (const std::exception& e) {
        {
          std::lock_guard<std::mutex> lk(em);
          if (err.empty()) err = "rank " + std::to_string(rank) + ": " + e.what();
        }
        barrier.wait();
      }
    });
  }
  for (auto& t : ts) t.join();
  return err;
}

// CudaAllreduceRingChunked<T, CudaDeviceWorkspace<T>> on one device pointer:
// the reference's ring-chunked schedule, device inboxes registered as receive
// buffers on the left pair, each chunk reduced by the HIP kernel.
template <typename T>
class DeviceRingChunked : public gloo::Algorithm {
 public:
  DeviceRingChunked(const std::shared_ptr<gloo::Context>& context, T* ptr, int count)
      : gloo::Algorithm(context), ptr_(ptr), count_(count), bytes_((size_t)count * sizeof(T)) {
    constexpr size_t minSize = 256;  // gloo/cuda_allreduce_ring_chunked.cc:70-80
    chunks_ = contextSize_ * 2;
    chunkSize_ = std::max(minSize, (size_t)(count_ + chunks_ - 1) / chunks_);
    HIPOK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) HIPOK(hipMalloc(&inbox_[i], std::max<size_t>(chunkSize_ * sizeof(T), 1)));
    if (count_ == 0 || contextSize_ == 1) return;
    auto& leftPair = getLeftPair();
    auto& rightPair = getRightPair();
    for (int i = 0; i < 2; i++) {
      auto slot = context_->nextSlot();
      sendDataBuf_[i] = rightPair->createSendBuffer(slot, ptr_, bytes_);
      recvDataBuf_[i] = leftPair->createRecvBuffer(slot, inbox_[i], chunkSize_ * sizeof(T));
    }
    auto notificationSlot = context_->nextSlot();
    sendNotificationBuf_ = leftPair->createSendBuffer(notificationSlot, nullptr, 0);
    recvNotificationBuf_ = rightPair->createRecvBuffer(notificationSlot, nullptr, 0);
  }
  ~DeviceRingChunked() override {
    sendDataBuf_[0].reset();
    sendDataBuf_[1].reset();
    recvDataBuf_[0].reset();
    recvDataBuf_[1].reset();
    sendNotificationBuf_.reset();
    recvNotificationBuf_.reset();
    for (int i = 0; i < 2; i++) (void)hipFree(inbox_[i]);
    (void)hipStreamDestroy(stream_);
  }

  void run() override {
    if (count_ == 0 || contextSize_ == 1) return;
    copyChunkAtOffset(2 * contextRank_);
    copyChunkAtOffset(2 * contextRank_ + 1);
    for (int round = 2; round < chunks_; round++) {
      const int chunkOffset = ((2 * contextRank_) - (round & ~0x1) + (round & 0x1) + chunks_) % chunks_;
      size_t offset, length;
      range(chunkOffset, offset, length);
      recvDataBuf_[chunkOffset & 1]->waitRecv();
      if (length > 0) {
        check(gloo_hip_reduce(GLOO_HIP_SUM, gloo::hip_bridge::DType<T>::value, ptr_ + offset, inbox_[chunkOffset & 1],
                              length, stream_));
        HIPOK(hipStreamSynchronize(stream_));
      }
      sendNotificationBuf_->send();
      recvNotificationBuf_->waitRecv();
      copyChunkAtOffset(chunkOffset);
    }
    for (int round = 0; round < chunks_ - 2; round++) {
      const int chunkOffset = ((2 * contextRank_) - (round & ~0x1) + (round & 0x1) + chunks_) % chunks_;
      size_t offset, length;
      range(chunkOffset, offset, length);
      recvDataBuf_[chunkOffset & 1]->waitRecv();
      if (length > 0) {
        HIPOK(hipMemcpyAsync(ptr_ + offset, inbox_[chunkOffset & 1], length * sizeof(T), hipMemcpyDeviceToDevice,
                             stream_));
        HIPOK(hipStreamSynchronize(stream_));
      }
      if (round < chunks_ - 4) {
        sendNotificationBuf_->send();
        recvNotificationBuf_->waitRecv();
        copyChunkAtOffset(chunkOffset);
      }
    }
    sendNotificationBuf_->send();
    recvNotificationBuf_->waitRecv();
    for (int i = 0; i < 2; i++) sendDataBuf_[i]->waitSend();
  }

 private:
  static void check(int rc) {
    if (rc != GLOO_HIP_OK) throw std::runtime_error(std::string("gloo_hip_reduce: ") + gloo_hip_last_error());
  }
  void range(int chunkOffset, size_t& offset, size_t& length) const {
    offset = (size_t)chunkOffset * chunkSize_;
    length = chunkSize_;
    if (offset + length <= (size_t)count_) {
    } else if (offset < (size_t)count_) {
      length = count_ - offset;
    } else {
      length = 0;
    }
  }
  void copyChunkAtOffset(int chunkOffset) {
    size_t offset = (size_t)(chunkOffset % chunks_) * chunkSize_, length = chunkSize_;
    if (offset + length <= (size_t)count_) {
    } else if (offset < (size_t)count_) {
      length = count_ - offset;
    } else {
      offset = 0;  // gloo/allreduce_ring_chunked.h:224-231
      length = 1;
    }
    sendDataBuf_[chunkOffset & 1]->send(offset * sizeof(T), length * sizeof(T));
  }

  T* ptr_;
  const int count_;
  const size_t bytes_;
  int chunks_ = 0;
  size_t chunkSize_ = 0;
  T* inbox_[2] = {nullptr, nullptr};
  hipStream_t stream_ = nullptr;
  std::unique_ptr<gloo::transport::Buffer> sendDataBuf_[2], recvDataBuf_[2], sendNotificationBuf_,
      recvNotificationBuf_;
};

// Values j * P + rank (exact in fp32 below 2^24 / P); result j * P^2 + P(P-1)/2.
std::string checkClosedForm(const std::vector<float>& h, int P, int run) {
  for (size_t j = 0; j < h.size(); j++) {
    const double want = (double)(j % 4096) * P * P + P * (P - 1) / 2.0;
    if ((double)h[j] != want)
      return "run " + std::to_string(run) + " element " + std::to_string(j) + ": " + std::to_string(h[j]) +
             " != " + std::to_string(want);
  }
  return "";
}
void fill(std::vector<float>& h, int P, int rank) {
  for (size_t j = 0; j < h.size(); j++) h[j] = (float)((j % 4096) * P + rank);
}

// make(ctx, ptr, count) -> algorithm on one device pointer, run `runs` times.
using Make = std::function<std::unique_ptr<gloo::Algorithm>(std::shared_ptr<gloo::Context>&, float*, int)>;
void deviceRank(std::shared_ptr<gloo::Context> ctx, int count, int runs, const Make& make) {
  const int P = ctx->size;
  float* d = nullptr;
  HIPOK(hipMalloc(&d, std::max<size_t>(1, count * sizeof(float))));
  std::vector<float> h(count);
  {
    auto a = make(ctx, d, count);
    for (int r = 0; r < runs; r++) {
      fill(h, P, ctx->rank);
      HIPOK(hipMemcpy(d, h.data(), count * sizeof(float), hipMemcpyHostToDevice));
      a->run();
      HIPOK(hipMemcpy(h.data(), d, count * sizeof(float), hipMemcpyDeviceToHost));
      const std::string e = checkClosedForm(h, P, r);
      if (!e.empty()) throw std::runtime_error(e);
    }
  }
  HIPOK(hipFree(d));
}

Make deviceRingChunked() {
  return [](std::shared_ptr<gloo::Context>& c, float* p, int n) {
    return std::unique_ptr<gloo::Algorithm>(new DeviceRingChunked<float>(c, p, n));
  };
}
Make bridgeRingChunked() {
  return [](std::shared_ptr<gloo::Context>& c, float* p, int n) {
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceRingChunked<float>(c, {p}, n));
  };
}
Make bridgeHalvingDoubling() {
  return [](std::shared_ptr<gloo::Context>& c, float* p, int n) {
    return std::unique_ptr<gloo::Algorithm>(new gloo::HipAllreduceHalvingDoubling<float>(c, {p}, n));
  };
}

// The reference's own CPU templates, unmodified, over this transport.
template <typename A>
std::string refHostCase(int P, int count) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    std::vector<float> h(count);
    std::vector<float*> ptrs{h.data()};
    A a(ctx, ptrs, count);
    for (int r = 0; r < 2; r++) {
      fill(h, P, ctx->rank);
      a.run();
      const std::string e = checkClosedForm(h, P, r);
      if (!e.empty()) throw std::runtime_error(e);
    }
  });
}

std::string connectCase(int P) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    for (int i = 0; i < P; i++) {
      if (i == ctx->rank) continue;
      auto& pair = ctx->getPair(i);
      if (!pair || !pair->isConnected()) throw std::runtime_error("pair to " + std::to_string(i) + " not connected");
      if (pair->address().str().find("hip:") != 0) throw std::runtime_error("not a hip pair");
    }
  });
}

// rendezvous::ContextFactory over this transport's bound (host) buffers,
// then a reference ring-chunked allreduce on the TCP context it made.
std::string contextFactoryCase(int P) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    gloo::rendezvous::ContextFactory factory(ctx);
    gloo::transport::tcp::attr attr("localhost");
    auto tcp = gloo::transport::tcp::CreateDevice(attr);
    auto c2 = factory.makeContext(tcp);
    std::vector<float> h(1000);
    std::vector<float*> ptrs{h.data()};
    fill(h, P, c2->rank);
    gloo::AllreduceRingChunked<float> a(c2, ptrs, (int)h.size());
    a.run();
    const std::string e = checkClosedForm(h, P, 0);
    if (!e.empty()) throw std::runtime_error(e);
  });
}

std::string ioExceptionCase() {
  std::string seen;
  std::mutex m;
  std::string err = spawn(2, 1500, [&](std::shared_ptr<gloo::Context> ctx) {
    float* d = nullptr;
    HIPOK(hipMalloc(&d, 1024 * sizeof(float)));
    auto buf = ctx->getPair(1 - ctx->rank)->createRecvBuffer(ctx->nextSlot(), d, 1024 * sizeof(float));
    if (ctx->rank == 0) {
      try {
        buf->waitRecv();  // rank 1 never sends
      } catch (const gloo::IoException& e) {
        std::lock_guard<std::mutex> lk(m);
        seen = e.what();
      }
    }
    buf.reset();
    HIPOK(hipFree(d));
  });
  if (!err.empty()) return err;
  return seen.empty() ? std::string("no IoException") : std::string();
}

std::string unboundRefusedCase() {
  bool refused = false;
  std::string err = spawn(2, 10000, [&](std::shared_ptr<gloo::Context> ctx) {
    char x[8];
    try {
      (void)ctx->createUnboundBuffer(x, sizeof(x));
    } catch (const gloo::InvalidOperationException&) {
      if (ctx->rank == 0) refused = true;
    }
  });
  if (!err.empty()) return err;
  return refused ? std::string() : std::string("createUnboundBuffer did not raise InvalidOperationException");
}

int procMain(int rank, int P, const std::string& dir, int count) {
  try {
    auto store = std::make_shared<gloo::rendezvous::FileStore>(dir);
    auto ctx = connectHip(rank, P, 60000, store);
    deviceRank(ctx, count, 2, deviceRingChunked());
    deviceRank(ctx, count, 1, bridgeRingChunked());
    // every rank finishes with the pairs before any tears down
    std::vector<char> done{1};
    store->set("done/" + std::to_string(rank), done);
    for (int r = 0; r < P; r++) store->wait({"done/" + std::to_string(r)}, std::chrono::seconds(60));
  } catch (const std::exception& e) {
    std::printf("FAIL rank %d: %s\n", rank, e.what());
    return 1;
  }
  std::printf("ok   proc rank %d\n", rank);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "proc") {
    if (argc < 6) return 2;
    return procMain(std::atoi(argv[2]), std::atoi(argv[3]), argv[4], std::atoi(argv[5]));
  }
  const std::string filter = argc > 1 ? argv[1] : "";
  struct Case {
    std::string name;
    std::function<std::string()> fn;
  };
  std::vector<Case> cases;
  for (int P : {2, 3, 5}) cases.push_back({"connect/P" + std::to_string(P), [=] { return connectCase(P); }});
  for (int P : {2, 3, 4, 5})
    for (int n : {1, 1000, 100003, 1 << 22})
      cases.push_back({"device_ring_chunked/P" + std::to_string(P) + "/n" + std::to_string(n), [=] {
                         return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> c) {
                           deviceRank(c, n, 2, deviceRingChunked());
                         });
                       }});
  for (int P : {2, 3, 4}) {
    cases.push_back({"bridge_ring_chunked/P" + std::to_string(P) + "/n100003", [=] {
                       return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> c) {
                         deviceRank(c, 100003, 2, bridgeRingChunked());
                       });
                     }});
    cases.push_back({"bridge_halving_doubling/P" + std::to_string(P) + "/n100003", [=] {
                       return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> c) {
                         deviceRank(c, 100003, 2, bridgeHalvingDoubling());
                       });
                     }});
  }
  for (int P : {2, 3, 4}) {
    cases.push_back({"ref_ring_chunked_host/P" + std::to_string(P) + "/n10007",
                     [=] { return refHostCase<gloo::AllreduceRingChunked<float>>(P, 10007); }});
    cases.push_back({"ref_halving_doubling_host/P" + std::to_string(P) + "/n10007",
                     [=] { return refHostCase<gloo::AllreduceHalvingDoubling<float>>(P, 10007); }});
  }
  cases.push_back({"context_factory/P3", [] { return contextFactoryCase(3); }});
  cases.push_back({"io_exception/silent_peer", [] { return ioExceptionCase(); }});
  cases.push_back({"unbound_refused", [] { return unboundRefusedCase(); }});
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

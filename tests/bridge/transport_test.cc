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
//   many_live             four DeviceRingChunked instances live at once on one
//                         context (12 slots per pair) run interleaved;
//   ref_allreduce_*, ref_allgather, ref_reduce
//                         the reference's own gloo::allreduce (RING, BCUBE),
//                         gloo::allgather and gloo::reduce, unmodified, on host
//                         buffers over this transport's unbound buffers;
//   unbound_*             recv-from-any, abort, device buffers, ordering.
// DeviceRingChunked's notification buffers are the reference's own host
// words (&dummy_, sizeof(dummy_), gloo/cuda_allreduce_ring_chunked.cc:119-123),
// also with ranks as processes (their bytes travel in the channel's payload).
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

#include "gloo/allgather.h"
#include "gloo/allreduce.h"
#include "gloo/allreduce_halving_doubling.h"
#include "gloo/allreduce_ring_chunked.h"
#include "gloo/math.h"
#include "gloo/reduce.h"
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
    // host words, as the reference does (gloo/cuda_allreduce_ring_chunked.cc:119-123)
    auto notificationSlot = context_->nextSlot();
    sendNotificationBuf_ = leftPair->createSendBuffer(notificationSlot, &dummy_, sizeof(dummy_));
    recvNotificationBuf_ = rightPair->createRecvBuffer(notificationSlot, &dummy_, sizeof(dummy_));
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
  int dummy_ = 0;
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

// One rank of a reference host-memory allreduce template, two runs, against
// the closed form.
template <typename A>
void refHostRank(std::shared_ptr<gloo::Context> ctx, int count, int P, const char* name) {
  std::vector<float> h(count);
  std::vector<float*> ptrs{h.data()};
  A a(ctx, ptrs, count);
  for (int r = 0; r < 2; r++) {
    fill(h, P, ctx->rank);
    a.run();
    const std::string e = checkClosedForm(h, P, r);
    if (!e.empty()) throw std::runtime_error(std::string(name) + " over processes: " + e);
  }
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

// Four DeviceRingChunked instances live on one context (3 slots each per
// pair, 12 in all), run interleaved: every slot needs its own channel.
std::string manyLiveCase(int P, int count) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    constexpr int kLive = 4;
    std::vector<float*> d(kLive, nullptr);
    std::vector<std::unique_ptr<gloo::Algorithm>> algos;
    for (int k = 0; k < kLive; k++) {
      HIPOK(hipMalloc(&d[k], count * sizeof(float)));
      algos.emplace_back(new DeviceRingChunked<float>(ctx, d[k], count));
    }
    std::vector<float> h(count);
    for (int r = 0; r < 2; r++)
      for (int k = 0; k < kLive; k++) {
        fill(h, P, ctx->rank);
        HIPOK(hipMemcpy(d[k], h.data(), count * sizeof(float), hipMemcpyHostToDevice));
        algos[k]->run();
        HIPOK(hipMemcpy(h.data(), d[k], count * sizeof(float), hipMemcpyDeviceToHost));
        const std::string e = checkClosedForm(h, P, r);
        if (!e.empty()) throw std::runtime_error("instance " + std::to_string(k) + ": " + e);
      }
    algos.clear();
    for (float* p : d) HIPOK(hipFree(p));
  });
}

using ReduceFn = void (*)(void*, const void*, const void*, size_t);

// The reference's gloo::allreduce(opts) (RING / BCUBE), unmodified, on host
// buffers over this transport's unbound buffers: two inputs per rank,
// segments of 4 KiB so the ring has many.
std::string refAllreduceCase(int P, int count, bool bcube) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    std::vector<float> a(count), b(count), out(count);
    for (int r = 0; r < 2; r++) {
      for (int j = 0; j < count; j++) {
        a[j] = (float)((j % 4096) * P + ctx->rank);
        b[j] = (float)(j % 7);
      }
      gloo::AllreduceOptions opts(ctx);
      opts.setAlgorithm(bcube ? gloo::AllreduceOptions::Algorithm::BCUBE : gloo::AllreduceOptions::Algorithm::RING);
      opts.setInputs(std::vector<float*>{a.data(), b.data()}, count);
      opts.setOutput(out.data(), count);
      opts.setReduceFunction(static_cast<ReduceFn>(&gloo::sum<float>));
      opts.setMaxSegmentSize(4096);
      opts.setTag(r);
      gloo::allreduce(opts);
      for (int j = 0; j < count; j++) {
        const double want = (double)(j % 4096) * P * P + P * (P - 1) / 2.0 + (double)P * (j % 7);
        if ((double)out[j] != want)
          throw std::runtime_error("element " + std::to_string(j) + ": " + std::to_string(out[j]) + " != " +
                                   std::to_string(want));
      }
    }
  });
}

// gloo::allgather (gloo/allgather.cc), unmodified, over this transport.
std::string refAllgatherCase(int P, int count) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    std::vector<int64_t> in(count), out((size_t)count * P);
    for (int j = 0; j < count; j++) in[j] = (int64_t)ctx->rank * 1000003 + j;
    gloo::AllgatherOptions opts(ctx);
    opts.setInput(in.data(), count);
    opts.setOutput(out.data(), (size_t)count * P);
    gloo::allgather(opts);
    for (int r = 0; r < P; r++)
      for (int j = 0; j < count; j++)
        if (out[(size_t)r * count + j] != (int64_t)r * 1000003 + j)
          throw std::runtime_error("allgather mismatch at rank block " + std::to_string(r));
  });
}

// gloo::reduce (gloo/reduce.cc), unmodified, over this transport.
std::string refReduceCase(int P, int count, int root) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    std::vector<double> in(count), out(count);
    for (int j = 0; j < count; j++) in[j] = (double)(j * P + ctx->rank);
    gloo::ReduceOptions opts(ctx);
    opts.setInput(in.data(), count);
    opts.setOutput(out.data(), count);
    opts.setRoot(root);
    opts.setReduceFunction(static_cast<ReduceFn>(&gloo::sum<double>));
    opts.setMaxSegmentSize(1024);
    gloo::reduce(opts);
    if (ctx->rank == root)
      for (int j = 0; j < count; j++)
        if (out[j] != (double)j * P * P + P * (P - 1) / 2.0)
          throw std::runtime_error("reduce mismatch at " + std::to_string(j));
  });
}

// Recv-from-any: rank 0 takes one message from each of ranks 1..P-1 on one
// slot, in whatever order they arrive, and learns who sent which.
std::string unboundRecvFromAnyCase(int P) {
  return spawn(P, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    const uint64_t slot = gloo::Slot::build(3, 0);
    if (ctx->rank == 0) {
      std::vector<int> got((size_t)P, -1);
      std::vector<int> srcs;
      for (int r = 1; r < P; r++) srcs.push_back(r);
      for (int k = 1; k < P; k++) {
        int v = -1, src = -1;
        auto buf = ctx->createUnboundBuffer(&v, sizeof(v));
        buf->recv(srcs, slot);
        if (!buf->waitRecv(&src)) throw std::runtime_error("recv aborted");
        if (src < 1 || src >= P || got[src] != -1 || v != 100 + src) throw std::runtime_error("bad message");
        got[src] = v;
      }
    } else {
      int v = 100 + ctx->rank;
      auto buf = ctx->createUnboundBuffer(&v, sizeof(v));
      buf->send(0, slot);
      int dst = -1;
      if (!buf->waitSend(&dst) || dst != 0) throw std::runtime_error("send not completed");
    }
  });
}

// Ordering per (source, slot), 0-byte messages, and device buffers.
std::string unboundOrderDeviceCase() {
  return spawn(2, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    const uint64_t slot = gloo::Slot::build(4, 1);
    constexpr int kMsgs = 200;  // more than the queue holds: the sender waits for the receiver
    float* d = nullptr;
    HIPOK(hipMalloc(&d, 1024 * sizeof(float)));
    auto buf = ctx->createUnboundBuffer(d, 1024 * sizeof(float));
    std::vector<float> h(1024);
    if (ctx->rank == 1) {
      for (int m = 0; m < kMsgs; m++) {
        for (int j = 0; j < 1024; j++) h[j] = (float)(m * 1024 + j);
        HIPOK(hipMemcpy(d, h.data(), sizeof(float) * 1024, hipMemcpyHostToDevice));
        buf->send(0, slot, 0, m % 5 == 4 ? 0 : 1024 * sizeof(float));
        buf->waitSend();
      }
    } else {
      for (int m = 0; m < kMsgs; m++) {
        const size_t n = m % 5 == 4 ? 0 : 1024 * sizeof(float);
        buf->recv(1, slot, 0, n);
        int src = -1;
        if (!buf->waitRecv(&src) || src != 1) throw std::runtime_error("recv failed");
        if (!n) continue;
        HIPOK(hipMemcpy(h.data(), d, sizeof(float) * 1024, hipMemcpyDeviceToHost));
        for (int j = 0; j < 1024; j++)
          if (h[j] != (float)(m * 1024 + j)) throw std::runtime_error("message " + std::to_string(m) + " out of order");
      }
    }
    buf.reset();
    HIPOK(hipFree(d));
  });
}

// abortWaitRecv from another thread ends a wait that would never complete.
std::string unboundAbortCase() {
  return spawn(2, 30000, [&](std::shared_ptr<gloo::Context> ctx) {
    if (ctx->rank != 0) return;
    int v = 0;
    auto buf = ctx->createUnboundBuffer(&v, sizeof(v));
    buf->recv(1, gloo::Slot::build(5, 0));
    std::thread t([&] {
      std::this_thread::sleep_for(std::chrono::milliseconds(200));
      buf->abortWaitRecv();
    });
    const bool done = buf->waitRecv();
    t.join();
    if (done) throw std::runtime_error("aborted wait reported completion");
  });
}

int procMain(int rank, int P, const std::string& dir, int count) {
  try {
    auto store = std::make_shared<gloo::rendezvous::FileStore>(dir);
    auto ctx = connectHip(rank, P, 60000, store);
    deviceRank(ctx, count, 2, deviceRingChunked());
    deviceRank(ctx, count, 1, bridgeRingChunked());
    // the reference's own host-memory templates between processes: their
    // inboxes are malloc'ed host buffers of chunkBytes_ registered as receive
    // buffers (gloo/allreduce_ring_chunked.h:44-46,60-61), so every data
    // message crosses through the receiver's landing segment
    refHostRank<gloo::AllreduceRingChunked<float>>(ctx, count, P, "AllreduceRingChunked<float>");
    refHostRank<gloo::AllreduceHalvingDoubling<float>>(ctx, count, P, "AllreduceHalvingDoubling<float>");
    // the reference's own gloo::allreduce on host buffers between processes
    // (unbound buffers staged in node shared memory)
    {
      std::vector<float> a(4099), out(4099);
      for (int j = 0; j < 4099; j++) a[j] = (float)(j * P + rank);
      gloo::AllreduceOptions opts(ctx);
      opts.setInput(a.data(), a.size());
      opts.setOutput(out.data(), out.size());
      opts.setReduceFunction(static_cast<void (*)(void*, const void*, const void*, size_t)>(&gloo::sum<float>));
      opts.setMaxSegmentSize(1024);
      gloo::allreduce(opts);
      for (int j = 0; j < 4099; j++)
        if ((double)out[j] != (double)j * P * P + P * (P - 1) / 2.0)
          throw std::runtime_error("gloo::allreduce over processes: element " + std::to_string(j));
    }
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
  cases.push_back({"many_live/P2/n10007", [] { return manyLiveCase(2, 10007); }});
  cases.push_back({"many_live/P3/n1000", [] { return manyLiveCase(3, 1000); }});
  for (int P : {2, 3, 4, 5}) {
    cases.push_back({"ref_allreduce_ring_host/P" + std::to_string(P) + "/n10007",
                     [=] { return refAllreduceCase(P, 10007, false); }});
    cases.push_back({"ref_allreduce_bcube_host/P" + std::to_string(P) + "/n10007",
                     [=] { return refAllreduceCase(P, 10007, true); }});
  }
  cases.push_back({"ref_allgather_host/P4/n777", [] { return refAllgatherCase(4, 777); }});
  cases.push_back({"ref_reduce_host/P5/n3001", [] { return refReduceCase(5, 3001, 3); }});
  cases.push_back({"unbound_recv_from_any/P4", [] { return unboundRecvFromAnyCase(4); }});
  cases.push_back({"unbound_order_device/P2", [] { return unboundOrderDeviceCase(); }});
  cases.push_back({"unbound_abort/P2", [] { return unboundAbortCase(); }});
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

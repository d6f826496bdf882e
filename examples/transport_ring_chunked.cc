// transport_ring_chunked.cc — a Gloo algorithm written against the
// transport interface, running over the xGMI transport
// (gloo_amd/include/gloo_amd/transport.h).
//
// RingChunked<T>::run() below is the schedule of gloo::AllreduceRingChunked
// (gloo/allreduce_ring_chunked.h:83-212) statement for statement: the same
// chunk geometry, the same double-buffered inboxes, send / waitRecv /
// notification handshake on transport::Pair / Buffer objects created with
// the same slots.  What differs is where the bytes live and who reduces
// them: ptrs and inboxes are device memory, Buffer::send is a device copy
// into the peer's inbox, and the per-chunk reduction is the HIP kernel
// (HipReductionFunction<T>::call, then a stream wait, as
// gloo/cuda_allreduce_ring_chunked.cc:185-190 does).
//
// Usage: transport_ring_chunked P count runs     (ranks as threads on GPU 0)
// Checks every element against a closed form (gloo/test/base_test.h:184-236
// with values kept below 2^24 so fp32 sums are exact); prints "ok".
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "gloo_amd/hip_allreduce.h"
#include "gloo_amd/store.h"
#include "gloo_amd/transport.h"

using gloo_amd::transport::Buffer;
using gloo_amd::transport::Device;

#define CHECK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static bool g_trace = std::getenv("TRANSPORT_TRACE") != nullptr;

template <typename T>
float firstValue(const T* p) {
  T v;
  if (hipMemcpy(&v, p, sizeof(T), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (float)v;
}

template <typename T>
class RingChunked {
 public:
  RingChunked(Device& dev, std::vector<T*> ptrs, int count, int& nextSlot)
      : dev_(dev), rank_(dev.context()->rank), size_(dev.context()->size), ptrs_(std::move(ptrs)),
        count_(count), bytes_(count_ * sizeof(T)), fn_(gloo_amd::HipReductionFunction<T>::sum) {
    constexpr size_t minSize = 256;
    chunks_ = size_ * 2;
    chunkSize_ = std::max(minSize, (size_t)(count_ + chunks_ - 1) / chunks_);
    chunkBytes_ = chunkSize_ * sizeof(T);
    for (int i = 0; i < 2; i++) CHECK(hipMalloc(&inbox_[i], std::max<size_t>(bytes_, 1)));
    CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    if (count_ == 0 || size_ == 1) return;
    auto& leftPair = dev.getPair((size_ + rank_ - 1) % size_);
    auto& rightPair = dev.getPair((rank_ + 1) % size_);
    for (int i = 0; i < 2; i++) {
      auto slot = nextSlot++;
      sendDataBuf_[i] = rightPair.createSendBuffer(slot, ptrs_[0], bytes_);
      recvDataBuf_[i] = leftPair.createRecvBuffer(slot, inbox_[i], chunkBytes_);
    }
    auto notificationSlot = nextSlot++;
    sendNotificationBuf_ = leftPair.createSendBuffer(notificationSlot, nullptr, 0);
    recvNotificationBuf_ = rightPair.createRecvBuffer(notificationSlot, nullptr, 0);
  }
  ~RingChunked() {
    sendDataBuf_[0].reset();
    sendDataBuf_[1].reset();
    sendNotificationBuf_.reset();
    for (int i = 0; i < 2; i++) (void)hipFree(inbox_[i]);
    (void)hipStreamDestroy(stream_);
  }

  void run() {
    if (count_ == 0) return;
    for (size_t i = 1; i < ptrs_.size(); i++) reduce(ptrs_[0], ptrs_[i], count_);
    if (size_ == 1) {
      for (size_t i = 1; i < ptrs_.size(); i++) copy(ptrs_[i], ptrs_[0], bytes_);
      return;
    }
    copyChunkAtOffset(2 * rank_);
    copyChunkAtOffset(2 * rank_ + 1);
    for (int round = 2; round < chunks_; round++) {
      auto chunkOffset = ((2 * rank_) - (round & ~0x1) + (round & 0x1) + chunks_) % chunks_;
      size_t offset = chunkOffset * chunkSize_, length = chunkSize_;
      if (offset + length <= (size_t)count_) {
      } else if (offset < (size_t)count_) {
        length = count_ - offset;
      } else {
        length = 0;
      }
      recvDataBuf_[chunkOffset & 1]->waitRecv();
      if (g_trace)
        std::fprintf(stderr, "r%d pass1 round %d chunk %d off %zu len %zu inbox %g mine %g\n", rank_, round,
                     (int)chunkOffset, offset, length, length ? firstValue(inbox_[chunkOffset & 1]) : 0.f,
                     length ? firstValue(&ptrs_[0][offset]) : 0.f);
      if (length > 0) reduce(&ptrs_[0][offset], inbox_[chunkOffset & 1], length);
      sendNotificationBuf_->send();
      recvNotificationBuf_->waitRecv();
      copyChunkAtOffset(chunkOffset);
    }
    for (int round = 0; round < (chunks_ - 2); round++) {
      auto chunkOffset = ((2 * rank_) - (round & ~0x1) + (round & 0x1) + chunks_) % chunks_;
      size_t offset = chunkOffset * chunkSize_, length = chunkSize_;
      if (offset + length <= (size_t)count_) {
      } else if (offset < (size_t)count_) {
        length = count_ - offset;
      } else {
        length = 0;
      }
      recvDataBuf_[chunkOffset & 1]->waitRecv();
      if (g_trace)
        std::fprintf(stderr, "r%d pass2 round %d chunk %d off %zu len %zu inbox %g\n", rank_, round, (int)chunkOffset,
                     offset, length, length ? firstValue(inbox_[chunkOffset & 1]) : 0.f);
      if (length > 0) copy(&ptrs_[0][offset], inbox_[chunkOffset & 1], length * sizeof(T));
      if (round < (chunks_ - 4)) {
        sendNotificationBuf_->send();
        recvNotificationBuf_->waitRecv();
        copyChunkAtOffset(chunkOffset);
      }
    }
    sendNotificationBuf_->send();
    recvNotificationBuf_->waitRecv();
    for (int i = 0; i < 2; i++) sendDataBuf_[i]->waitSend();
    for (size_t i = 1; i < ptrs_.size(); i++) copy(ptrs_[i], ptrs_[0], bytes_);
  }

 private:
  // fn_->call on the device, then the stream wait of
  // gloo/cuda_allreduce_ring_chunked.cc:185-190
  void reduce(T* dst, const T* src, size_t n) {
    fn_->call(dst, src, n, stream_);
    CHECK(hipStreamSynchronize(stream_));
  }
  // The reference's memcpy: a device copy that has COMPLETED on return.
  // (hipMemcpy device-to-device may return before the copy ran, and a
  // notification sent after it would let the peer overwrite the inbox first.)
  void copy(void* dst, const void* src, size_t bytes) {
    CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream_));
    CHECK(hipStreamSynchronize(stream_));
  }
  void copyChunkAtOffset(int chunkOffset) {
    size_t offset = (chunkOffset % chunks_) * chunkSize_, length = chunkSize_;
    if (offset + length <= (size_t)count_) {
    } else if (offset < (size_t)count_) {
      length = count_ - offset;
    } else {
      offset = 0;
      length = 1;  // gloo/allreduce_ring_chunked.h:224-231
    }
    if (g_trace)
      std::fprintf(stderr, "r%d send chunk %d buf %d off %zu len %zu value %g\n", rank_, chunkOffset, chunkOffset & 1,
                   offset, length, firstValue(&ptrs_[0][offset]));
    sendDataBuf_[chunkOffset & 0x1]->send(offset * sizeof(T), length * sizeof(T));
  }

  Device& dev_;
  const int rank_, size_;
  std::vector<T*> ptrs_;
  const int count_;
  const size_t bytes_;
  const gloo_amd::HipReductionFunction<T>* fn_;
  int chunks_ = 0;
  size_t chunkSize_ = 0, chunkBytes_ = 0;
  T* inbox_[2] = {nullptr, nullptr};
  hipStream_t stream_ = nullptr;
  std::unique_ptr<Buffer> sendDataBuf_[2], recvDataBuf_[2], sendNotificationBuf_, recvNotificationBuf_;
};

int main(int argc, char** argv) {
  const int P = argc > 1 ? std::atoi(argv[1]) : 4;
  const int count = argc > 2 ? std::atoi(argv[2]) : 100003;
  const int runs = argc > 3 ? std::atoi(argv[3]) : 2;
  // process mode: `transport_ring_chunked P count runs RANK STORE_DIR` runs
  // one rank in this process (receive buffers shared through HIP IPC)
  const int only = argc > 5 ? std::atoi(argv[4]) : -1;
  const std::string url = only >= 0 ? std::string("file:") + argv[5]
                                    : "mem:transport_ring_chunked_" + std::to_string(::getpid());
  std::vector<std::string> errors(P);
  std::vector<std::thread> ts;
  for (int rank = 0; rank < P; rank++) {
    if (only >= 0 && rank != only) continue;
    ts.emplace_back([&, rank] {
      try {
        CHECK(hipSetDevice(0));
        auto ctx = std::make_shared<gloo_amd::Context>(rank, P, std::chrono::seconds(60));
        ctx->connect(gloo_amd::openStore(url), 0);
        Device dev(ctx);
        float* d = nullptr;
        CHECK(hipMalloc(&d, std::max<size_t>(1, count * sizeof(float))));
        std::vector<float> h(count);
        int nextSlot = 0;
        {
          RingChunked<float> a(dev, {d}, count, nextSlot);
          for (int r = 0; r < runs; r++) {
            // values j % 1024 * P + rank: sums stay exact in fp32
            for (int j = 0; j < count; j++) h[j] = (float)((j % 1024) * P + rank);
            CHECK(hipMemcpy(d, h.data(), count * sizeof(float), hipMemcpyHostToDevice));
            a.run();
            CHECK(hipMemcpy(h.data(), d, count * sizeof(float), hipMemcpyDeviceToHost));
            for (int j = 0; j < count; j++) {
              const double want = (double)(j % 1024) * P * P + P * (P - 1) / 2.0;
              if ((double)h[j] != want)
                throw std::runtime_error("run " + std::to_string(r) + " element " + std::to_string(j) + ": " +
                                         std::to_string(h[j]) + " != " + std::to_string(want));
            }
          }
        }
        ctx->barrier("done");
        CHECK(hipFree(d));
      } catch (const std::exception& e) {
        errors[rank] = e.what();
      }
    });
  }
  for (auto& t : ts) t.join();
  int bad = 0;
  for (int r = 0; r < P; r++)
    if (!errors[r].empty()) {
      std::printf("rank %d: %s\n", r, errors[r].c_str());
      bad++;
    }
  if (bad) return 1;
  std::printf("ok: transport ring-chunked P=%d count=%d runs=%d\n", P, count, runs);
  return 0;
}

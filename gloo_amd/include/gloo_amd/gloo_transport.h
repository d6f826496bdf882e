// gloo_transport.h — the xGMI transport as a gloo::transport::Device.
//
// HEADER-ONLY and compiled on the GLOO side, like gloo_bridge.h: it includes
// the reference's transport headers and crosses into libgloo_amd.so only
// through the C-ABI of include/gloo_amd.h (gloo_hip_context_create_kv,
// gloo_hip_transport_*, gloo_hip_buffer_*).  libgloo_amd.so never links Gloo.
//
//   gloo::transport::tcp::CreateDevice(attr)  ->  gloo::transport::hip::CreateDevice(attr)
//        (gloo/transport/tcp/device.h:31; gloo/transport/device.h:34-54)
//   transport::Context::createAndConnectAllPairs(store)
//        (gloo/transport/context.cc:26-89): the set-up records travel through
//        the same gloo::IStore, so
//          gloo::transport::hip::attr a; a.device = localRank;
//          auto dev = gloo::transport::hip::CreateDevice(a);
//          auto ctx = std::make_shared<gloo::rendezvous::Context>(rank, size);
//          ctx->connectFullMesh(store, dev);   // gloo/rendezvous/context.cc:25-35
//        gives a gloo::Context whose pairs move bytes GPU to GPU;
//   Pair::createSendBuffer / createRecvBuffer (gloo/transport/pair.h:33-41)
//        over DEVICE memory: a receive buffer is HBM the peer writes into
//        (HIP IPC across processes; the pointer itself within one process,
//        where host memory is accepted too);
//   Buffer::send(offset, length, roffset) / waitRecv / waitSend
//        (gloo/transport/buffer.h:26-34): a device copy into the peer's
//        receive buffer — a direct xGMI copy between GPUs — whose arrival is
//        published stream-ordered after the bytes landed; waitRecv raises
//        gloo::IoException after the context timeout, as the TCP transport
//        does (gloo/transport/tcp/buffer.cc:67-73).
//
// This is what the reference's device algorithms need from a transport:
// CudaAllreduceRingChunked<T, CudaDeviceWorkspace<T>> creates its inboxes as
// device receive buffers on context->getPair(i)
// (gloo/cuda_allreduce_ring_chunked.cc:333-352) and relies on a transport
// that writes into GPU memory (ibverbs GPUDirect in the reference).
//
// Unbound buffers (gloo/transport/unbound_buffer.h:32-121):
//   Context::createUnboundBuffer(ptr, size), UnboundBuffer::send / recv
//   (recv-from-any over a rank list too), waitSend / waitRecv(rank, timeout),
//   abortWaitSend / abortWaitRecv, and Pair::send / recv(UnboundBuffer*):
//   two-sided messages matched per (source, slot) in order, through the
//   library's message queues (gloo_hip_ubuf_*: eager sends staged in node
//   shared memory).  So the reference's own gloo::allreduce, gloo::allgather,
//   gloo::reduce (gloo/allreduce.cc, allgather.cc, reduce.cc) run over this
//   transport unchanged, on host buffers as in the reference (they reduce on
//   the CPU with the options' reduce function).  The device-memory form of
//   those collectives is gloo_collectives.h (gloo::hip::allreduce / reduce).
//
// All ranks of a context run on one node (the arrival counters live in a
// node-local control block); each drives the HIP device given at CreateDevice.
// As with Gloo's own transports, buffers must be destroyed before the
// gloo::Context whose pairs created them, and a receive buffer must stay
// allocated while its pair lives.
#pragma once

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "gloo/common/error.h"
#include "gloo/common/logging.h"
#include "gloo/common/store.h"
#include "gloo/transport/address.h"
#include "gloo/transport/buffer.h"
#include "gloo/transport/context.h"
#include "gloo/transport/device.h"
#include "gloo/transport/pair.h"
#include "gloo/transport/unbound_buffer.h"
#include "gloo_amd.h"

namespace gloo {
namespace transport {
namespace hip {

struct attr {
  int device = -1;  // HIP device ordinal this rank drives; -1 = the calling thread's current device
  hipStream_t stream = nullptr;  // sends are ordered on it; nullptr = a stream of the transport's own
};

namespace detail {

inline void check(int rc, const char* what) {
  if (rc == GLOO_HIP_OK) return;
  const std::string msg = std::string(what) + ": " + gloo_hip_last_error();
  if (rc == GLOO_HIP_EIO) GLOO_THROW_IO_EXCEPTION(msg);
  GLOO_ENFORCE(false, msg);
}

}  // namespace detail

class Context;

// A pair's address: (rank, peer).  Connection state lives in the node's
// control block, so the bytes only confirm that both ends agree.
class Address : public ::gloo::transport::Address {
 public:
  Address(int rank, int peer) : rank_(rank), peer_(peer) {}
  std::string str() const override { return "hip:" + std::to_string(rank_) + "->" + std::to_string(peer_); }
  std::vector<char> bytes() const override {
    std::vector<char> b(2 * sizeof(int));
    std::memcpy(b.data(), &rank_, sizeof(int));
    std::memcpy(b.data() + sizeof(int), &peer_, sizeof(int));
    return b;
  }

 private:
  int rank_, peer_;
};

class Buffer : public ::gloo::transport::Buffer {
 public:
  Buffer(gloo_hip_buffer_t h, int slot, void* ptr, size_t size, bool isSend)
      : ::gloo::transport::Buffer(slot, ptr, size), h_(h), isSend_(isSend) {}
  ~Buffer() override { (void)gloo_hip_buffer_destroy(h_); }

  void send(size_t offset, size_t length, size_t roffset = 0) override {
    GLOO_ENFORCE(isSend_, "send on a receive buffer (slot ", slot_, ")");
    detail::check(gloo_hip_buffer_send(h_, offset, length, roffset), "hip::Buffer::send");
  }
  void waitRecv() override {
    GLOO_ENFORCE(!isSend_, "waitRecv on a send buffer (slot ", slot_, ")");
    detail::check(gloo_hip_buffer_wait_recv(h_), "hip::Buffer::waitRecv");
  }
  void waitSend() override {
    if (isSend_) detail::check(gloo_hip_buffer_wait_send(h_), "hip::Buffer::waitSend");
  }

 private:
  gloo_hip_buffer_t h_;
  bool isSend_;
};

class UnboundBuffer : public ::gloo::transport::UnboundBuffer {
 public:
  UnboundBuffer(Context* ctx, void* ptr, size_t size);
  ~UnboundBuffer() override { (void)gloo_hip_ubuf_destroy(h_); }

  bool waitRecv(int* rank, std::chrono::milliseconds timeout) override {
    return finish(gloo_hip_ubuf_wait_recv(h_, rank, (int)timeout.count()), "hip::UnboundBuffer::waitRecv");
  }
  bool waitSend(int* rank, std::chrono::milliseconds timeout) override {
    return finish(gloo_hip_ubuf_wait_send(h_, rank, (int)timeout.count()), "hip::UnboundBuffer::waitSend");
  }
  void abortWaitRecv() override { detail::check(gloo_hip_ubuf_abort_wait_recv(h_), "abortWaitRecv"); }
  void abortWaitSend() override { detail::check(gloo_hip_ubuf_abort_wait_send(h_), "abortWaitSend"); }

  void send(int dstRank, uint64_t slot, size_t offset = 0, size_t nbytes = kUnspecifiedByteCount) override {
    detail::check(gloo_hip_ubuf_send(h_, dstRank, slot, offset, nbytes), "hip::UnboundBuffer::send");
  }
  void recv(int srcRank, uint64_t slot, size_t offset = 0, size_t nbytes = kUnspecifiedByteCount) override {
    detail::check(gloo_hip_ubuf_recv(h_, &srcRank, 1, slot, offset, nbytes), "hip::UnboundBuffer::recv");
  }
  void recv(std::vector<int> srcRanks, uint64_t slot, size_t offset = 0,
            size_t nbytes = kUnspecifiedByteCount) override {
    detail::check(gloo_hip_ubuf_recv(h_, srcRanks.data(), (int)srcRanks.size(), slot, offset, nbytes),
                  "hip::UnboundBuffer::recv");
  }

 private:
  // 0: done; 1: aborted (false); a timeout raises IoException as in the
  // reference's transports
  static bool finish(int rc, const char* what) {
    if (rc == 1) return false;
    detail::check(rc, what);
    return true;
  }
  gloo_hip_ubuf_t h_ = nullptr;
};

class Pair : public ::gloo::transport::Pair {
 public:
  Pair(Context* ctx, int rank, int peer) : ctx_(ctx), address_(rank, peer), peer_(peer) { localRank_ = 0; }

  const ::gloo::transport::Address& address() const override { return address_; }

  void connect(const std::vector<char>& bytes) override {
    GLOO_ENFORCE_EQ(bytes.size(), 2 * sizeof(int), "bad hip pair address");
    int r = -1, p = -1;
    std::memcpy(&r, bytes.data(), sizeof(int));
    std::memcpy(&p, bytes.data() + sizeof(int), sizeof(int));
    GLOO_ENFORCE(r == peer_, "pair to rank ", peer_, " was handed the address of rank ", r);
    connected_ = true;
  }
  void close() override {}
  Context* hipContext() const { return ctx_; }
  // Waits poll the control block and back off on their own.
  void setSync(bool, bool) override {}
  bool isConnected() override { return connected_; }

  inline std::unique_ptr<::gloo::transport::Buffer> createSendBuffer(int slot, void* ptr, size_t size) override;
  inline std::unique_ptr<::gloo::transport::Buffer> createRecvBuffer(int slot, void* ptr, size_t size) override;

  // gloo/transport/pair.h:51-62: the buffer's send / recv with this pair's peer
  void send(::gloo::transport::UnboundBuffer* buf, uint64_t slot, size_t offset, size_t nbytes) override {
    auto* b = dynamic_cast<UnboundBuffer*>(buf);
    GLOO_ENFORCE(b != nullptr, "not an unbound buffer of the hip transport");
    b->send(peer_, slot, offset, nbytes);
  }
  void recv(::gloo::transport::UnboundBuffer* buf, uint64_t slot, size_t offset, size_t nbytes) override {
    auto* b = dynamic_cast<UnboundBuffer*>(buf);
    GLOO_ENFORCE(b != nullptr, "not an unbound buffer of the hip transport");
    b->recv(peer_, slot, offset, nbytes);
  }

 private:
  Context* ctx_;
  Address address_;
  int peer_;
  bool connected_ = false;
};

class Context : public ::gloo::transport::Context {
 public:
  Context(int rank, int size, int device, hipStream_t stream)
      : ::gloo::transport::Context(rank, size), device_(device), stream_(stream) {}

  ~Context() override {
    // buffers outlive neither their pairs nor the transport (the caller
    // destroys its algorithms before the gloo::Context)
    pairs_.clear();
    if (transport_) (void)gloo_hip_transport_destroy(transport_);
    if (ctx_) (void)gloo_hip_context_destroy(ctx_);
  }

  std::unique_ptr<::gloo::transport::Pair>& createPair(int peer) override {
    GLOO_ENFORCE(peer >= 0 && peer < size && peer != rank, "no pair to rank ", peer);
    pairs_[peer].reset(new Pair(this, rank, peer));
    return pairs_[peer];
  }

  // gloo/transport/context.cc:26-89, over the same store: the library's
  // context (control block, barriers) and the transport are set up through
  // it, then every pair is created and handed its peer's address.
  void createAndConnectAllPairs(std::shared_ptr<IStore> store) override {
    store_ = std::move(store);
    const int timeoutMs = (int)getTimeout().count();
    detail::check(gloo_hip_context_create_kv(rank, size, device_, timeoutMs, &Context::kvSet, &Context::kvGet, this,
                                             &ctx_),
                  "gloo_hip_context_create_kv");
    detail::check(gloo_hip_transport_create(ctx_, stream_, &transport_), "gloo_hip_transport_create");
    for (int i = 0; i < size; i++) {
      if (i == rank) continue;
      createPair(i);
    }
    for (int i = 0; i < size; i++) {
      if (i == rank) continue;
      getPair(i)->connect(Address(i, rank).bytes());
    }
  }

  std::unique_ptr<::gloo::transport::UnboundBuffer> createUnboundBuffer(void* ptr, size_t size) override {
    return std::unique_ptr<::gloo::transport::UnboundBuffer>(new UnboundBuffer(this, ptr, size));
  }

  gloo_hip_transport_t handle() const { return transport_; }

  // An all-gather of fixed `block`-byte records through the context's store
  // (set-up only; every rank calls it in the same order).  gloo_bridge.h
  // bootstraps the HipAllreduce* algorithms with it when the gloo::Context
  // runs on this transport: gloo::allgather needs unbound buffers.
  int allgather(const void* in, void* out, size_t block) {
    try {
      const std::string prefix = "gloo_amd/allgather/" + std::to_string(allgatherSeq_++) + "/";
      const char* p = static_cast<const char*>(in);
      store_->set(prefix + std::to_string(rank), std::vector<char>(p, p + block));
      for (int r = 0; r < size; r++) {
        const auto v = r == rank ? std::vector<char>(p, p + block)
                                 : store_->wait_get(prefix + std::to_string(r), getTimeout());
        if (v.size() != block) return GLOO_HIP_EIO;
        std::memcpy(static_cast<char*>(out) + (size_t)r * block, v.data(), block);
      }
      return 0;
    } catch (const std::exception&) {
      return GLOO_HIP_EIO;
    }
  }

 private:
  static int kvSet(void* user, const char* key, const void* data, size_t len) {
    try {
      auto* self = static_cast<Context*>(user);
      // one marker byte ahead of the value: Gloo's FileStore refuses an
      // empty value (gloo/rendezvous/file_store.cc:111) and records may be empty
      std::vector<char> v(1 + len, 'v');
      if (len) std::memcpy(v.data() + 1, data, len);
      self->store_->set(key, v);
      return 0;
    } catch (const std::exception&) {
      return GLOO_HIP_EIO;
    }
  }
  static int kvGet(void* user, const char* key, int timeoutMs, void* out, size_t cap, size_t* len) {
    try {
      auto* self = static_cast<Context*>(user);
      const auto v = self->store_->wait_get(key, std::chrono::milliseconds(timeoutMs));
      if (v.empty() || v[0] != 'v') return GLOO_HIP_EINVAL_ARG;
      *len = v.size() - 1;
      if (*len && *len <= cap) std::memcpy(out, v.data() + 1, *len);
      return 0;
    } catch (const std::exception&) {
      return GLOO_HIP_EIO;
    }
  }

  int device_;
  hipStream_t stream_;
  std::shared_ptr<IStore> store_;
  gloo_hip_context_t ctx_ = nullptr;
  gloo_hip_transport_t transport_ = nullptr;
  uint64_t allgatherSeq_ = 0;
};

inline UnboundBuffer::UnboundBuffer(Context* ctx, void* ptr, size_t size)
    : ::gloo::transport::UnboundBuffer(ptr, size) {
  GLOO_ENFORCE(ctx->handle() != nullptr, "transport not connected");
  detail::check(gloo_hip_ubuf_create(ctx->handle(), ptr, size, &h_), "hip::Context::createUnboundBuffer");
}

inline std::unique_ptr<::gloo::transport::Buffer> Pair::createSendBuffer(int slot, void* ptr, size_t size) {
  gloo_hip_buffer_t h = nullptr;
  detail::check(gloo_hip_buffer_create(ctx_->handle(), peer_, slot, ptr, size, 1, &h), "hip::Pair::createSendBuffer");
  return std::unique_ptr<::gloo::transport::Buffer>(new Buffer(h, slot, ptr, size, true));
}

inline std::unique_ptr<::gloo::transport::Buffer> Pair::createRecvBuffer(int slot, void* ptr, size_t size) {
  gloo_hip_buffer_t h = nullptr;
  detail::check(gloo_hip_buffer_create(ctx_->handle(), peer_, slot, ptr, size, 0, &h), "hip::Pair::createRecvBuffer");
  return std::unique_ptr<::gloo::transport::Buffer>(new Buffer(h, slot, ptr, size, false));
}

class Device : public ::gloo::transport::Device {
 public:
  explicit Device(const attr& a) : attr_(a) {
    if (attr_.device < 0) detail::check(hipGetDevice(&attr_.device) == hipSuccess ? 0 : GLOO_HIP_EINVAL_ARG,
                                        "hipGetDevice");
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), attr_.device) == hipSuccess) pciBusID_ = bus;
  }
  std::string str() const override { return "hip:" + std::to_string(attr_.device) + " (" + pciBusID_ + ")"; }
  const std::string& getPCIBusID() const override { return pciBusID_; }
  bool hasGPUDirect() const override { return true; }  // peers write straight into HBM
  std::shared_ptr<::gloo::transport::Context> createContext(int rank, int size) override {
    return std::make_shared<Context>(rank, size, attr_.device, attr_.stream);
  }

 private:
  attr attr_;
  std::string pciBusID_;
};

inline std::shared_ptr<::gloo::transport::Device> CreateDevice(const attr& a) {
  return std::make_shared<Device>(a);
}

}  // namespace hip
}  // namespace transport
}  // namespace gloo

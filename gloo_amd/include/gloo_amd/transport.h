// transport.h — an xGMI transport with the shape of Gloo's
// transport::Device / Pair / Buffer (gloo/transport/pair.h:21-81,
// gloo/transport/buffer.h:16-41), so an algorithm written against those
// interfaces moves device chunks GPU to GPU with no socket in between.
//
//   Pair::createRecvBuffer(slot, ptr, size)   registers a DEVICE buffer the
//        peer writes into: its allocation is exported (HIP IPC across
//        processes, the raw pointer within one) through the context's store;
//   Pair::createSendBuffer(slot, ptr, size)   a local device buffer; on its
//        first send it resolves the peer's receive buffer of the same slot;
//   Buffer::send(offset, length, roffset)     one-sided write: a device copy
//        (over the direct xGMI link when the peer is another GPU) into the
//        peer's buffer at roffset, then — stream-ordered, after the copy has
//        landed — the arrival counter of (me -> peer, slot) is bumped in the
//        node's control block (gloo_amd::Context);
//   Buffer::waitRecv()                        blocks until the next message of
//        this receive buffer has arrived (counter, bounded by the context
//        timeout -> IoException, as gloo/transport/tcp/buffer.cc:67-73);
//   Buffer::waitSend()                        blocks until the last send's
//        copy out of this buffer has completed.
//
// Chunks are written into the receiver's HBM and reduced there by the HIP
// kernels; nothing is staged through host memory.  Slots are arbitrary ints
// as in Gloo (context->nextSlot()); per (direction, peer) at most
// GLOO_HIP_NUM_SLOTS distinct slots modulo GLOO_HIP_NUM_SLOTS may be live.
// The store must support set/get (file: or mem: contexts).
//
// Receive buffers are the caller's memory, so unlike the executor's inboxes
// (executor.cc: a nonce at the arena's start, read back through every new
// IPC mapping) their imports are not verified; on ROCm 7 an import has been
// seen to show a previous allocation of the same size (DESIGN.md §4,
// "IPC imports are verified").  Keep receive buffers alive for the life of
// the pairs that use them, as Gloo's own transports require.
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <utility>
#include <vector>

#include "gloo_amd/context.h"

namespace gloo_amd {
namespace transport {

class Pair;

// One per rank: the transport device over a connected gloo_amd::Context.
// Construction reserves one of the context's counter instances; like
// algorithm construction it is collective (every rank in the same order).
class Device {
 public:
  explicit Device(std::shared_ptr<Context> ctx, hipStream_t stream = nullptr);
  ~Device();
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;

  // The pair to `peer` (gloo::Context::getPair, gloo/context.h:38).
  Pair& getPair(int peer);
  hipStream_t stream() const { return stream_; }
  const std::shared_ptr<Context>& context() const { return ctx_; }
  uint64_t instance() const { return inst_; }

  // (direction, peer, slot % kSlots) channels in use: a second live buffer
  // on one channel would share its counter.
  void claim(bool send, int peer, int slot);
  void release(bool send, int peer, int slot);

 private:
  std::shared_ptr<Context> ctx_;
  uint64_t inst_;
  hipStream_t stream_ = nullptr;
  bool ownStream_ = false;
  std::map<int, std::unique_ptr<Pair>> pairs_;
  std::mutex m_;
  std::set<std::tuple<bool, int, int>> channels_;
};

class Buffer {
 public:
  virtual ~Buffer() = default;
  virtual void send(size_t offset, size_t length, size_t roffset = 0) = 0;
  // the whole buffer (gloo/transport/buffer.h:28-31)
  void send() { send(0, size_); }
  virtual void waitRecv() = 0;
  virtual void waitSend() = 0;
  int slot() const { return slot_; }
  size_t size() const { return size_; }

 protected:
  Buffer(int slot, void* ptr, size_t size) : slot_(slot), ptr_(static_cast<char*>(ptr)), size_(size) {}
  int slot_;
  char* ptr_;
  size_t size_;
};

class Pair {
 public:
  Pair(Device* dev, int peer) : dev_(dev), peer_(peer) {}
  std::unique_ptr<Buffer> createSendBuffer(int slot, void* ptr, size_t size);
  std::unique_ptr<Buffer> createRecvBuffer(int slot, void* ptr, size_t size);
  int peer() const { return peer_; }

 private:
  Device* dev_;
  int peer_;
};

}  // namespace transport
}  // namespace gloo_amd

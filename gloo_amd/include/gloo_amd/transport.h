// transport.h — an xGMI transport with the shape of Gloo's
// transport::Device / Pair / Buffer / UnboundBuffer (gloo/transport/pair.h:21-81,
// gloo/transport/buffer.h:16-41, gloo/transport/unbound_buffer.h:32-121), so an
// algorithm written against those interfaces moves device chunks GPU to GPU
// with no socket in between.
//
// Bound buffers (the GPU algorithms' inboxes):
//   Pair::createRecvBuffer(slot, ptr, size)   registers memory the peer writes
//        into: DEVICE memory is exported (HIP IPC across processes, the raw
//        pointer within one); HOST memory is written directly within one
//        process, and across processes through a LANDING segment of the same
//        size in node shared memory that the receiver creates with the buffer:
//        the sender writes a message at its offset there, and the receiver's
//        waitRecv copies exactly that message's range into the buffer — any
//        length, as the reference's TCP pair writes any length into a
//        registered buffer (gloo/transport/tcp/pair.cc:413-426);
//   Pair::createSendBuffer(slot, ptr, size)   a local buffer; on its first send
//        it resolves the peer's receive buffer of the same slot;
//   Buffer::send(offset, length, roffset)     one-sided write into the peer's
//        buffer at roffset, then the channel's arrival counter := the
//        message's arrival number.  Device bytes move stream-ordered and the
//        arrival is published FROM THE DEVICE: a device-to-device message is
//        one copy kernel with the signal fused in (signal.h launchCopySignal;
//        over the direct xGMI link when the peer is another GPU), any other
//        device-side copy is followed by the signal kernel — no host callback
//        and no host round trip per message.  Host-to-host messages are
//        written and published by the sending thread itself;
//   Buffer::waitRecv()                        blocks until the next message of
//        this receive buffer has arrived (bounded by the context timeout ->
//        IoException, as gloo/transport/tcp/buffer.cc:67-73);
//   Buffer::waitSend()                        blocks until the last send's copy
//        out of this buffer has completed.
// Every receive buffer owns one channel (an arrival counter, plus a ring of
// kMsgRing message records) of the transport block, allocated by the
// receiver per (sender, slot) and published with its record (with the
// counter's value at creation, so the sender numbers its messages), so any
// number of slots may be live — as many as kChannels per (sender, receiver)
// at once — and Gloo's ever-increasing context->nextSlot() values never
// collide.  A landed message k (the k-th arrival of its channel) is described
// by record k % kMsgRing, tagged with k; the receiver copies it out in the
// waitRecv that expects arrival k and acknowledges it, and the sender reuses a
// record only once its last message was acknowledged (waiting on the sending
// thread, bounded by the context timeout, when kMsgRing messages are
// unconsumed).  So a second send before the receiver's wait keeps both
// messages, as the reference's direct writes do, and a device receive buffer
// reusing the channel never reads a record.
//
// Unbound buffers (the new-style collectives, gloo/allreduce.cc,
// gloo/allgather.cc, gloo/reduce.cc): two-sided send / recv matched per
// (source, slot) in order, recv-from-any over a set of source ranks (the
// earliest announced message wins, as the reference's Tally keeps arrival
// order, gloo/transport/context.h:107-125).  Sends are EAGER: the bytes are
// staged in a shared-memory segment of their own (a device buffer through a
// device-to-host copy) and announced in the (sender, receiver) queue of the
// transport block; the send is complete at once (waitSend reports the
// destination), and the receiver copies the bytes out in waitRecv.  So
// neither side ever waits for the other to post first, and host buffers
// work between processes.  This path moves bytes through host memory: it
// serves the reference's host-memory algorithms (which reduce on the CPU
// anyway), not the device hot path, which is the executor's (executor.h).
//
// All ranks of a context run on one node; each drives the HIP device given
// at construction.  The transport block is created by the transport's
// collective construction (every rank, same order as its algorithms).
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "gloo_amd/context.h"

namespace gloo_amd {
namespace transport {

class Pair;

constexpr int kChannels = 128;       // live receive buffers per (sender, receiver)
constexpr int kAnnouncements = 128;  // unbound messages in flight per (sender, receiver)
constexpr int kMsgRing = 16;          // landed messages in flight per channel (host receive buffers)

// One per rank: the transport device over a connected gloo_amd::Context.
// Construction is collective (every rank, in the same order as its
// algorithms): it maps the transport block.
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

  // A (direction, peer, slot) may hold one live buffer at a time.
  void claim(bool send, int peer, uint64_t slot);
  void release(bool send, int peer, uint64_t slot);

  struct Channel {
    std::atomic<uint64_t> count;  // arrivals
    // the arrival number of the last message sent on the channel: senders
    // number their messages from it, so a send buffer closed and created
    // again on the same slot continues the numbering (set to the count's
    // value by the receive buffer that takes the channel)
    std::atomic<uint64_t> sent;
    uint64_t pad[6];
  };
  static_assert(sizeof(Channel) == 64, "one line per channel");
  struct MsgRecord {
    std::atomic<uint64_t> seq;  // the arrival number of the message it describes (0: never used)
    std::atomic<uint64_t> ack;  // the arrival number the receiver consumed from it
    uint64_t off, len;          // the message's place in the receive buffer (and its landing segment)
    uint64_t pad[4];
  };
  static_assert(sizeof(MsgRecord) == 64, "one line per record");
  Channel& channel(int src, int dst, int idx);
  // The channel's arrival counter as a device kernel addresses it (the
  // transport block registered with HIP on first use).
  uint64_t* channelDevicePtr(int src, int dst, int idx);
  // The record arrival `k` of channel (src -> dst, idx) uses.
  MsgRecord& msgRecord(int src, int dst, int idx, uint64_t k);
  int allocChannel(int src);  // receiver side: a free channel of (src -> me)
  void freeChannel(int src, int idx);

  // Unbound messages (transport.cc).
  struct Announcement {
    std::atomic<uint32_t> state;  // 0 free, 1 being written, 2 ready, 3 being taken
    uint32_t pad;
    uint64_t slot, nbytes, order;
    char name[32];                // the staging segment ("" for 0 bytes)
  };
  static_assert(sizeof(Announcement) == 64, "one line per announcement");
  // Eager send of [ptr, ptr + n) (host or device memory) to `dst` on `slot`.
  void announce(int dst, uint64_t slot, const void* ptr, size_t n);
  // Takes the earliest announced message on `slot` from any of `srcs` and
  // copies it to `dst` (n bytes, which must be the message's size).
  // Returns false if none has been announced yet.
  bool take(const std::vector<int>& srcs, uint64_t slot, void* dst, size_t n, int* src);

 private:
  Announcement& announcement(int src, int dst, int idx);
  std::atomic<uint64_t>& orderCounter(int dst);

  std::shared_ptr<Context> ctx_;
  uint64_t inst_;
  hipStream_t stream_ = nullptr;
  bool ownStream_ = false;
  std::map<int, std::unique_ptr<Pair>> pairs_;
  std::mutex m_;
  std::set<std::tuple<bool, int, uint64_t>> live_;
  std::vector<std::vector<bool>> channelUsed_;  // [src][idx], this rank as receiver
  void* block_ = nullptr;
  size_t blockBytes_ = 0;
  void* blockDev_ = nullptr;  // block_ as registered with HIP (channelDevicePtr)
};

class Buffer {
 public:
  virtual ~Buffer() = default;
  virtual void send(size_t offset, size_t length, size_t roffset = 0) = 0;
  // the whole buffer (gloo/transport/buffer.h:28-31)
  void send() { send(0, size_); }
  virtual void waitRecv() = 0;
  virtual void waitSend() = 0;
  uint64_t slot() const { return slot_; }
  size_t size() const { return size_; }

 protected:
  Buffer(uint64_t slot, void* ptr, size_t size) : slot_(slot), ptr_(static_cast<char*>(ptr)), size_(size) {}
  uint64_t slot_;
  char* ptr_;
  size_t size_;
};

class Pair {
 public:
  Pair(Device* dev, int peer) : dev_(dev), peer_(peer) {}
  std::unique_ptr<Buffer> createSendBuffer(uint64_t slot, void* ptr, size_t size);
  std::unique_ptr<Buffer> createRecvBuffer(uint64_t slot, void* ptr, size_t size);
  int peer() const { return peer_; }

 private:
  Device* dev_;
  int peer_;
};

// gloo::transport::UnboundBuffer (gloo/transport/unbound_buffer.h:32-121) over
// the Device's message queues.  One thread uses a buffer at a time.
class UnboundBuffer {
 public:
  UnboundBuffer(Device* dev, void* ptr, size_t size) : dev_(dev), ptr_(static_cast<char*>(ptr)), size_(size) {}
  void send(int dst, uint64_t slot, size_t offset, size_t nbytes);
  void recv(const std::vector<int>& srcs, uint64_t slot, size_t offset, size_t nbytes);
  // true: completed (*rank = the peer); false: aborted.  timeout < 0: the
  // context's.  Throws IoException on timeout.
  bool waitRecv(int* rank, std::chrono::milliseconds timeout);
  bool waitSend(int* rank, std::chrono::milliseconds timeout);
  void abortWaitRecv() { abortRecv_ = true; }
  void abortWaitSend() { abortSend_ = true; }

 private:
  struct PendingRecv {
    std::vector<int> srcs;
    uint64_t slot;
    size_t offset, nbytes;
  };
  Device* dev_;
  char* ptr_;
  size_t size_;
  std::deque<PendingRecv> recvs_;
  std::deque<int> sent_;  // destinations of completed sends not yet waited for
  std::atomic<bool> abortRecv_{false}, abortSend_{false};
};

}  // namespace transport
}  // namespace gloo_amd

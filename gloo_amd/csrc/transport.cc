// transport.cc — see transport.h.
#include "gloo_amd/transport.h"

#include <sched.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <string>
#include <thread>

#include "gloo_amd.h"
#include "gloo_amd/common.h"

namespace gloo_amd {
namespace transport {
namespace {

// What a receive buffer publishes for the peer that writes into it.
struct RecvRecord {
  int32_t pid;
  int32_t device;
  uint64_t ptr;     // the buffer itself (same process)
  uint64_t size;    // bytes the peer may write
  uint64_t offset;  // from the start of its allocation (IPC maps whole allocations)
  int32_t ipc;      // handle valid
  hipIpcMemHandle_t handle;
};

std::string recordKey(uint64_t inst, int sender, int receiver, int slot) {
  return strcat_("gloo_amd/xgmi/", inst, "/", sender, "->", receiver, "/", slot);
}

void bump(void* p) { static_cast<std::atomic<uint64_t>*>(p)->fetch_add(1, std::memory_order_acq_rel); }

int channel(int slot) { return ((slot % GLOO_HIP_NUM_SLOTS) + GLOO_HIP_NUM_SLOTS) % GLOO_HIP_NUM_SLOTS; }

class SendBuffer : public Buffer {
 public:
  SendBuffer(Device* dev, int peer, int slot, void* ptr, size_t size)
      : Buffer(slot, ptr, size), dev_(dev), peer_(peer) {
    dev_->claim(true, peer_, slot_);
    GLOO_AMD_HIP_CHECK(hipEventCreateWithFlags(&sent_, hipEventDisableTiming));
  }
  ~SendBuffer() override {
    (void)hipEventSynchronize(sent_);
    (void)hipEventDestroy(sent_);
    if (opened_) GLOO_AMD_HIP_RELEASE(hipIpcCloseMemHandle(opened_));
    dev_->release(true, peer_, slot_);
  }

  void send(size_t offset, size_t length, size_t roffset) override {
    Context& ctx = *dev_->context();
    GLOO_AMD_HIP_CHECK(hipSetDevice(ctx.device()));
    resolve();
    GLOO_AMD_ENFORCE(offset + length <= size_, "send of [", offset, ", +", length, ") beyond a ", size_,
                     "-byte send buffer");
    GLOO_AMD_ENFORCE(roffset + length <= peerSize_, "send of ", length, " bytes at ", roffset, " beyond rank ", peer_,
                     "'s ", peerSize_, "-byte receive buffer (slot ", slot_, ")");
    hipStream_t s = dev_->stream();
    if (length) GLOO_AMD_HIP_CHECK(hipMemcpyAsync(remote_ + roffset, ptr_ + offset, length, hipMemcpyDefault, s));
    // stream-ordered: the arrival is published only once the bytes landed
    GLOO_AMD_HIP_CHECK(hipLaunchHostFunc(s, bump, &ctx.counter(dev_->instance(), ctx.rank, peer_, channel(slot_))));
    GLOO_AMD_HIP_CHECK(hipEventRecord(sent_, s));
  }
  void waitRecv() override { throw EnforceNotMet("waitRecv on a send buffer"); }
  void waitSend() override { GLOO_AMD_HIP_CHECK(hipEventSynchronize(sent_)); }

 private:
  // The peer's receive buffer of this slot (published when it was created).
  void resolve() {
    if (resolved_) return;
    Context& ctx = *dev_->context();
    const auto v = ctx.store().get(recordKey(dev_->instance(), ctx.rank, peer_, slot_), ctx.timeout());
    GLOO_AMD_ENFORCE(v.size() == sizeof(RecvRecord), "bad receive-buffer record from rank ", peer_);
    RecvRecord r;
    std::memcpy(&r, v.data(), sizeof(r));
    peerSize_ = r.size;
    if (r.size == 0) {
      remote_ = nullptr;  // a notification buffer: arrivals only
    } else if (r.pid == ctx.pid()) {
      remote_ = reinterpret_cast<char*>(r.ptr);
      if (r.device != ctx.device()) {
        hipError_t e = hipDeviceEnablePeerAccess(r.device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) GLOO_AMD_HIP_CHECK(e);
        (void)hipGetLastError();
      }
    } else {
      GLOO_AMD_ENFORCE(r.ipc, "rank ", peer_, "'s receive buffer is not IPC-exportable");
      void* base = nullptr;
      GLOO_AMD_HIP_ALLOC(hipIpcOpenMemHandle(&base, r.handle, hipIpcMemLazyEnablePeerAccess));
      opened_ = base;
      remote_ = static_cast<char*>(base) + r.offset;
      // the runtime's record of the mapping must reach the whole buffer (an
      // import can come back at the size of an earlier allocation at the same
      // address: executor.cc, DESIGN.md §4 "IPC imports must also be sized right")
      void* rb = nullptr;
      size_t rs = 0;
      if (hipMemGetAddressRange(&rb, &rs, base) == hipSuccess && rb) {
        GLOO_AMD_ENFORCE(static_cast<char*>(rb) + rs >= remote_ + r.size, "the IPC mapping of rank ", peer_,
                         "'s receive buffer (slot ", slot_, ") reaches ", rs, " B from ", rb, ", short of its ",
                         r.offset + r.size, " B");
      } else {
        (void)hipGetLastError();
      }
    }
    resolved_ = true;
  }

  Device* dev_;
  int peer_;
  bool resolved_ = false;
  char* remote_ = nullptr;
  void* opened_ = nullptr;
  size_t peerSize_ = 0;
  hipEvent_t sent_ = nullptr;
};

class RecvBuffer : public Buffer {
 public:
  RecvBuffer(Device* dev, int peer, int slot, void* ptr, size_t size)
      : Buffer(slot, ptr, size), dev_(dev), peer_(peer) {
    Context& ctx = *dev_->context();
    dev_->claim(false, peer_, slot_);
    // baseline before the record is published, i.e. before the peer's
    // first send can land (the sender resolves the record first)
    baseline_ = ctx.counter(dev_->instance(), peer_, ctx.rank, channel(slot_)).load(std::memory_order_acquire);
    RecvRecord r;
    std::memset(&r, 0, sizeof(r));
    r.pid = ctx.pid();
    r.device = ctx.device();
    r.ptr = reinterpret_cast<uint64_t>(ptr_);
    r.size = ptr_ ? size_ : 0;
    if (ptr_ && size_) {
      void* base = nullptr;
      size_t allocSize = 0;
      if (hipMemGetAddressRange(&base, &allocSize, ptr_) == hipSuccess && base &&
          hipIpcGetMemHandle(&r.handle, base) == hipSuccess) {
        r.ipc = 1;
        r.offset = (uint64_t)(ptr_ - static_cast<char*>(base));
      }
      (void)hipGetLastError();
    }
    std::vector<char> blob(sizeof(r));
    std::memcpy(blob.data(), &r, sizeof(r));
    ctx.store().set(recordKey(dev_->instance(), peer_, ctx.rank, slot_), blob);
  }
  ~RecvBuffer() override { dev_->release(false, peer_, slot_); }

  void send(size_t, size_t, size_t) override { throw EnforceNotMet("send on a receive buffer"); }
  void waitSend() override {}
  void waitRecv() override {
    Context& ctx = *dev_->context();
    auto& c = ctx.counter(dev_->instance(), peer_, ctx.rank, channel(slot_));
    const uint64_t target = baseline_ + ++received_;
    auto met = [&] { return (int64_t)(c.load(std::memory_order_acquire) - target) >= 0; };
    const auto deadline = std::chrono::steady_clock::now() + ctx.timeout();
    for (uint64_t i = 0; !met(); i++) {
      if (i < 4096) {
        __builtin_ia32_pause();
      } else if (i < 8192) {
        sched_yield();
      } else {
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
      if ((i & 255) == 255 && std::chrono::steady_clock::now() > deadline)
        throw IoException(strcat_("Timed out waiting for rank ", peer_, " (slot ", slot_, ") on rank ", ctx.rank,
                                  " after ", ctx.timeout().count(), " ms"));
    }
  }

 private:
  Device* dev_;
  int peer_;
  uint64_t baseline_ = 0, received_ = 0;
};

}  // namespace

Device::Device(std::shared_ptr<Context> ctx, hipStream_t stream) : ctx_(std::move(ctx)) {
  GLOO_AMD_HIP_CHECK(hipSetDevice(ctx_->device()));
  inst_ = ctx_->acquireInstance();
  if (stream) {
    stream_ = stream;
  } else {
    GLOO_AMD_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    ownStream_ = true;
  }
}

Device::~Device() {
  pairs_.clear();
  if (stream_) (void)hipStreamSynchronize(stream_);
  if (ownStream_) (void)hipStreamDestroy(stream_);
  ctx_->releaseInstance(inst_);
}

Pair& Device::getPair(int peer) {
  GLOO_AMD_ENFORCE(peer >= 0 && peer < ctx_->size && peer != ctx_->rank, "no pair to rank ", peer);
  auto& p = pairs_[peer];
  if (!p) p.reset(new Pair(this, peer));
  return *p;
}

void Device::claim(bool send, int peer, int slot) {
  std::lock_guard<std::mutex> lk(m_);
  GLOO_AMD_ENFORCE(channels_.insert(std::make_tuple(send, peer, channel(slot))).second, "slot ", slot,
                   " shares its channel with a live ", send ? "send" : "receive", " buffer to/from rank ", peer);
}

void Device::release(bool send, int peer, int slot) {
  std::lock_guard<std::mutex> lk(m_);
  channels_.erase(std::make_tuple(send, peer, channel(slot)));
}

std::unique_ptr<Buffer> Pair::createSendBuffer(int slot, void* ptr, size_t size) {
  return std::unique_ptr<Buffer>(new SendBuffer(dev_, peer_, slot, ptr, size));
}

std::unique_ptr<Buffer> Pair::createRecvBuffer(int slot, void* ptr, size_t size) {
  return std::unique_ptr<Buffer>(new RecvBuffer(dev_, peer_, slot, ptr, size));
}

}  // namespace transport
}  // namespace gloo_amd

// context.h — gloo_amd::Context: rank, size, timeout, device, and the
// node-local control block through which ranks signal each other.
//
// Mirrors gloo::Context (gloo/context.h:26-59: rank, size, nextSlot,
// timeout) bootstrapped like rendezvous::Context::connectFullMesh
// (gloo/rendezvous/context.cc:25-35).  The "transport" for GPU chunks is not
// a socket: every rank maps the peers' inbox arenas (HIP IPC across
// processes, plain pointers within one process) and moves chunks with
// device-to-device copies over xGMI; arrivals and notifications are
// monotonically increasing 64-bit counters in a POSIX shared-memory block
// that all ranks of the node map.
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "gloo_amd/store.h"

namespace gloo_amd {

class Context : public std::enable_shared_from_this<Context> {
 public:
  Context(int rank, int size, std::chrono::milliseconds timeout = std::chrono::seconds(30));
  ~Context();

  // Collective: create/map the control block, record the HIP device this
  // rank drives, and barrier.  The store carries only setup metadata.
  void connect(std::shared_ptr<Store> store, int device);

  const int rank;
  const int size;
  // AllreduceBcube's group size (gloo::Context::base, gloo/context.h:28-33)
  int base = 2;

  int device() const { return device_; }
  std::chrono::milliseconds timeout() const { return timeout_; }
  void setTimeout(std::chrono::milliseconds t) { timeout_ = t; }
  Store& store() { return *store_; }
  int pid() const { return pid_; }

  // Algorithm instances are numbered in construction order, which must be
  // the same on every rank (the role of gloo::Context::nextSlot).
  uint64_t nextInstance() { return nextInstance_++; }
  static constexpr uint64_t kMaxLiveInstances = 64;
  // nextInstance() for a user of the control block's counters (an
  // algorithm's executor, a transport device), registered live until
  // releaseInstance: counters are recycled modulo kMaxLiveInstances, so at
  // most that many may be live at once.
  uint64_t acquireInstance();
  void releaseInstance(uint64_t inst);

  // Counter for messages src -> dst on `slot` of instance `inst`.
  std::atomic<uint64_t>& counter(uint64_t inst, int src, int dst, int slot);
  // The same counter as a GPU-addressable pointer (the control block is
  // registered with hipHostRegister on first use).
  uint64_t* counterDevicePtr(uint64_t inst, int src, int dst, int slot);
  // Per-rank error word written by device-side waits that time out.
  std::atomic<uint32_t>& errorWord(int r);
  uint32_t* errorWordDevicePtr(int r);

  // Store-based barrier among all ranks (setup / teardown only).
  void barrier(const std::string& tag);
  // Collective exchange of one small blob per rank (setup / teardown only);
  // every rank calls it in the same order.
  std::vector<std::vector<char>> allgather(const std::string& tag, const std::vector<char>& mine);

 private:
  std::chrono::milliseconds timeout_;
  std::shared_ptr<Store> store_;
  int device_ = -1;
  int pid_;
  uint64_t nextInstance_ = 0;
  std::mutex liveMutex_;
  std::set<uint64_t> live_;
  std::string shmName_;
  void* shm_ = nullptr;
  void* shmDev_ = nullptr;
  size_t shmBytes_ = 0;
  size_t countersBytes_ = 0;
  void ensureDeviceMapped();
  uint64_t barrierGen_ = 0;
};

}  // namespace gloo_amd

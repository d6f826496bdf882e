// context.cc — see context.h.
#include "gloo_amd/context.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <random>

#include "gloo_amd.h"
#include "gloo_amd/common.h"

#include <hip/hip_runtime_api.h>

namespace gloo_amd {

namespace {
struct ShmHeader {
  uint64_t magic;
  uint64_t size;
  uint64_t slots;
  uint64_t pad;
};
constexpr uint64_t kMagic = 0x676c6f6f5f616d64ull;  // "gloo_amd"

std::vector<char> bytes(const std::string& s) { return std::vector<char>(s.begin(), s.end()); }
}  // namespace

Context::Context(int r, int s, std::chrono::milliseconds timeout)
    : rank(r), size(s), timeout_(timeout), pid_((int)::getpid()) {
  GLOO_AMD_ENFORCE(size >= 1 && rank >= 0 && rank < size, "bad rank ", rank, " / size ", size);
}

Context::~Context() {
  if (shmDev_) GLOO_AMD_HIP_RELEASE(hipHostUnregister(shm_));
  if (shm_) ::munmap(shm_, shmBytes_);
}

void Context::connect(std::shared_ptr<Store> store, int device) {
  store_ = std::move(store);
  device_ = device;
  countersBytes_ = kMaxLiveInstances * (size_t)size * size * GLOO_HIP_NUM_SLOTS * sizeof(uint64_t);
  shmBytes_ = sizeof(ShmHeader) + countersBytes_ + ((size_t)size * sizeof(uint32_t) + 63) / 64 * 64;
  shmBytes_ = (shmBytes_ + 4095) / 4096 * 4096;
  if (rank == 0) {
    std::random_device rd;
    shmName_ = strcat_("/gloo_amd_", pid_, "_", rd(), rd());
    int fd = ::shm_open(shmName_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    GLOO_AMD_ENFORCE(fd >= 0, "shm_open(create) failed for ", shmName_);
    GLOO_AMD_ENFORCE(::ftruncate(fd, (off_t)shmBytes_) == 0, "ftruncate failed");
    shm_ = ::mmap(nullptr, shmBytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    GLOO_AMD_ENFORCE(shm_ != MAP_FAILED, "mmap failed");
    auto* h = static_cast<ShmHeader*>(shm_);
    h->size = size;
    h->slots = GLOO_HIP_NUM_SLOTS;
    std::atomic_thread_fence(std::memory_order_release);
    h->magic = kMagic;
  }
  // rank 0 publishes the control block's name
  const auto names = allgather("shm", rank == 0 ? bytes(shmName_) : std::vector<char>{});
  if (rank != 0) {
    shmName_.assign(names[0].begin(), names[0].end());
    int fd = ::shm_open(shmName_.c_str(), O_RDWR, 0600);
    GLOO_AMD_ENFORCE(fd >= 0, "shm_open failed for ", shmName_);
    shm_ = ::mmap(nullptr, shmBytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    GLOO_AMD_ENFORCE(shm_ != MAP_FAILED, "mmap failed");
    auto* h = static_cast<ShmHeader*>(shm_);
    GLOO_AMD_ENFORCE(h->magic == kMagic && (int)h->size == size, "control block mismatch");
  }
  barrier("connect");
  if (rank == 0) ::shm_unlink(shmName_.c_str());  // every rank has it mapped now
}

std::atomic<uint64_t>& Context::counter(uint64_t inst, int src, int dst, int slot) {
  GLOO_AMD_ENFORCE(shm_ != nullptr, "context not connected");
  auto* base = reinterpret_cast<std::atomic<uint64_t>*>(static_cast<char*>(shm_) + sizeof(ShmHeader));
  const size_t i = (((inst % kMaxLiveInstances) * size + src) * size + dst) * GLOO_HIP_NUM_SLOTS + slot;
  return base[i];
}

void Context::ensureDeviceMapped() {
  if (shmDev_) return;
  GLOO_AMD_HIP_ALLOC(hipHostRegister(shm_, shmBytes_, hipHostRegisterMapped | hipHostRegisterPortable));
  void* d = nullptr;
  GLOO_AMD_HIP_CHECK(hipHostGetDevicePointer(&d, shm_, 0));
  shmDev_ = d;
}

uint64_t* Context::counterDevicePtr(uint64_t inst, int src, int dst, int slot) {
  ensureDeviceMapped();
  const size_t off = reinterpret_cast<char*>(&counter(inst, src, dst, slot)) - static_cast<char*>(shm_);
  return reinterpret_cast<uint64_t*>(static_cast<char*>(shmDev_) + off);
}

std::atomic<uint32_t>& Context::errorWord(int r) {
  auto* base = reinterpret_cast<std::atomic<uint32_t>*>(static_cast<char*>(shm_) + sizeof(ShmHeader) + countersBytes_);
  return base[r];
}

uint32_t* Context::errorWordDevicePtr(int r) {
  ensureDeviceMapped();
  const size_t off = reinterpret_cast<char*>(&errorWord(r)) - static_cast<char*>(shm_);
  return reinterpret_cast<uint32_t*>(static_cast<char*>(shmDev_) + off);
}

uint64_t Context::acquireInstance() {
  const uint64_t inst = nextInstance();
  std::lock_guard<std::mutex> lk(liveMutex_);
  GLOO_AMD_ENFORCE(live_.insert(inst % kMaxLiveInstances).second, "more than ", kMaxLiveInstances,
                   " live algorithm instances on one context");
  return inst;
}

void Context::releaseInstance(uint64_t inst) {
  std::lock_guard<std::mutex> lk(liveMutex_);
  live_.erase(inst % kMaxLiveInstances);
}

void Context::barrier(const std::string& tag) { (void)allgather("barrier/" + tag, {}); }

std::vector<std::vector<char>> Context::allgather(const std::string& tag, const std::vector<char>& mine) {
  const uint64_t gen = barrierGen_++;
  return store_->allgather(strcat_("gloo_amd/ag/", gen, "/", tag), rank, size, mine, timeout_);
}

}  // namespace gloo_amd

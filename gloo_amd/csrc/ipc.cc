// ipc.cc — see gloo_amd/ipc.h.
#include "gloo_amd/ipc.h"

#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "gloo_amd/common.h"

namespace gloo_amd {
namespace ipc {
namespace {

constexpr size_t kGranule = size_t(2) << 20;

size_t sizeClass(size_t bytes) {
  // powers of two up to 1 GiB, then multiples of 256 MiB (no upper bound:
  // VMM imports of any size map, ipc.h)
  constexpr size_t kBig = size_t(1) << 30, kStep = size_t(256) << 20;
  if (bytes > kBig) return (bytes + kStep - 1) / kStep * kStep;
  size_t c = kGranule;
  while (c < bytes) c <<= 1;
  return c;
}

hipMemAllocationProp propFor(int device, bool fine) {
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof(p));
  // uncached: what a peer GPU or process writes is never behind a stale
  // line of this GPU's caches (the executor's cross-written inboxes and
  // mailboxes, as hipDeviceMallocFinegrained memory was before)
  p.type = fine ? hipMemAllocationTypeUncached : hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  return p;
}

// A virtual range of `bytes` never mapped before (ranges are never freed:
// a range mapped twice kept the first mapping's translations, ipc.h).
void* freshRange(size_t bytes) {
  void* va = nullptr;
  GLOO_AMD_HIP_ALLOC(hipMemAddressReserve(&va, bytes, kGranule, nullptr, 0));
  return va;
}

// Read-write access to [va, va + bytes) from `device` (the mapping's other
// devices keep theirs).
hipError_t allowAccess(void* va, size_t bytes, int device) {
  hipMemAccessDesc d;
  std::memset(&d, 0, sizeof(d));
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = device;
  d.flags = hipMemAccessFlagsProtReadWrite;
  return hipMemSetAccess(va, bytes, &d, 1);
}

void mapAt(void* va, size_t bytes, hipMemGenericAllocationHandle_t h, int device) {
  GLOO_AMD_HIP_CHECK(hipMemMap(va, bytes, 0, h, 0));
  hipMemAccessDesc d;
  std::memset(&d, 0, sizeof(d));
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = device;
  d.flags = hipMemAccessFlagsProtReadWrite;
  const hipError_t e = hipMemSetAccess(va, bytes, &d, 1);
  if (e != hipSuccess) {
    (void)hipMemUnmap(va, bytes);
    GLOO_AMD_HIP_CHECK(e);
  }
}

struct Pool {
  std::mutex m;
  std::vector<std::unique_ptr<Slab>> slabs;  // every exported slab (never freed: ipc.h)
  std::vector<Slab*> free;
  uint64_t nextId = 1;
  struct Mapping {
    uint64_t incarnation;
    void* ptr;
    size_t bytes;
    size_t users;  // executors holding it (import / unimport)
    hipMemGenericAllocationHandle_t handle;
    uint64_t devices;  // bit d: device d may access it
  };
  std::map<std::pair<int, uint64_t>, Mapping> imports;  // (exporter pid, slab id)
  struct Exported {
    int fd;
    uint64_t bytes;  // of the whole dma-buf
  };
  std::map<uint64_t, Exported> exports;  // exportRange: id -> dma-buf
  size_t opens = 0, dropped = 0;
  static Pool& get() {
    static Pool* p = new Pool();  // never destroyed: releaseAllAtExit unmaps
    return *p;
  }
};

// ---- the fd server -----------------------------------------------------------
//
// Requests are one uint64 slab id per connection; the answer is a Reply,
// with the slab's dma-buf fd attached (SCM_RIGHTS) when ok.  Only processes
// of this user are answered (SO_PEERCRED).

struct Reply {
  int32_t ok;
  int32_t pad;
  uint64_t bytes;
};

void socketName(int pid, uint64_t inc, sockaddr_un* a, socklen_t* len) {
  std::memset(a, 0, sizeof(*a));
  a->sun_family = AF_UNIX;
  // abstract namespace: sun_path[0] == 0, nothing on the filesystem
  const int n = std::snprintf(a->sun_path + 1, sizeof(a->sun_path) - 1, "gloo_amd_vmm/%d/%016llx", pid,
                              (unsigned long long)inc);
  *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + (size_t)n);
}

void serveConnection(int c) {
  timeval tv{5, 0};
  (void)setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  ucred cred;
  socklen_t cl = sizeof(cred);
  if (getsockopt(c, SOL_SOCKET, SO_PEERCRED, &cred, &cl) != 0 || cred.uid != ::getuid()) return;
  uint64_t id = 0;
  if (::recv(c, &id, sizeof(id), MSG_WAITALL) != (ssize_t)sizeof(id)) return;
  Reply r{0, 0, 0};
  int fd = -1;
  {
    Pool& p = Pool::get();
    std::lock_guard<std::mutex> lk(p.m);
    for (const auto& s : p.slabs)
      if (s->id == id) {
        fd = s->fd;
        r.ok = 1;
        r.bytes = s->bytes;
      }
    auto e = p.exports.find(id);
    if (e != p.exports.end()) {
      fd = e->second.fd;
      r.ok = 1;
      r.bytes = e->second.bytes;
    }
    // a duplicate taken under the lock: an export may be closed
    // (unexportRange) while the reply is on its way
    if (fd >= 0) fd = ::fcntl(fd, F_DUPFD_CLOEXEC, 0);
    if (fd < 0) r.ok = 0;
  }
  iovec iov{&r, sizeof(r)};
  msghdr h;
  std::memset(&h, 0, sizeof(h));
  h.msg_iov = &iov;
  h.msg_iovlen = 1;
  alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int))];
  if (fd >= 0) {
    h.msg_control = ctl;
    h.msg_controllen = sizeof(ctl);
    cmsghdr* cm = CMSG_FIRSTHDR(&h);
    cm->cmsg_level = SOL_SOCKET;
    cm->cmsg_type = SCM_RIGHTS;
    cm->cmsg_len = CMSG_LEN(sizeof(int));
    std::memcpy(CMSG_DATA(cm), &fd, sizeof(fd));
  }
  (void)::sendmsg(c, &h, MSG_NOSIGNAL);
  if (fd >= 0) ::close(fd);
}

std::mutex& serverMutex() {
  static std::mutex m;
  return m;
}
int g_serverPid = 0;

// Starts this process's fd server (again after a fork).
void ensureServer() {
  std::lock_guard<std::mutex> lk(serverMutex());
  if (g_serverPid == ::getpid()) return;
  const int s = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  GLOO_AMD_ENFORCE(s >= 0, "fd server: socket() failed: ", std::strerror(errno));
  sockaddr_un a;
  socklen_t len;
  socketName(::getpid(), incarnation(), &a, &len);
  if (::bind(s, reinterpret_cast<sockaddr*>(&a), len) != 0 || ::listen(s, 128) != 0) {
    const int e = errno;
    ::close(s);
    GLOO_AMD_ENFORCE(false, "fd server: bind/listen failed: ", std::strerror(e));
  }
  std::thread([s] {
    for (;;) {
      const int c = ::accept4(s, nullptr, nullptr, SOCK_CLOEXEC);
      if (c < 0) {
        if (errno == EINTR || errno == ECONNABORTED) continue;
        return;
      }
      serveConnection(c);
      ::close(c);
    }
  }).detach();
  g_serverPid = ::getpid();
}

// The dma-buf fd of slab `id` of process (pid, inc); its size class in *bytes.
int fetchFd(int pid, uint64_t inc, uint64_t id, size_t* bytes) {
  sockaddr_un a;
  socklen_t len;
  socketName(pid, inc, &a, &len);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(30);
  int c = -1;
  for (;;) {
    c = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    GLOO_AMD_ENFORCE(c >= 0, "fd client: socket() failed: ", std::strerror(errno));
    if (::connect(c, reinterpret_cast<sockaddr*>(&a), len) == 0) break;
    const int e = errno;
    ::close(c);
    GLOO_AMD_ENFORCE(std::chrono::steady_clock::now() < deadline, "no fd server of pid ", pid, ": ",
                     std::strerror(e));
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  timeval tv{30, 0};
  (void)setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  const bool sent = ::send(c, &id, sizeof(id), MSG_NOSIGNAL) == (ssize_t)sizeof(id);
  Reply r{0, 0, 0};
  iovec iov{&r, sizeof(r)};
  msghdr h;
  std::memset(&h, 0, sizeof(h));
  h.msg_iov = &iov;
  h.msg_iovlen = 1;
  alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int))];
  h.msg_control = ctl;
  h.msg_controllen = sizeof(ctl);
  const ssize_t got = sent ? ::recvmsg(c, &h, MSG_WAITALL | MSG_CMSG_CLOEXEC) : -1;
  int fd = -1;
  if (got == (ssize_t)sizeof(r))
    for (cmsghdr* cm = CMSG_FIRSTHDR(&h); cm; cm = CMSG_NXTHDR(&h, cm))
      if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) std::memcpy(&fd, CMSG_DATA(cm), sizeof(int));
  ::close(c);
  if (got != (ssize_t)sizeof(r) || !r.ok || fd < 0) {
    if (fd >= 0) ::close(fd);
    GLOO_AMD_ENFORCE(false, "pid ", pid, " did not hand over its slab ", id, " (", got != (ssize_t)sizeof(r) ? "no reply" : "unknown slab", ")");
  }
  *bytes = r.bytes;
  return fd;
}

// The device the caller runs on, restored on scope exit.
struct DeviceScope {
  explicit DeviceScope(int device) {
    GLOO_AMD_HIP_CHECK(hipGetDevice(&prev));
    if (device != prev) GLOO_AMD_HIP_CHECK(hipSetDevice(device));
  }
  ~DeviceScope() { (void)hipSetDevice(prev); }
  int prev = 0;
};

// The imported handle of dma-buf `fd` (hipMemImportFromShareableHandle; the
// fd by value on HIP 7.2, by address on 7.0: runtimeVersion()); the fd is
// closed unless the runtime already did (only while it still
// names this dma-buf).
hipError_t importFd(int fd, hipMemGenericAllocationHandle_t* h) {
  int fdv = fd;
  void* osHandle = runtimeVersion() >= 70200000 ? reinterpret_cast<void*>(static_cast<intptr_t>(fd))
                                                : static_cast<void*>(&fdv);
  struct stat before;
  const bool known = ::fstat(fd, &before) == 0;
  const hipError_t e = hipMemImportFromShareableHandle(h, osHandle, hipMemHandleTypePosixFileDescriptor);
  struct stat after;
  if (known && ::fstat(fd, &after) == 0 && after.st_dev == before.st_dev && after.st_ino == before.st_ino)
    ::close(fd);
  return e;
}

// At process exit, before the HIP runtime tears down (atexit handlers run in
// reverse order of registration, and this one is registered after the
// runtime's first use): unmap and release every mapping and slab, so the
// runtime never finds VMM mappings of its own allocations or imports alive.
void releaseAllAtExit() {
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  for (auto& kv : p.imports) {
    (void)hipMemUnmap(kv.second.ptr, kv.second.bytes);
    (void)hipMemRelease(kv.second.handle);
  }
  for (auto& s : p.slabs) {
    (void)hipMemUnmap(s->ptr, s->bytes);
    (void)hipMemRelease(s->handle);
    if (s->fd >= 0) ::close(s->fd);
  }
  for (auto& kv : p.exports) ::close(kv.second.fd);
  p.exports.clear();
}
void registerAtExit() {
  static std::once_flag once;
  std::call_once(once, [] { std::atexit(releaseAllAtExit); });
}

}  // namespace

uint64_t incarnation() {
  static const uint64_t v = [] {
    std::random_device rd;
    return ((uint64_t)rd() << 32 ^ rd()) ^ ((uint64_t)::getpid() << 17) ^ 0x9e3779b97f4a7c15ull;
  }();
  return v;
}

int runtimeVersion() {
  static const int v = [] {
    int version = 0;
    if (hipRuntimeGetVersion(&version) != hipSuccess) (void)hipGetLastError();
    return version;
  }();
  return v;
}

Remote describe(const Slab& s) {
  Remote r;
  r.pid = (int)::getpid();
  r.incarnation = incarnation();
  r.id = s.id;
  return r;
}

Slab* acquire(int device, size_t bytes, bool fine) {
  const size_t want = sizeClass(bytes);
  ensureServer();
  registerAtExit();
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  // Best fit: the smallest free slab of this device and kind that
  // holds the request.  Slabs are never freed (ipc.h), so a request of a
  // class never used before is served from a larger idle one before a new
  // one is created; peers map the whole slab (an import accepts any slab of
  // at least the published bytes).
  size_t best = p.free.size();
  for (size_t i = 0; i < p.free.size(); i++) {
    const Slab* s = p.free[i];
    if (s->device == device && s->fine == fine && s->bytes >= bytes &&
        (best == p.free.size() || s->bytes < p.free[best]->bytes))
      best = i;
  }
  if (best < p.free.size()) {
    Slab* s = p.free[best];
    p.free.erase(p.free.begin() + (long)best);
    return s;
  }
  DeviceScope ds(device);
  auto s = std::make_unique<Slab>();
  s->bytes = want;
  s->device = device;
  s->fine = fine;
  const hipMemAllocationProp prop = propFor(device, fine);
  const hipError_t ce = hipMemCreate(&s->handle, want, &prop, 0);
  if (ce == hipErrorOutOfMemory || ce == hipErrorMemoryAllocation) {
    (void)hipGetLastError();
    size_t held = 0, idle = 0, nidle = 0;
    for (const auto& x : p.slabs)
      if (x->device == device) held += x->bytes;
    for (const Slab* x : p.free)
      if (x->device == device) idle += x->bytes, nidle++;
    throw EnforceNotMet(strcat_("out of device memory for a ", want, "-byte cross-process slab on device ", device,
                                ": the pool holds ", held, " B there, ", idle, " B of it in ", nidle,
                                " idle slabs too small for this request, which HIP cannot return while the "
                                "process lives (gloo_amd/include/gloo_amd/ipc.h)"));
  }
  GLOO_AMD_HIP_ALLOC(ce);
  try {
    void* va = freshRange(want);
    mapAt(va, want, s->handle, device);
    s->ptr = static_cast<char*>(va);
    s->devices = device < 64 ? uint64_t(1) << device : 0;
    GLOO_AMD_HIP_CHECK(hipMemExportToShareableHandle(&s->fd, s->handle, hipMemHandleTypePosixFileDescriptor, 0));
  } catch (...) {
    if (s->ptr) (void)hipMemUnmap(s->ptr, want);
    (void)hipMemRelease(s->handle);
    throw;
  }
  s->id = p.nextId++;
  p.slabs.push_back(std::move(s));
  return p.slabs.back().get();
}

void release(Slab* s) {
  if (!s) return;
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  p.free.push_back(s);
}

namespace {
// Unmaps the imports nobody holds whose exporter has exited (they
// kept the dead peer's device memory alive until this process ended).  The
// virtual range stays reserved and is never mapped again, as on the
// pid-reuse path.  Caller holds p.m.
void dropDeadImports(Pool& p) {
  for (auto it = p.imports.begin(); it != p.imports.end();) {
    const bool dead = it->second.users == 0 && ::kill(it->first.first, 0) != 0 && errno == ESRCH;
    if (!dead) {
      ++it;
      continue;
    }
    GLOO_AMD_HIP_RELEASE(hipMemUnmap(it->second.ptr, it->second.bytes));
    GLOO_AMD_HIP_RELEASE(hipMemRelease(it->second.handle));
    p.dropped++;
    it = p.imports.erase(it);
  }
}
}  // namespace

void unimport(void* mapped) {
  if (!mapped) return;
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  for (auto& kv : p.imports)
    if (kv.second.ptr == mapped) {
      if (kv.second.users) kv.second.users--;
      break;  // kept for reuse while its exporter lives (ipc.h)
    }
  dropDeadImports(p);
}

void* import(const Remote& r, size_t bytes, int device) {
  Pool& p = Pool::get();
  registerAtExit();
  const auto key = std::make_pair(r.pid, r.id);
  {
    std::lock_guard<std::mutex> lk(p.m);
    dropDeadImports(p);
    auto it = p.imports.find(key);
    if (it != p.imports.end()) {
      if (it->second.incarnation == r.incarnation) {
        GLOO_AMD_ENFORCE(it->second.bytes >= bytes, "slab of pid ", r.pid, " mapped at ", it->second.bytes,
                         " B, now published at ", bytes, " B");
        // an executor of this process on another GPU reuses the mapping
        const uint64_t bit = device < 64 ? uint64_t(1) << device : 0;
        if (bit && !(it->second.devices & bit)) {
          GLOO_AMD_HIP_CHECK(allowAccess(it->second.ptr, it->second.bytes, device));
          it->second.devices |= bit;
        }
        it->second.users++;
        return it->second.ptr;
      }
      // a new process reusing a dead one's pid: its mapping is of no use (the
      // range stays reserved, never mapped again)
      GLOO_AMD_HIP_RELEASE(hipMemUnmap(it->second.ptr, it->second.bytes));
      GLOO_AMD_HIP_RELEASE(hipMemRelease(it->second.handle));
      p.dropped++;
      p.imports.erase(it);
    }
  }
  // The pool's lock is NOT held across the request: the exporter may be
  // importing from this process at the same moment, and its request is
  // answered by this process's fd server, which takes the lock.
  size_t slabBytes = 0;
  const int fd = fetchFd(r.pid, r.incarnation, r.id, &slabBytes);
  GLOO_AMD_ENFORCE(slabBytes >= bytes, "slab ", r.id, " of pid ", r.pid, " holds ", slabBytes, " B, ", bytes,
                   " B expected");
  DeviceScope ds(device);
  hipMemGenericAllocationHandle_t h = nullptr;
  // HIP 7.2 takes the fd by value (as CUDA does); HIP 7.0.51831, the runtime
  // PyTorch 2.10+rocm7.0 bundles, takes its address and crashes on the value
  // (tools/vmm_probe, profiles/round5/r5j_vmm_torch_*).  The import does not
  // take the descriptor over (the dma-buf stays referenced by the mapping):
  // importFd closes it unless the runtime already did — and a number the
  // runtime closed may already name another thread's file (an fd server's
  // accepted socket), so only while it still names this dma-buf.
  GLOO_AMD_HIP_ALLOC(importFd(fd, &h));
  void* va = nullptr;
  try {
    va = freshRange(slabBytes);
    mapAt(va, slabBytes, h, device);
  } catch (...) {
    (void)hipMemRelease(h);
    throw;
  }
  std::lock_guard<std::mutex> lk(p.m);
  auto it = p.imports.find(key);
  if (it != p.imports.end() && it->second.incarnation == r.incarnation) {
    // another thread of this process mapped it meanwhile: keep that one
    GLOO_AMD_HIP_RELEASE(hipMemUnmap(va, slabBytes));
    GLOO_AMD_HIP_RELEASE(hipMemRelease(h));
    const uint64_t bit = device < 64 ? uint64_t(1) << device : 0;
    if (bit && !(it->second.devices & bit)) {
      GLOO_AMD_HIP_CHECK(allowAccess(it->second.ptr, it->second.bytes, device));
      it->second.devices |= bit;
    }
    it->second.users++;
    return it->second.ptr;
  }
  p.opens++;
  p.imports[key] = {r.incarnation, va, slabBytes, 1, h, device < 64 ? uint64_t(1) << device : 0};
  return va;
}

void grantAccess(void* mapped, int device) {
  if (!mapped) return;
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  const uint64_t bit = device < 64 ? uint64_t(1) << device : 0;
  for (auto& s : p.slabs)
    if (s->ptr == mapped) {
      if (bit && !(s->devices & bit)) {
        GLOO_AMD_HIP_CHECK(allowAccess(s->ptr, s->bytes, device));
        s->devices |= bit;
      }
      return;
    }
  for (auto& kv : p.imports)
    if (kv.second.ptr == mapped) {
      if (bit && !(kv.second.devices & bit)) {
        GLOO_AMD_HIP_CHECK(allowAccess(kv.second.ptr, kv.second.bytes, device));
        kv.second.devices |= bit;
      }
      return;
    }
}

namespace {
// hsa_amd_portable_export_dmabuf of the HSA runtime the HIP runtime loaded
// (the system ROCm's, or the one PyTorch bundles): found by soname, never
// loaded by us.
using ExportDmabufFn = int (*)(const void*, size_t, int*, uint64_t*);
ExportDmabufFn exportDmabuf() {
  static const ExportDmabufFn f = [] {
    void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("libhsa-runtime64.so", RTLD_NOW | RTLD_NOLOAD);
    return h ? reinterpret_cast<ExportDmabufFn>(dlsym(h, "hsa_amd_portable_export_dmabuf")) : nullptr;
  }();
  return f;
}

}  // namespace

bool exportRange(const void* ptr, size_t bytes, RangeExport* out) {
  ExportDmabufFn f = exportDmabuf();
  if (!f || !ptr || !bytes) return false;
  int fd = -1;
  uint64_t off = 0;
  if (f(ptr, bytes, &fd, &off) != 0 || fd < 0) return false;
  ensureServer();
  registerAtExit();
  const off_t end = ::lseek(fd, 0, SEEK_END);  // a dma-buf's size
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  out->id = p.nextId++;
  out->offset = off;
  out->bytes = bytes;
  p.exports[out->id] = {fd, end > 0 ? (uint64_t)end : off + bytes};
  return true;
}

void unexportRange(const RangeExport& e) {
  if (!e.id) return;
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  auto it = p.exports.find(e.id);
  if (it == p.exports.end()) return;
  ::close(it->second.fd);  // the peers' mappings keep the memory referenced
  p.exports.erase(it);
}

RangeImport importRange(const Remote& r, uint64_t offset, size_t bytes, int device) {
  size_t bufBytes = 0;
  const int fd = fetchFd(r.pid, r.incarnation, r.id, &bufBytes);
  if (offset + bytes > bufBytes) {
    ::close(fd);
    GLOO_AMD_ENFORCE(false, "exported range ", r.id, " of pid ", r.pid, ": [", offset, ", +", bytes, ") beyond its ",
                     bufBytes, "-byte buffer");
  }
  DeviceScope ds(device);
  RangeImport m;
  GLOO_AMD_HIP_ALLOC(importFd(fd, &m.handle));
  m.vaBytes = (offset + bytes + kGranule - 1) / kGranule * kGranule;
  if (m.vaBytes > bufBytes) m.vaBytes = (offset + bytes + 4095) / 4096 * 4096;  // a small allocation's dma-buf
  try {
    m.va = freshRange(m.vaBytes);
    mapAt(m.va, m.vaBytes, m.handle, device);
  } catch (...) {
    (void)hipMemRelease(m.handle);
    throw;
  }
  m.ptr = static_cast<char*>(m.va) + offset;
  return m;
}

void unimportRange(RangeImport* m) {
  if (!m || !m->va) return;
  GLOO_AMD_HIP_RELEASE(hipMemUnmap(m->va, m->vaBytes));
  GLOO_AMD_HIP_RELEASE(hipMemRelease(m->handle));
  // the range stays reserved: never mapped again (ipc.h)
  *m = RangeImport();
}

Stats stats() {
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  Stats s;
  s.slabs = p.slabs.size();
  for (const auto& x : p.slabs) s.slabBytes += x->bytes;
  s.free = p.free.size();
  s.imports = p.imports.size();
  s.opens = p.opens;
  s.dropped = p.dropped;
  return s;
}

}  // namespace ipc
}  // namespace gloo_amd

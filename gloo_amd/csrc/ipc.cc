// ipc.cc — see gloo_amd/ipc.h.
#include "gloo_amd/ipc.h"

#include <errno.h>
#include <sys/socket.h>
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
  static const bool exact = [] {
    const char* e = std::getenv("GLOO_AMD_IPC_EXACT");
    return e && e[0] == '1';
  }();
  if (exact) return (bytes + kGranule - 1) / kGranule * kGranule;
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
  std::vector<std::unique_ptr<Slab>> slabs;  // every live exported slab (freed only by a trim)
  std::vector<Slab*> free;
  uint64_t nextId = 1;
  struct Mapping {
    uint64_t incarnation;
    void* ptr;
    size_t bytes;
    size_t users;  // executors holding it (import / unimport)
    hipMemGenericAllocationHandle_t handle;  // VMM (nullptr: a hipIpc mapping)
  };
  // (exporter pid, slab id (VMM) or exporter address (hipIpc))
  std::map<std::pair<int, uint64_t>, Mapping> imports;
  // hipIpc: device -> [start, end) of every slab a trim freed: no later slab
  // may overlap one (the runtime hands out pieces of freed blocks again; an
  // export over such memory failed, and a peer's import of it showed stale
  // pages, profiles/round4/r4d_*, r4e_*)
  std::map<int, std::map<uintptr_t, uintptr_t>> retiredRanges;
  size_t opens = 0, trims = 0, trimmedBytes = 0, closes = 0, retired = 0, parked = 0;
  static Pool& get() {
    static Pool* p = new Pool();  // never destroyed: process exit releases device memory
    return *p;
  }
};

// GLOO_AMD_IPC_POOL_MAX: bytes of exported slabs per process (suffix K, M
// or G); an executor whose slabs would take a rank's pool past it trims
// collectively first (executor.cc).  Default 16 GiB.
size_t poolMax() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_IPC_POOL_MAX");
    if (!e || !*e) return size_t(16) << 30;
    char* end = nullptr;
    const double x = std::strtod(e, &end);
    size_t mul = 1;
    if (end && (*end == 'K' || *end == 'k')) mul = size_t(1) << 10;
    if (end && (*end == 'M' || *end == 'm')) mul = size_t(1) << 20;
    if (end && (*end == 'G' || *end == 'g')) mul = size_t(1) << 30;
    return (size_t)(x * (double)mul);
  }();
  return v;
}

bool overlapsRetired(const Pool& p, int device, const void* ptr, size_t bytes) {
  auto d = p.retiredRanges.find(device);
  if (d == p.retiredRanges.end()) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr), b = a + bytes;
  auto it = d->second.upper_bound(a);  // first range starting after a
  if (it != d->second.end() && it->first < b) return true;
  if (it != d->second.begin()) {
    --it;
    if (it->second > a) return true;
  }
  return false;
}

// ---- the fd server (VMM) -----------------------------------------------------
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

// Closes every mapping of a peer slab that no executor holds; p.m held.
void closeUnusedLocked(Pool& p) {
  for (auto it = p.imports.begin(); it != p.imports.end();) {
    Pool::Mapping& mp = it->second;
    // VMM mappings stay: their memory would only come back with their virtual
    // range, and a freed range handed out again showed stale pages (ipc.h)
    if (mp.users == 0 && !mp.handle) {
      GLOO_AMD_HIP_RELEASE(hipIpcCloseMemHandle(mp.ptr));
      p.closes++;
      it = p.imports.erase(it);
    } else {
      ++it;
    }
  }
}

// Frees every free-listed hipIpc slab and retires its address range; p.m
// held.  A slab is free-listed only after its executor's collective tear-down
// barrier (no peer writes it any more), and the trims that call this are
// collective: every peer has closed the mappings no executor holds first
// (ROCm 7 fails the next hipIpc export of memory allocated over a slab freed
// while a peer still mapped it, profiles/round4/r4e_*).  VMM slabs stay.
void freeUnusedLocked(Pool& p) {
  std::vector<Slab*> keep;
  for (Slab* s : p.free) {
    if (s->handle) {  // VMM: kept for reuse (see closeUnusedLocked)
      keep.push_back(s);
      continue;
    }
    for (size_t i = 0; i < p.slabs.size(); i++)
      if (p.slabs[i].get() == s) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(s->device);
        GLOO_AMD_HIP_RELEASE(hipFree(s->ptr));
        if (prev >= 0) (void)hipSetDevice(prev);
        p.retiredRanges[s->device][reinterpret_cast<uintptr_t>(s->ptr)] = reinterpret_cast<uintptr_t>(s->ptr) + s->bytes;
        p.retired++;
        p.trimmedBytes += s->bytes;
        p.slabs.erase(p.slabs.begin() + (long)i);
        break;
      }
  }
  p.free = keep;
  p.trims++;
}

size_t slabBytesLocked(const Pool& p) {
  size_t b = 0;
  for (const auto& x : p.slabs) b += x->bytes;
  return b;
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

// At process exit, before the HIP runtime tears down (atexit handlers run in
// reverse order of registration, and this one is registered after the
// runtime's first use): unmap and release every mapping and slab, so the
// runtime never finds VMM mappings of its own allocations or imports alive.
void releaseAllAtExit() {
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  for (auto& kv : p.imports)
    if (kv.second.handle) {
      (void)hipMemUnmap(kv.second.ptr, kv.second.bytes);
      (void)hipMemRelease(kv.second.handle);
    }
  for (auto& s : p.slabs)
    if (s->handle) {
      (void)hipMemUnmap(s->ptr, s->bytes);
      (void)hipMemRelease(s->handle);
      if (s->fd >= 0) ::close(s->fd);
    }
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

bool vmm() {
  static const bool v = [] {
    const char* e = std::getenv("GLOO_AMD_IPC");
    return !(e && std::string(e) == "hipipc");
  }();
  return v;
}

size_t maxSlabBytes() {
  // hipIpc: imports of 2^31 bytes and more hang (profiles/round3/r3t_*); the
  // size classes above 1 GiB are multiples of 256 MiB, so 1.75 GiB
  return vmm() ? ~size_t(0) : size_t(7) << 28;
}

Remote describe(const Slab& s) {
  Remote r;
  r.pid = (int)::getpid();
  r.incarnation = incarnation();
  r.id = s.id;
  r.ptr = reinterpret_cast<uint64_t>(s.ptr);
  r.ipcHandle = s.ipcHandle;
  return r;
}

Slab* acquire(int device, size_t bytes, bool fine) {
  const size_t want = sizeClass(bytes);
  GLOO_AMD_ENFORCE(want <= maxSlabBytes(), "a cross-process block of ", want, " B: HIP IPC imports of 2 GiB and more ",
                   "hang on this HIP runtime, so at most ", maxSlabBytes(), " B can be shared (the VMM mechanism of HIP ",
                   "7.2 and later has no such limit: ipc.h)");
  if (vmm()) {
    ensureServer();
    registerAtExit();
  }
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  for (size_t i = 0; i < p.free.size(); i++) {
    Slab* s = p.free[i];
    if (s->device == device && s->fine == fine && s->bytes == want) {
      p.free.erase(p.free.begin() + (long)i);
      return s;
    }
  }
  DeviceScope ds(device);
  auto s = std::make_unique<Slab>();
  s->bytes = want;
  s->device = device;
  s->fine = fine;
  if (vmm()) {
    const hipMemAllocationProp prop = propFor(device, fine);
    GLOO_AMD_HIP_ALLOC(hipMemCreate(&s->handle, want, &prop, 0));
    try {
      void* va = freshRange(want);
      mapAt(va, want, s->handle, device);
      s->ptr = static_cast<char*>(va);
      GLOO_AMD_HIP_CHECK(hipMemExportToShareableHandle(&s->fd, s->handle, hipMemHandleTypePosixFileDescriptor, 0));
    } catch (...) {
      if (s->ptr) (void)hipMemUnmap(s->ptr, want);
      (void)hipMemRelease(s->handle);
      throw;
    }
  } else {
    // Never export memory overlapping a retired slab, and never keep a block
    // the runtime refuses to export: park it (allocated, not exported) and
    // allocate again while it is held, then free the parked blocks.
    std::vector<void*> parked;
    void* ptr = nullptr;
    hipError_t eh = hipSuccess;
    for (;;) {
      ptr = nullptr;
      hipError_t e = fine ? hipExtMallocWithFlags(&ptr, want, hipDeviceMallocFinegrained) : hipMalloc(&ptr, want);
      if (e != hipSuccess) {
        for (void* q : parked) (void)hipFree(q);
        GLOO_AMD_HIP_ALLOC(e);
      }
      if (!overlapsRetired(p, device, ptr, want)) {
        eh = hipIpcGetMemHandle(&s->ipcHandle, ptr);
        if (eh == hipSuccess) break;
        (void)hipGetLastError();
      }
      parked.push_back(ptr);
      p.parked++;
      if (parked.size() > 64) {
        for (void* q : parked) (void)hipFree(q);
        GLOO_AMD_ENFORCE(false, "IPC pool: no exportable block of ", want, " B after 64 tries (",
                         eh == hipSuccess ? "retired ranges" : hipGetErrorString(eh), ")");
      }
    }
    for (void* q : parked) GLOO_AMD_HIP_RELEASE(hipFree(q));
    s->ptr = static_cast<char*>(ptr);
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

void unimport(void* mapped) {
  if (!mapped) return;
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  for (auto& kv : p.imports)
    if (kv.second.ptr == mapped) {
      if (kv.second.users) kv.second.users--;
      return;  // kept until a trim
    }
}

void closeUnusedImports() {
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  closeUnusedLocked(p);
}

void freeUnusedSlabs() {
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  freeUnusedLocked(p);
}

bool overCeiling(size_t more) {
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  // VMM slabs are never released (closeUnusedLocked): nothing to trim
  return !vmm() && !p.free.empty() && slabBytesLocked(p) + more > poolMax();
}

namespace {
// Drops a mapping of either kind; p.m held.
void dropMapping(Pool& p, Pool::Mapping& mp) {
  if (mp.handle) {
    GLOO_AMD_HIP_RELEASE(hipMemUnmap(mp.ptr, mp.bytes));
    GLOO_AMD_HIP_RELEASE(hipMemRelease(mp.handle));
    p.retired++;
  } else {
    GLOO_AMD_HIP_RELEASE(hipIpcCloseMemHandle(mp.ptr));
  }
}

// Bytes the runtime maps from `m` to the end of its allocation (a hipIpc
// import spans the exporter's whole slab), or 0 when it keeps no record.
size_t mappedSpan(void* m) {
  void* rb = nullptr;
  size_t rs = 0;
  size_t span = 0;
  if (hipMemGetAddressRange(&rb, &rs, m) == hipSuccess && rb && static_cast<char*>(rb) + rs > static_cast<char*>(m))
    span = (size_t)(static_cast<char*>(rb) + rs - static_cast<char*>(m));
  (void)hipGetLastError();
  return span;
}
}  // namespace

void* import(const Remote& r, size_t bytes, int device) {
  Pool& p = Pool::get();
  const bool viaVmm = vmm();
  if (viaVmm) registerAtExit();
  const auto key = std::make_pair(r.pid, viaVmm ? r.id : r.ptr);
  {
    std::lock_guard<std::mutex> lk(p.m);
    auto it = p.imports.find(key);
    if (it != p.imports.end()) {
      if (it->second.incarnation == r.incarnation) {
        if (!viaVmm && it->second.bytes < bytes) it->second.bytes = std::max(it->second.bytes, mappedSpan(it->second.ptr));
        GLOO_AMD_ENFORCE(it->second.bytes >= bytes, "slab of pid ", r.pid, " mapped at ", it->second.bytes,
                         " B, now published at ", bytes, " B");
        it->second.users++;
        return it->second.ptr;
      }
      // a new process reusing a dead one's pid: its mapping is of no use
      dropMapping(p, it->second);
      p.imports.erase(it);
    }
    if (!viaVmm) {
      void* m = nullptr;
      DeviceScope ds(device);
      GLOO_AMD_HIP_ALLOC(hipIpcOpenMemHandle(&m, r.ipcHandle, hipIpcMemLazyEnablePeerAccess));
      p.opens++;
      // the mapping spans the exporter's whole slab (its size class), not
      // just what this first importer asked for
      p.imports[key] = {r.incarnation, m, std::max(bytes, mappedSpan(m)), 1, nullptr};
      return m;
    }
  }
  // VMM.  The pool's lock is NOT held across the request: the exporter may be
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
  // (tools/vmm_probe, profiles/round5/r5j_vmm_torch_*)
  int fdv = fd;
  void* osHandle = runtimeVersion() >= 70200000 ? reinterpret_cast<void*>(static_cast<intptr_t>(fd))
                                                : static_cast<void*>(&fdv);
  const hipError_t e = hipMemImportFromShareableHandle(&h, osHandle, hipMemHandleTypePosixFileDescriptor);
  ::close(fd);
  GLOO_AMD_HIP_ALLOC(e);
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
    p.retired++;
    it->second.users++;
    return it->second.ptr;
  }
  p.opens++;
  p.imports[key] = {r.incarnation, va, slabBytes, 1, h};
  return va;
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
  s.trims = p.trims;
  s.trimmedBytes = p.trimmedBytes;
  s.closes = p.closes;
  s.retired = p.retired;
  s.parked = p.parked;
  s.max = poolMax();
  s.vmm = vmm() ? 1 : 0;
  return s;
}

}  // namespace ipc
}  // namespace gloo_amd

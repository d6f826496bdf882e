// ipc.cc — see gloo_amd/ipc.h.
#include "gloo_amd/ipc.h"

#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
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
  // powers of two up to 1 GiB, then multiples of 256 MiB: a 1.5 GiB arena
  // stays below 2^31 bytes (importing blocks of 2 GiB and more concurrently
  // hangs: executor.cc)
  constexpr size_t kBig = size_t(1) << 30, kStep = size_t(256) << 20;
  if (bytes > kBig) return (bytes + kStep - 1) / kStep * kStep;
  size_t c = kGranule;
  while (c < bytes) c <<= 1;
  return c;
}

struct Pool {
  std::mutex m;
  std::vector<std::unique_ptr<Slab>> slabs;  // every live exported slab (freed only by a trim)
  std::vector<Slab*> free;
  // device -> [start, end) of every slab a trim freed: no later slab may
  // overlap one (the runtime caches freed blocks and hands out pieces of
  // them again; an export over such memory failed, and a peer's import of
  // it showed stale pages, profiles/round4/r4d_*, r4e_*)
  std::map<int, std::map<uintptr_t, uintptr_t>> retired;
  size_t retiredCount = 0;
  struct Mapping {
    uint64_t incarnation;
    void* ptr;
    size_t bytes;
    size_t users;  // executors holding it (import / unimport)
  };
  std::map<std::pair<int, uint64_t>, Mapping> imports;  // (pid, exporter address)
  size_t opens = 0, trims = 0, trimmedBytes = 0, closes = 0, parked = 0;
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

// Closes every mapping of a peer slab that no executor holds; p.m held.
void closeUnusedLocked(Pool& p) {
  for (auto it = p.imports.begin(); it != p.imports.end();) {
    if (it->second.users == 0) {
      GLOO_AMD_HIP_RELEASE(hipIpcCloseMemHandle(it->second.ptr));
      p.closes++;
      it = p.imports.erase(it);
    } else {
      ++it;
    }
  }
}

// Frees every free-listed slab and retires its address; p.m held.  A slab is
// free-listed only after its executor's collective tear-down barrier (no
// peer writes it any more); the address is retired so that no later slab of
// this process is exported there, and a byte-identical handle keeps meaning
// the same pages.  Freeing a slab a peer still maps is not safe on ROCm 7:
// the next export of memory allocated over it can fail ("invalid argument",
// profiles/round4/r4e_*), so callers free only after every peer has closed
// its unused mappings (the collective trims of executor.cc and
// gloo_hip_ipc_trim).
void freeUnusedLocked(Pool& p) {
  for (Slab* s : p.free) {
    for (size_t i = 0; i < p.slabs.size(); i++)
      if (p.slabs[i].get() == s) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(s->device);
        GLOO_AMD_HIP_RELEASE(hipFree(s->ptr));
        if (prev >= 0) (void)hipSetDevice(prev);
        p.retired[s->device][reinterpret_cast<uintptr_t>(s->ptr)] = reinterpret_cast<uintptr_t>(s->ptr) + s->bytes;
        p.retiredCount++;
        p.trimmedBytes += s->bytes;
        p.slabs.erase(p.slabs.begin() + (long)i);
        break;
      }
  }
  p.free.clear();
  p.trims++;
}

bool overlapsRetired(const Pool& p, int device, const void* ptr, size_t bytes) {
  auto d = p.retired.find(device);
  if (d == p.retired.end()) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr), b = a + bytes;
  auto it = d->second.upper_bound(a);  // first range starting after a
  if (it != d->second.end() && it->first < b) return true;
  if (it != d->second.begin()) {
    --it;
    if (it->second > a) return true;
  }
  return false;
}

size_t slabBytesLocked(const Pool& p) {
  size_t b = 0;
  for (const auto& x : p.slabs) b += x->bytes;
  return b;
}

// Bytes the runtime maps from `m` to the end of its allocation (the
// exporter's whole slab), or 0 when it keeps no record.
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

bool poolEnabled() {
  static const bool v = [] {
    const char* e = std::getenv("GLOO_AMD_IPC_POOL");
    return !(e && e[0] == '0');
  }();
  return v;
}

uint64_t incarnation() {
  static const uint64_t v = [] {
    std::random_device rd;
    return ((uint64_t)rd() << 32 ^ rd()) ^ ((uint64_t)::getpid() << 17) ^ 0x9e3779b97f4a7c15ull;
  }();
  return v;
}

Slab* acquire(int device, size_t bytes, bool fine) {
  const size_t want = sizeClass(bytes);
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  for (size_t i = 0; poolEnabled() && i < p.free.size(); i++) {
    Slab* s = p.free[i];
    if (s->device == device && s->fine == fine && s->bytes == want) {
      p.free.erase(p.free.begin() + (long)i);
      return s;
    }
  }
  auto s = std::make_unique<Slab>();
  s->bytes = want;
  s->device = device;
  s->fine = fine;
  int prev = -1;
  GLOO_AMD_HIP_CHECK(hipGetDevice(&prev));
  GLOO_AMD_HIP_CHECK(hipSetDevice(device));
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
      (void)hipSetDevice(prev);
      GLOO_AMD_HIP_ALLOC(e);
    }
    if (!overlapsRetired(p, device, ptr, want)) {
      eh = hipIpcGetMemHandle(&s->handle, ptr);
      if (eh == hipSuccess) break;
      (void)hipGetLastError();
    }
    parked.push_back(ptr);
    p.parked++;
    if (parked.size() > 64) {
      for (void* q : parked) (void)hipFree(q);
      (void)hipSetDevice(prev);
      GLOO_AMD_ENFORCE(false, "IPC pool: no exportable block of ", want, " B after 64 tries (",
                       eh == hipSuccess ? "retired ranges" : hipGetErrorString(eh), ")");
    }
  }
  for (void* q : parked) GLOO_AMD_HIP_RELEASE(hipFree(q));
  s->ptr = static_cast<char*>(ptr);
  (void)hipSetDevice(prev);
  p.slabs.push_back(std::move(s));
  return p.slabs.back().get();
}

void release(Slab* s) {
  if (!s) return;
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  if (poolEnabled()) {
    p.free.push_back(s);
    return;
  }
  // diagnosis (GLOO_AMD_IPC_POOL=0): free at once, as before the pool
  for (size_t i = 0; i < p.slabs.size(); i++)
    if (p.slabs[i].get() == s) {
      GLOO_AMD_HIP_RELEASE(hipFree(s->ptr));
      p.slabs.erase(p.slabs.begin() + (long)i);
      return;
    }
}

void unimport(void* mapped) {
  if (!mapped) return;
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  for (auto it = p.imports.begin(); it != p.imports.end(); ++it)
    if (it->second.ptr == mapped) {
      if (it->second.users) it->second.users--;
      if (poolEnabled()) return;  // mappings of pool slabs are kept until a trim
      GLOO_AMD_HIP_RELEASE(hipIpcCloseMemHandle(mapped));
      p.imports.erase(it);
      return;
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
  return poolEnabled() && !p.free.empty() && slabBytesLocked(p) + more > poolMax();
}

void* import(int pid, uint64_t inc, uint64_t ptr, size_t bytes, const hipIpcMemHandle_t& handle) {
  Pool& p = Pool::get();
  std::lock_guard<std::mutex> lk(p.m);
  const auto key = std::make_pair(pid, ptr);
  auto it = p.imports.find(key);
  if (it != p.imports.end()) {
    if (it->second.incarnation == inc && poolEnabled()) {
      if (it->second.bytes < bytes) it->second.bytes = std::max(it->second.bytes, mappedSpan(it->second.ptr));
      GLOO_AMD_ENFORCE(it->second.bytes >= bytes, "slab of pid ", pid, " at ", (void*)ptr, " imported at ",
                       it->second.bytes, " B, now published at ", bytes, " B");
      it->second.users++;
      return it->second.ptr;
    }
    // a new process reusing a dead one's pid: its mapping is of no use
    GLOO_AMD_HIP_RELEASE(hipIpcCloseMemHandle(it->second.ptr));
    p.imports.erase(it);
  }
  void* m = nullptr;
  GLOO_AMD_HIP_ALLOC(hipIpcOpenMemHandle(&m, handle, hipIpcMemLazyEnablePeerAccess));
  p.opens++;
  // The mapping spans the exporter's whole slab (its size class), not just
  // the bytes this first importer asked for: a later use of the same slab
  // (a mailbox slab reused as an arena) may publish more of it.
  p.imports[key] = {inc, m, std::max(bytes, mappedSpan(m)), 1};
  return m;
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
  s.retired = p.retiredCount;
  s.parked = p.parked;
  s.max = poolMax();
  return s;
}

}  // namespace ipc
}  // namespace gloo_amd

// executor.cc — see executor.h.
#include "gloo_amd/executor.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <deque>
#include <exception>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <thread>

#include "gloo_amd.h"
#include "gloo_amd/common.h"
#include "gloo_amd/errors.h"
#include "gloo_amd/ipc.h"
#include "gloo_amd/signal.h"

namespace gloo_amd {

namespace {

struct ArenaRecord {
  int32_t pid;
  int32_t device;
  uint64_t ptr;
  uint64_t bytes;
  uint64_t slabId;           // DEVICE workspace shared with other processes: the pool slab (ipc.h)
  int32_t host;              // HOST workspace: the arena is the shm segment `shm`
  char shm[60];
  int32_t deviceSignal;      // this rank signals with stream-ordered kernels
  int32_t hasMailbox;        // ... into device-resident mailboxes
  uint64_t mailboxPtr;
  uint64_t mailboxSlabId;
  int32_t interpSlices;      // slices this rank could run its plan in (0: no sliced interpreter)
  uint64_t nonce;            // written at the start of a DEVICE arena: the importer checks its mapping
  uint64_t mailboxNonce;     // written behind the mailbox's counters: likewise
  uint64_t incarnation;      // ipc::incarnation() of the exporting process
  uint64_t mailboxBytes;
  uint64_t slabBytes;        // size class of the arena's pool slab (ipc.h): what an import maps
  uint64_t mailboxSlabBytes; // likewise for the mailbox's slab
};
// A peer's arena record, checked for shape.
void parseArena(const std::vector<char>& v, int peer, ArenaRecord* r) {
  GLOO_AMD_ENFORCE(v.size() == sizeof(ArenaRecord), "bad arena record from rank ", peer);
  std::memcpy(r, v.data(), sizeof(*r));
}

// A value no earlier arena of this process or its peers is likely to hold.
uint64_t arenaNonce() {
  static std::atomic<uint64_t> k{0};
  static const uint64_t seed = std::random_device{}() * 0x9e3779b97f4a7c15ull ^ ((uint64_t)::getpid() << 32);
  return (seed + (++k) * 0xbf58476d1ce4e5b9ull) | 1;
}

// GLOO_AMD_IPC_DIAG=1: log every arena export / import / close to stderr and
// probe a mapping that fails its check (diagnosis of stale IPC imports).
bool ipcDiag() {
  static const bool v = [] {
    const char* e = std::getenv("GLOO_AMD_IPC_DIAG");
    return e && e[0] == '1';
  }();
  return v;
}

// GLOO_AMD_TRACE=1: construction phases to stderr (diagnosis of hangs).
bool traceOn() {
  static const bool v = [] {
    const char* e = std::getenv("GLOO_AMD_TRACE");
    return e && e[0] == '1';
  }();
  return v;
}
#define GLOO_AMD_TRACE_PHASE(...)                                                                       \
  do {                                                                                                  \
    if (traceOn()) std::fprintf(stderr, "[trace r%d inst%llu] %s\n", ctx_->rank, (unsigned long long)inst_, \
                                strcat_(__VA_ARGS__).c_str());                                          \
  } while (0)

struct DiagLog {
  std::mutex m;
  std::map<std::string, int> handles;  // handle bytes -> times opened
  std::map<void*, int> mapped;         // importer address -> times handed out
  std::map<void*, int> exported;       // own arena address -> times exported
  static DiagLog& get() {
    static DiagLog* d = new DiagLog();
    return *d;
  }
};

// The first word at p read through hipMemcpy (the runtime's record of the
// pointer) and four ways by a kernel (the GPU's page tables), plus what the
// runtime says about the pointer.
std::string diagProbe(const void* p, hipStream_t s) {
  uint64_t viaCopy = 0;
  hipError_t e1 = hipMemcpy(&viaCopy, p, sizeof(viaCopy), hipMemcpyDeviceToHost);
  uint64_t* out = nullptr;
  uint64_t k[4] = {0, 0, 0, 0};
  hipError_t e2 = hipHostMalloc(reinterpret_cast<void**>(&out), 4 * sizeof(uint64_t), hipHostMallocDefault);
  if (e2 == hipSuccess) {
    std::memset(out, 0, 4 * sizeof(uint64_t));
    e2 = launchProbe(static_cast<const uint64_t*>(p), out, s);
    if (e2 == hipSuccess) e2 = hipStreamSynchronize(s);
    std::memcpy(k, out, sizeof(k));
    (void)hipHostFree(out);
  }
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof(a));
  hipError_t e3 = hipPointerGetAttributes(&a, p);
  void* rb = nullptr;
  size_t rs = 0;
  hipError_t e4 = hipMemGetAddressRange(&rb, &rs, const_cast<void*>(p));
  (void)hipGetLastError();
  return strcat_("memcpy=", std::hex, viaCopy, " (rc ", std::dec, (int)e1, ") kernel plain/sys/nt/plain=", std::hex,
                 k[0], "/", k[1], "/", k[2], "/", k[3], " (rc ", std::dec, (int)e2, ") attr(rc ", (int)e3,
                 ") type=", (int)a.type, " dev=", a.device, " dptr=", a.devicePointer, " hptr=", a.hostPointer,
                 " flags=", a.allocationFlags, " range(rc ", (int)e4, ")=", rb, "+", rs);
}

bool mailboxesEnabled() {
  const char* e = std::getenv("GLOO_AMD_MAILBOX");
  return !(e && e[0] == '0');
}

void bumpCounter(void* p) { static_cast<std::atomic<uint64_t>*>(p)->fetch_add(1, std::memory_order_acq_rel); }

void enqueueBump(hipStream_t s, std::atomic<uint64_t>& c) {
  GLOO_AMD_HIP_CHECK(hipLaunchHostFunc(s, bumpCounter, &c));
}

void checkRc(int rc, const char* what) {
  if (rc != GLOO_HIP_OK) throw EnforceNotMet(strcat_(what, " failed (", rc, "): ", gloo_hip_last_error()));
}

// Device memmove: non-overlapping pieces, walking away from the overlap.
void deviceMove(char* dst, const char* src, size_t bytes, hipStream_t s) {
  if (bytes == 0 || dst == src) return;
  const bool overlap = (dst < src + bytes) && (src < dst + bytes);
  if (!overlap) {
    GLOO_AMD_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    return;
  }
  const size_t gap = dst < src ? (size_t)(src - dst) : (size_t)(dst - src);
  if (dst < src) {
    for (size_t off = 0; off < bytes; off += gap) {
      const size_t n = std::min(gap, bytes - off);
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(dst + off, src + off, n, hipMemcpyDeviceToDevice, s));
    }
  } else {
    for (size_t end = bytes; end > 0;) {
      const size_t n = std::min(gap, end);
      end -= n;
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(dst + end, src + end, n, hipMemcpyDeviceToDevice, s));
    }
  }
}

// Largest message whose wait / body / notify chain is fused into one launch.
size_t fuseBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_FUSE_BYTES");
    return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)(64 << 10);
  }();
  return v;
}

// Largest message below which GLOO_AMD_GRAPH=auto replays a mesh plan as a
// hipGraph (executor constructor); larger mesh plans are enqueued eagerly.
size_t graphBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_GRAPH_BYTES");
    return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)(4u << 20);
  }();
  return v;
}

// Largest message of a plan the one-launch interpreter runs (0: never).
size_t interpBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_INTERP_BYTES");
    return e ? (size_t)std::strtoull(e, nullptr, 10) : fuseBytes();
  }();
  return v;
}

// Workgroups per sliced interpreter launch: about one per this many bytes of
// the plan's largest message.
size_t sliceBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_INTERP_SLICE_BYTES");
    return e ? std::max<size_t>(1, std::strtoull(e, nullptr, 10)) : (size_t)(32 << 10);
  }();
  return v;
}

// Most bytes of the largest message per slice: above maxSlices() slices of
// sliceBytes() the slices grow up to this, so plans with messages up to
// maxSlices() x this run sliced (2 MiB with the defaults).  Measured, HD
// fp32 4 MiB per rank, 2 rank processes on one MI355X: 32 x 64 KiB slices
// 32.8 us against graph replay 40.9 us; at 8 MiB messages 128 x 64 KiB
// slices lose to graph replay (profiles/round3/r3y_latency_*).
size_t sliceCapBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_INTERP_SLICE_MAX_BYTES");
    return e ? std::max<size_t>(sliceBytes(), std::strtoull(e, nullptr, 10)) : 2 * sliceBytes();
  }();
  return v;
}

// A range of one of a rank's buffers, symbolically: output j = j, input j =
// kIn + j, the inbox arena = kArena.
struct Access {
  int buf;
  size_t off, len;
};
constexpr int kIn = 1 << 20, kArena = -1;

// The sliced form splits a plan's whole-range local steps (LOCAL_REDUCE /
// LOCAL_BCAST over [0, n)) at every boundary the other steps use in the
// user buffers, so that the pieces later steps read are exactly pieces that
// were written.  Element-wise, so the bytes are the same.
std::vector<size_t> userCuts(const Plan& plan) {
  std::set<size_t> c;
  auto add = [&](size_t off, size_t len) {
    c.insert(off);
    c.insert(off + len);
  };
  for (const Step& t : plan.steps) {
    switch (t.kind) {
      case GLOO_HIP_STEP_SEND:
      case GLOO_HIP_STEP_FOLD_SRC:
        if (!(t.flags & GLOO_HIP_SRC_ARENA)) add(t.src_off, t.length);
        break;
      case GLOO_HIP_STEP_REDUCE:
        add(t.dst_off, t.length);
        break;
      case GLOO_HIP_STEP_COPY:
        if (!(t.flags & GLOO_HIP_SRC_ARENA)) add(t.src_off, t.length);
        if (!(t.flags & GLOO_HIP_DST_ARENA)) add(t.dst_off, t.length);
        break;
      case GLOO_HIP_STEP_FOLD:
        if (!(t.flags & GLOO_HIP_DST_ARENA)) add(t.dst_off, t.length);
        break;
      default:
        break;
    }
  }
  return std::vector<size_t>(c.begin(), c.end());
}

// [off, off + len) cut at `cuts` (sorted): the (offset, length) pieces.
std::vector<std::pair<size_t, size_t>> cutRange(const std::vector<size_t>& cuts, size_t off, size_t len) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t at = off;
  for (size_t c : cuts)
    if (c > at && c < off + len) {
      out.push_back({at, c - at});
      at = c;
    }
  if (off + len > at) out.push_back({at, off + len - at});
  return out;
}

// Can the plan run as slices (signal.h, sliced interpreter)?  Workgroup g
// handles slice g of every step and never meets the others, so every step
// must read exactly the ranges earlier steps wrote: a read overlapping an
// earlier write (a peer's message into the arena counts as one, written
// before anything) must be that same range, and a write overlapping any
// earlier access must be that same range.  Reads of data nobody wrote this
// run (the user's buffers) may overlap freely.
bool sliceable(const Plan& plan, int nin, int nout, const std::vector<Access>& remoteWrites) {
  const std::vector<size_t> cuts = userCuts(plan);
  std::map<int, std::vector<Access>> reads, writes;
  auto clash = [](const Access& a, const Access& b) {
    const bool overlap = a.off < b.off + b.len && b.off < a.off + a.len;
    return overlap && !(a.off == b.off && a.len == b.len);
  };
  auto write = [&](const Access& w) {
    if (!w.len) return true;
    for (const Access& x : reads[w.buf])
      if (clash(x, w)) return false;
    for (const Access& x : writes[w.buf])
      if (clash(x, w)) return false;
    writes[w.buf].push_back(w);
    return true;
  };
  auto read = [&](const Access& r) {
    if (!r.len) return true;
    for (const Access& x : writes[r.buf])
      if (clash(x, r)) return false;
    reads[r.buf].push_back(r);
    return true;
  };
  for (const Access& w : remoteWrites)
    if (!write(w)) return false;
  auto sendBuf = [](const Step& t) {
    return t.flags & GLOO_HIP_SRC_ARENA ? kArena : t.flags & GLOO_HIP_FROM_INPUTS ? kIn : 0;
  };
  for (const Step& t : plan.steps) {
    const size_t L = t.length;
    bool ok = true;
    switch (t.kind) {
      case GLOO_HIP_STEP_SEND:
      case GLOO_HIP_STEP_FOLD_SRC:
        ok = read({sendBuf(t), t.src_off, L});
        break;
      case GLOO_HIP_STEP_REDUCE:
        ok = read({t.flags & GLOO_HIP_FROM_INPUTS ? kIn : 0, t.dst_off, L}) && read({kArena, t.src_off, L}) &&
             write({0, t.dst_off, L});
        break;
      case GLOO_HIP_STEP_COPY:
        ok = read({t.flags & GLOO_HIP_SRC_ARENA ? kArena : 0, t.src_off, L}) &&
             write({t.flags & GLOO_HIP_DST_ARENA ? kArena : 0, t.dst_off, L});
        break;
      case GLOO_HIP_STEP_FOLD:
        ok = write({t.flags & GLOO_HIP_DST_ARENA ? kArena : 0, t.dst_off, L});
        break;
      case GLOO_HIP_STEP_LOCAL_REDUCE: {
        const bool fromIn = t.flags & GLOO_HIP_FROM_INPUTS;
        for (const auto& pc : cutRange(cuts, t.dst_off, L)) {
          for (int j = 0; j < (fromIn ? nin : nout) && ok; j++)
            ok = read({(fromIn ? kIn : 0) + j, pc.first, pc.second});
          ok = ok && write({0, pc.first, pc.second});
        }
        break;
      }
      case GLOO_HIP_STEP_LOCAL_BCAST:
        for (const auto& pc : cutRange(cuts, t.dst_off, L)) {
          ok = ok && read({0, pc.first, pc.second});
          for (int j = 1; j < nout && ok; j++) ok = write({j, pc.first, pc.second});
        }
        break;
      default:
        break;
    }
    if (!ok) return false;
  }
  return true;
}

// Upper bound on the interpreter steps buildInterp() emits for the sliced
// form of `plan`: it mirrors buildInterp's pushes, with the whole-range local
// steps counted once per piece.  A plan over the device list's capacity
// (kInterpMaxSteps) must not be proposed for slicing, because a sliced plan
// has no other route (many small segments of a large new-style call).
size_t slicedInterpSteps(const Plan& plan, int nin, int nout) {
  const std::vector<size_t> cuts = userCuts(plan);
  size_t k = 0;
  for (const Step& t : plan.steps) {
    switch (t.kind) {
      case GLOO_HIP_STEP_DECL_RECV:
      case GLOO_HIP_STEP_WAIT_SEND:
      case GLOO_HIP_STEP_FOLD_SRC:
        break;
      case GLOO_HIP_STEP_LOCAL_REDUCE: {
        const size_t srcs = (size_t)std::max(1, t.flags & GLOO_HIP_FROM_INPUTS ? nin : nout);
        const size_t per =
            srcs <= GLOO_HIP_MAX_SRCS ? 1 : 1 + (srcs - GLOO_HIP_MAX_SRCS + GLOO_HIP_MAX_SRCS - 2) / (GLOO_HIP_MAX_SRCS - 1);
        k += cutRange(cuts, t.dst_off, t.length).size() * per;
        break;
      }
      case GLOO_HIP_STEP_LOCAL_BCAST:
        k += cutRange(cuts, t.dst_off, t.length).size() * (size_t)std::max(0, nout - 1);
        break;
      default:
        k += 1;
        break;
    }
  }
  return k;
}

// Most workgroups of a sliced launch (<= kMaxSlices).  Ranks that share a
// GPU each bring this many, and a slice spins until its peer slice runs, so
// the default keeps 8 ranks on one GPU co-resident.
// The environment knobs that choose which plan a collective executes
// (INTEGRATION.md §4).  They are read here and nowhere else; every rank must
// read them alike, and the "where" exchange carries them with a fingerprint
// of the plan they produce, so a rank-inconsistent choice is refused on
// every rank instead of running mismatched step lists.
struct RouteKnobs {
  bool mesh = true;      // GLOO_AMD_MESH: derived mesh plans (mesh.cc) where P allows
  bool ringMesh = true;  // GLOO_AMD_RING_MESH: ring-chunked as its mesh plan
  bool ringPipe = true;  // GLOO_AMD_RING_PIPE: ring-chunked's ring route pipelined
  int32_t bits() const { return (mesh ? 1 : 0) | (ringMesh ? 2 : 0) | (ringPipe ? 4 : 0); }
};
RouteKnobs routeKnobs() {
  auto on = [](const char* name) {
    const char* e = std::getenv(name);
    return !(e && e[0] == '0');
  };
  RouteKnobs k;
  k.mesh = on("GLOO_AMD_MESH");
  k.ringMesh = on("GLOO_AMD_RING_MESH");
  k.ringPipe = on("GLOO_AMD_RING_PIPE");
  return k;
}
std::string knobText(int32_t bits) {
  return strcat_("GLOO_AMD_MESH=", bits & 1 ? 1 : 0, " GLOO_AMD_RING_MESH=", bits & 2 ? 1 : 0,
                 " GLOO_AMD_RING_PIPE=", bits & 4 ? 1 : 0);
}

// The plan `algo` executes as, given the knobs.  A custom op is called as the
// reference calls its function: two operands at a time on the reference's own
// routes (the mesh plans fold with reverse / tree association), and its ring
// keeps the reference's literal two-inbox order.
int selectPlanAlgo(int algo, int P, bool custom, const RouteKnobs& k) {
  int planAlgo = algo;
  const bool mesh = k.mesh && P >= 2 && P <= GLOO_HIP_MAX_SRCS && !custom;
  // AllreduceRingChunked's result with mesh data movement (plan.cc
  // planRingChunkedMesh): same bytes, two all-to-all hops over every xGMI
  // link instead of 2(P-1) hops around the ring.  Halving-doubling,
  // reduce-scatter and the new-style collectives likewise run as their
  // derived mesh plans (mesh.cc).
  if (mesh && algo == GLOO_HIP_ALGO_RING_CHUNKED && k.ringMesh) planAlgo = GLOO_HIP_ALGO_RING_CHUNKED_MESH;
  if (mesh && (algo == GLOO_HIP_ALGO_HALVING_DOUBLING || algo == GLOO_HIP_ALGO_REDUCE_SCATTER || isNewStyle(algo)))
    planAlgo = algo | GLOO_HIP_ALGO_MESH;
  // Ring-chunked on its ring route (the mesh off, or P > 8): three inboxes
  // per channel, so each round reduces and forwards in one pass (plan.cc
  // planRingChunkedPipe; the reference's bytes).
  if (planAlgo == GLOO_HIP_ALGO_RING_CHUNKED && !custom && k.ringPipe) planAlgo = GLOO_HIP_ALGO_RING_CHUNKED_PIPE;
  return planAlgo;
}

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
  return h;
}
template <typename T>
uint64_t fnvOf(uint64_t h, const T& v) {
  return fnv1a(h, &v, sizeof(v));
}
// What a rank's peers depend on in its plan: every step that talks to a peer
// (its kind, peer, slot, length, and the region offset of a SEND or a
// DECL_RECV), in order.  Local steps may differ between ranks (their pointer
// counts may), so they are left out.
uint64_t exchangeHash(const Plan& p) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (const Step& s : p.steps) {
    const bool talks = s.kind == GLOO_HIP_STEP_SEND || s.kind == GLOO_HIP_STEP_DECL_RECV ||
                       s.kind == GLOO_HIP_STEP_WAIT_RECV || s.kind == GLOO_HIP_STEP_NOTIFY ||
                       s.kind == GLOO_HIP_STEP_WAIT_NOTIFY || s.kind == GLOO_HIP_STEP_WAIT_SEND;
    if (!talks) continue;
    h = fnvOf(h, s.kind);
    h = fnvOf(h, s.peer);
    h = fnvOf(h, s.slot);
    h = fnvOf(h, s.length);
    if (s.kind == GLOO_HIP_STEP_SEND || s.kind == GLOO_HIP_STEP_DECL_RECV) h = fnvOf(h, s.dst_off);
  }
  return h;
}

int maxSlices() {
  static const int v = [] {
    const char* e = std::getenv("GLOO_AMD_INTERP_MAX_SLICES");
    return e ? std::min(kMaxSlices, std::max(1, std::atoi(e))) : 32;
  }();
  return v;
}

}  // namespace

void markInterpBatches(InterpStep* v, size_t n, size_t es) {
  using Range = std::pair<const char*, const char*>;
  auto touch = [&](const InterpStep& t, std::vector<Range>* rd, std::vector<Range>* wr) {
    const size_t bytes = t.n * es;
    if (t.kind == kInterpCopy || t.kind == kInterpSend) {
      rd->push_back({t.src[0], t.src[0] + bytes});
      wr->push_back({t.dst, t.dst + bytes});
    } else if (t.kind == kInterpFold) {
      for (int j = 0; j < t.nsrc; j++) rd->push_back({t.src[j], t.src[j] + bytes});
      wr->push_back({t.dst, t.dst + bytes});
    }
  };
  auto meet = [](const std::vector<Range>& x, const std::vector<Range>& y) {
    for (const Range& a : x)
      for (const Range& b : y)
        if (a.first < b.second && b.first < a.second) return true;
    return false;
  };
  // The kernel drains only at a batch's last step, so step i+1 may join the
  // open batch only if it is independent of EVERY step already in it, not
  // just of step i: a SIGNAL touches no bytes, and a pairwise check would let
  // REDUCE, NOTIFY, SEND-from-inside-the-reduced-range (the halving-doubling
  // reduce-scatter, plan.cc) run without a drain between the fold's stores
  // and the send's loads.
  std::vector<Range> brd, bwr;  // reads and writes of the open batch
  for (size_t i = 0; i < n; i++) v[i].flags &= ~kInterpDefer;
  for (size_t i = 0; i + 1 < n; i++) {
    const InterpStep &a = v[i], &b = v[i + 1];
    if (i == 0 || !(v[i - 1].flags & kInterpDefer)) brd.clear(), bwr.clear();
    touch(a, &brd, &bwr);
    const bool aw = a.kind == kInterpWait, bw = b.kind == kInterpWait;
    bool batch = aw && bw;
    if (!aw && !bw) {
      std::vector<Range> rb, wb;
      touch(b, &rb, &wb);
      batch = !meet(bwr, rb) && !meet(bwr, wb) && !meet(brd, wb);
    }
    if (batch) v[i].flags |= kInterpDefer;
  }
}

// A pinned host-memory segment every rank of the node can map (HOST workspace).
struct PlanExecutor::HostShm {
  std::string name;
  void* host = nullptr;
  void* dev = nullptr;
  size_t bytes = 0;
  bool owner = false;

  static std::unique_ptr<HostShm> create(size_t bytes) {
    auto h = std::make_unique<HostShm>();
    std::random_device rd;
    h->name = strcat_("/gloo_amd_ws_", ::getpid(), "_", rd(), rd());
    h->bytes = bytes;
    h->owner = true;
    const int fd = ::shm_open(h->name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    GLOO_AMD_ENFORCE(fd >= 0, "shm_open(create) failed for ", h->name);
    const bool sized = ::ftruncate(fd, (off_t)bytes) == 0;
    if (sized) h->host = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (!sized || h->host == MAP_FAILED) {
      h->host = nullptr;
      ::shm_unlink(h->name.c_str());
      throw EnforceNotMet(strcat_("cannot map a ", bytes, "-byte host workspace"));
    }
    h->map();
    return h;
  }
  static std::unique_ptr<HostShm> open(const std::string& name, size_t bytes) {
    auto h = std::make_unique<HostShm>();
    h->name = name;
    h->bytes = bytes;
    const int fd = ::shm_open(name.c_str(), O_RDWR, 0600);
    GLOO_AMD_ENFORCE(fd >= 0, "shm_open failed for ", name);
    h->host = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (h->host == MAP_FAILED) {
      h->host = nullptr;
      throw EnforceNotMet(strcat_("cannot map host workspace ", name));
    }
    h->map();
    return h;
  }
  void map() {
    GLOO_AMD_HIP_ALLOC(hipHostRegister(host, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    GLOO_AMD_HIP_CHECK(hipHostGetDevicePointer(&dev, host, 0));
  }
  void unlink() {
    if (owner && !name.empty()) ::shm_unlink(name.c_str());
    owner = false;
  }
  ~HostShm() {
    if (host) {
      GLOO_AMD_HIP_RELEASE(hipHostUnregister(host));
      ::munmap(host, bytes);
    }
    unlink();
  }
};

namespace {
Plan planFor(int algo, int rank, int size, size_t count, int nin, int nout, size_t es, size_t maxSeg,
             const std::vector<int>& recvElems) {
  if (isNewStyle(algo)) {
    NewStyleOptions o;
    o.ninputs = nin;
    o.noutputs = nout;
    o.elemSize = es;
    o.maxSegmentBytes = maxSeg;
    if ((algo & ~GLOO_HIP_ALGO_MESH) == GLOO_HIP_ALGO_REDUCE) o.root = recvElems.empty() ? 0 : recvElems[0];  // {root}
    return makeNewStylePlan(algo, rank, size, count, o);
  }
  return makePlan(algo, rank, size, count, nout, recvElems);
}

// The text of a failed import check (tests and tools look for it).
constexpr const char* kStaleImport = "does not show its contents";
}  // namespace

void PlanExecutor::setBuffers(const std::vector<void*>& inputs, const std::vector<void*>& outputs) {
  GLOO_AMD_ENFORCE(inputs.size() == inputs_.size() && outputs.size() == ptrs_.size(),
                   "buffer count differs from the one the algorithm was built for");
  if (inputs != inputs_ || outputs != ptrs_) {
    dropGraph();
    stableRuns_ = 0;
    interpDirty_ = true;
  }
  inputs_ = inputs;
  ptrs_ = outputs;
  classifyPointers();
}

void PlanExecutor::setStream(hipStream_t s) {
  setStreams(s ? std::vector<hipStream_t>{s} : std::vector<hipStream_t>{});
}

void PlanExecutor::setStreams(const std::vector<hipStream_t>& streams) {
  GLOO_AMD_ENFORCE(streams.size() <= 1 || streams.size() == ptrs_.size(), "one stream per pointer: ",
                   ptrs_.size(), " pointers, ", streams.size(), " streams");
  hipStream_t next = streams.empty() ? nullptr : streams[0];
  for (hipStream_t t : streams) GLOO_AMD_ENFORCE(t != nullptr || streams.size() == 1, "null stream in the list");
  if (!next) {
    if (!ownedStream_) GLOO_AMD_HIP_CHECK(hipStreamCreateWithFlags(&ownedStream_, hipStreamNonBlocking));
    next = ownedStream_;
  }
  if (next != stream_) {
    // the new stream's work (which reuses the inboxes and this rank's
    // buffers) starts after everything queued before: a run on a caller's
    // stream left doneEvent_ behind; a run on the own stream has completed
    if (donePending_) GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(next, doneEvent_, 0));
    stream_ = next;
  }
  ownStream_ = stream_ == ownedStream_;
  sideStreams_.assign(streams.size() > 1 ? streams.begin() + 1 : streams.end(), streams.end());
  while (sideEvents_.size() < sideStreams_.size()) {
    hipEvent_t e;
    GLOO_AMD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    sideEvents_.push_back(e);
  }
}

void PlanExecutor::quiesce() {
  if (ownedStream_) (void)hipStreamSynchronize(ownedStream_);
  if (donePending_) {
    (void)hipEventSynchronize(doneEvent_);
    donePending_ = false;
  }
}

void PlanExecutor::dropGraph() {
  if (!graphExec_) return;
  quiesce();
  (void)hipGraphExecDestroy(graphExec_);
  graphExec_ = nullptr;
}

void PlanExecutor::classifyPointers() {
  const char* forced = std::getenv("GLOO_AMD_FORCE_STAGING");  // tests: stage even same-device pointers
  const bool force = forced && forced[0] == '1';
  anyRemote_ = false;  // recomputed for every buffer set (setBuffers)
  auto classify = [&](const std::vector<void*>& v, std::vector<bool>& remote, std::vector<char*>& stage,
                      size_t first) {
    remote.assign(v.size(), false);
    stage.resize(v.size(), nullptr);
    for (size_t j = first; j < v.size(); j++) {
      if (!v[j]) continue;
      hipPointerAttribute_t attr;
      int dev = ctx_->device();
      if (hipPointerGetAttributes(&attr, v[j]) == hipSuccess) dev = attr.device;
      (void)hipGetLastError();
      remote[j] = force || dev != ctx_->device();
      if (remote[j] && dev != ctx_->device()) {
        hipError_t e = hipDeviceEnablePeerAccess(dev, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) GLOO_AMD_HIP_CHECK(e);
        (void)hipGetLastError();
      }
      if (remote[j] && !stage[j]) GLOO_AMD_HIP_ALLOC(hipMalloc(&stage[j], std::max<size_t>(256, count_ * es_)));
      anyRemote_ = anyRemote_ || remote[j];
    }
  };
  classify(ptrs_, outRemote_, outStage_, 1);   // output 0 is the rank's working buffer
  classify(inputs_, inRemote_, inStage_, 0);
  // gloo::reduce reads its input in SEND / REDUCE steps, not only in the
  // staged local fold
  GLOO_AMD_ENFORCE(algo_ != GLOO_HIP_ALGO_REDUCE || inputs_.empty() || !inRemote_[0],
                   "gloo::reduce: the input must live on the rank's own device");
}

PlanExecutor::PlanExecutor(std::shared_ptr<Context> ctx, int algo, int op, int dtype,
                           const std::vector<void*>& ptrs, size_t count, const std::vector<int>& recvElems,
                           hipStream_t stream, const std::vector<void*>& inputs, size_t maxSegmentBytes,
                           int workspace)
    : ctx_(std::move(ctx)), algo_(algo), op_(op), dtype_(dtype), ptrs_(ptrs), inputs_(inputs), count_(count),
      maxSegmentBytes_(maxSegmentBytes), recvElems_(recvElems) {
  es_ = gloo_hip_dtype_size(dtype_);
  GLOO_AMD_ENFORCE(es_ > 0, "unknown dtype ", dtype_);
  {
    gloo_hip_custom_fn fn;
    void* user;
    custom_ = customOp(op_, &fn, &user);
    GLOO_AMD_ENFORCE(custom_ || isBuiltinOp(op_), "unknown op ", op_);
  }
  GLOO_AMD_ENFORCE(!ptrs_.empty(), "need at least one pointer");
  for (void* p : ptrs_) GLOO_AMD_ENFORCE(p != nullptr || count_ == 0, "null device pointer");
  const int me = ctx_->rank, P = ctx_->size;
  // The executed plan: the algorithm's, or its mesh / pipelined form
  // (selectPlanAlgo).  Every rank must choose alike; the choice depends only
  // on the route knobs and P, and the "where" exchange below checks it.
  const RouteKnobs knobs = routeKnobs();
  planAlgo_ = selectPlanAlgo(algo_, P, custom_, knobs);
  plan_ = planFor(planAlgo_, me, P, count_, (int)inputs_.size(), (int)ptrs_.size(), es_, maxSegmentBytes_,
                  recvElems_);
  GLOO_AMD_HIP_CHECK(hipSetDevice(ctx_->device()));
  classifyPointers();
  inst_ = ctx_->acquireInstance();
  GLOO_AMD_HIP_CHECK(hipSetDevice(ctx_->device()));
  GLOO_AMD_HIP_CHECK(hipEventCreateWithFlags(&doneEvent_, hipEventDisableTiming));
  if (stream) {
    stream_ = stream;
  } else {
    GLOO_AMD_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    ownedStream_ = stream_;
    ownStream_ = true;
  }
  // Baseline every channel before anyone can signal this instance (instance
  // slots of the host control block are recycled modulo kMaxLiveInstances;
  // a device mailbox is fresh, so its channels start at 0), count its
  // messages per run, and give every step its sequence number (StepSeq).
  // Runs before the ready barrier, i.e. before any peer can signal.
  auto assignSeqs = [&] {
    std::map<std::pair<int, int>, uint64_t> base, perRun, seen;
    auto isWait = [](int k) { return k == GLOO_HIP_STEP_WAIT_RECV || k == GLOO_HIP_STEP_WAIT_NOTIFY; };
    auto isSend = [](int k) { return k == GLOO_HIP_STEP_SEND || k == GLOO_HIP_STEP_NOTIFY; };
    for (const Step& s : plan_.steps) {
      if (!isWait(s.kind) && !isSend(s.kind)) continue;
      // waits count the peer->me channel, sends the me->peer one; keep the
      // two apart in the maps by the sign of the key
      const std::pair<int, int> key{isWait(s.kind) ? -1 - s.peer : s.peer, s.slot};
      if (!base.count(key))
        base[key] = mailboxWith(s.peer) ? 0
                    : isWait(s.kind)   ? ctx_->counter(inst_, s.peer, me, s.slot).load(std::memory_order_acquire)
                                       : ctx_->counter(inst_, me, s.peer, s.slot).load(std::memory_order_acquire);
      perRun[key]++;
    }
    stepSeq_.resize(plan_.steps.size());
    for (size_t i = 0; i < plan_.steps.size(); i++) {
      const Step& s = plan_.steps[i];
      if (!isWait(s.kind) && !isSend(s.kind)) continue;
      const std::pair<int, int> key{isWait(s.kind) ? -1 - s.peer : s.peer, s.slot};
      const uint64_t j = seen[key]++;
      stepSeq_[i].base = base[key] + j + 1 - perRun[key];
      // a previous-run credit: one run behind (met at once in run 1)
      if (isWait(s.kind) && (s.flags & GLOO_HIP_PREV_RUN)) stepSeq_[i].base -= perRun[key];
      stepSeq_[i].perRun = perRun[key];
    }
  };

  if (P == 1) {  // no transport: local reduce / broadcast only
    assignSeqs();
    return;
  }

  // Phase 1: who is where.  Every rank publishes (pid, device); each rank
  // reads the records of every peer its plan talks to.
  std::set<int> planPeers, sendPeers, recvPeers;
  for (const Step& s : plan_.steps) {
    const bool talks = s.kind == GLOO_HIP_STEP_SEND || s.kind == GLOO_HIP_STEP_DECL_RECV ||
                       s.kind == GLOO_HIP_STEP_WAIT_RECV || s.kind == GLOO_HIP_STEP_NOTIFY ||
                       s.kind == GLOO_HIP_STEP_WAIT_NOTIFY || s.kind == GLOO_HIP_STEP_WAIT_SEND;
    if (talks && s.peer >= 0 && s.peer != me) planPeers.insert(s.peer);
    if (s.kind == GLOO_HIP_STEP_SEND) sendPeers.insert(s.peer);
    if (s.kind == GLOO_HIP_STEP_DECL_RECV) recvPeers.insert(s.peer);
  }
  constexpr size_t kArenaGranule = 2u << 20;
  auto arenaBytesOf = [&](const Plan& p) {
    return (std::max<size_t>(256, p.arena * es_) + kArenaGranule - 1) / kArenaGranule * kArenaGranule;
  };
  // (pid, device, and the plan fingerprint: the route knobs, the executed
  // plan, the call's shape and the hash of the plan's exchange)
  struct Where {
    int32_t pid, device, knobs, planAlgo;
    uint64_t call, exchange;
  };
  const uint64_t callHash = [&] {
    uint64_t h = 0xcbf29ce484222325ull;
    h = fnvOf(h, algo_);
    h = fnvOf(h, op_);
    h = fnvOf(h, dtype_);
    h = fnvOf(h, (uint64_t)count_);
    h = fnvOf(h, (uint64_t)maxSegmentBytes_);
    for (int v : recvElems_) h = fnvOf(h, v);
    return h;
  }();
  std::vector<Where> where(P);
  {
    Where w{ctx_->pid(), ctx_->device(), knobs.bits(), planAlgo_, callHash, exchangeHash(plan_)};
    std::vector<char> blob(sizeof(w));
    std::memcpy(blob.data(), &w, sizeof(w));
    const auto all = ctx_->allgather(strcat_("inst", inst_, "/where"), blob);
    for (int r = 0; r < P; r++) {
      GLOO_AMD_ENFORCE(all.at(r).size() == sizeof(Where), "bad record from rank ", r);
      std::memcpy(&where[r], all[r].data(), sizeof(Where));
    }
  }
  GLOO_AMD_TRACE_PHASE("where exchanged");
  // Rank-consistent plans: every rank sees the same
  // records and reaches the same verdict, so an inconsistent choice raises
  // on every rank (after the collective release) instead of running step
  // lists that do not match — a hang at best, writes into regions a peer
  // never declared at worst.
  {
    std::string why;
    for (int r = 0; r < P && why.empty(); r++) {
      const Where& w = where[r];
      if (w.planAlgo != where[0].planAlgo)
        why = strcat_("rank ", r, " executes plan ", w.planAlgo, " (", knobText(w.knobs), ") but rank 0 executes plan ",
                      where[0].planAlgo, " (", knobText(where[0].knobs), ")");
      else if (w.call != where[0].call)
        why = strcat_("rank ", r, " was called with another algorithm, op, dtype, count, segment size or receive "
                      "counts than rank 0");
    }
    for (int r = 0; r < P && why.empty(); r++) {
      const Plan pr = r == me ? plan_
                              : planFor(where[r].planAlgo, r, P, count_, 0, 1, es_, maxSegmentBytes_, recvElems_);
      if (exchangeHash(pr) != where[r].exchange)
        why = strcat_("rank ", r, "'s exchange steps differ from the plan every rank derives for it");
    }
    if (!why.empty()) {
      release();
      GLOO_AMD_ENFORCE(false, "rank-inconsistent collective: ", why, ". The plan-selecting knobs (GLOO_AMD_MESH, "
                       "GLOO_AMD_RING_MESH, GLOO_AMD_RING_PIPE) and the call's arguments must be equal on every rank");
    }
  }
  peers_.resize(P);
  bool sharesDeviceInProcess = false, crossSender = false;
  for (int peer : planPeers) {
    const Where& w = where.at(peer);
    peers_[peer].pid = w.pid;
    peers_[peer].device = w.device;
    if (w.pid == ctx_->pid() && w.device == ctx_->device()) sharesDeviceInProcess = true;
    if (recvPeers.count(peer) && (w.device != ctx_->device() || w.pid != ctx_->pid())) crossSender = true;
    if (w.pid != ctx_->pid()) crossProcess_ = true;
  }
  const char* sig = std::getenv("GLOO_AMD_SIGNAL");
  const std::string sigMode = sig ? sig : "auto";
  deviceSignal_ = sigMode == "device" || (sigMode == "auto" && !sharesDeviceInProcess);
  // A peer GPU (over xGMI) or a peer PROCESS (through its own IPC mapping)
  // writes this rank's inboxes: keep them in fine-grained memory, so no
  // stale line of an L2 can be read on either side.  Measured with
  // coarse-grained inboxes and two processes on one MI355X: after an
  // executor of the same size had run, the importer read the previous
  // contents through its mapping even after a device synchronise, and a
  // ring route's messages were not seen by the receiver (bench.py
  // config-3 variants back to back, tests/test_bench_gpu.py).
  const char* ar = std::getenv("GLOO_AMD_ARENA");
  const std::string arMode = ar ? ar : "auto";
  GLOO_AMD_ENFORCE(workspace == GLOO_HIP_WORKSPACE_DEVICE || workspace == GLOO_HIP_WORKSPACE_HOST,
                   "unknown workspace ", workspace);
  hostArena_ = workspace == GLOO_HIP_WORKSPACE_HOST || arMode == "host";
  fineArena_ = !hostArena_ && (arMode == "fine" || (arMode == "auto" && crossSender));

  // Phase 2: the inbox arena.  Whole 2 MiB granules.  When a peer in
  // another process maps it, it is a slab of the process-wide pool (ipc.h):
  // a VMM block at a virtual range never mapped before, exported once as a
  // dma-buf and reused by later executors of its size class, so a mapping a
  // peer holds always shows these pages.  Any size: there is no 2 GiB import
  // limit on this route (profiles/round5/r5b_vmm_fresh_va.jsonl).
  const size_t arenaBytes = arenaBytesOf(plan_);
  arenaBytes_ = arenaBytes;
  if (hostArena_) {
    arenaShm_ = HostShm::create(arenaBytes);
    arena_ = static_cast<char*>(arenaShm_->dev);
  } else if (crossProcess_) {
    GLOO_AMD_TRACE_PHASE("acquiring a slab of ", arenaBytes, " B fine=", fineArena_);
    arenaSlab_ = ipc::acquire(ctx_->device(), arenaBytes, fineArena_);
    arena_ = arenaSlab_->ptr;
    GLOO_AMD_TRACE_PHASE("slab ", (void*)arena_, " of ", arenaSlab_->bytes, " B");
  } else if (fineArena_) {
    GLOO_AMD_HIP_ALLOC(hipExtMallocWithFlags(reinterpret_cast<void**>(&arena_), arenaBytes,
                                             hipDeviceMallocFinegrained));
  } else {
    GLOO_AMD_HIP_ALLOC(hipMalloc(&arena_, arenaBytes));
  }
  // Device-side signalling polls a mailbox in this GPU's own (fine-grained)
  // memory that the peers write over xGMI: one 64-bit counter per
  // (sender, slot).  Measured on MI355X: a cross-rank hop costs about 1 us
  // this way against about 2.4 us through the host control block
  // (tools/pingpong.cc, profiles/round1/r1q_pingpong.jsonl).  Shared with
  // other processes, it is a pool slab too, and a nonce behind the counters
  // lets every importer check its mapping.
  size_t mbBytes = 0;
  uint64_t mbNonce = 0;
  if (deviceSignal_ && mailboxesEnabled()) {
    // one word per (sender, slot, slice): slices of the sliced interpreter
    mbBytes = ((size_t)P * GLOO_HIP_NUM_SLOTS * kMaxSlices * sizeof(uint64_t) + 4095) / 4096 * 4096;
    if (crossProcess_) {
      mailboxSlab_ = ipc::acquire(ctx_->device(), mbBytes + 4096, true);
      mailbox_ = reinterpret_cast<uint64_t*>(mailboxSlab_->ptr);
    } else {
      GLOO_AMD_HIP_ALLOC(hipExtMallocWithFlags(reinterpret_cast<void**>(&mailbox_), mbBytes + 4096,
                                               hipDeviceMallocFinegrained));
    }
    GLOO_AMD_HIP_CHECK(hipMemsetAsync(mailbox_, 0, mbBytes, stream_));
    mbNonce = arenaNonce();
    GLOO_AMD_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<char*>(mailbox_) + mbBytes, &mbNonce, sizeof(mbNonce),
                                      hipMemcpyHostToDevice, stream_));
    GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  // Interpreter (executor.h): the knobs every rank reads alike, and this
  // rank's proposal for the sliced form — one workgroup per sliceBytes() of
  // its largest message, if its own plan and the messages its peers write
  // into its arena slice consistently (sliceable).  All ranks then take the
  // smallest proposal, so they agree.
  {
    const char* im = std::getenv("GLOO_AMD_INTERP");
    const char* gm = std::getenv("GLOO_AMD_GRAPH");
    interpMode_ = deviceSignal_ && !(im && std::string(im) == "0") && !(gm && std::string(gm) == "1") &&
                  interpBytes() > 0 && !custom_;
  }
  int32_t proposal = 0;
  if (interpMode_ && mailbox_ && !anyRemote_ && !hostArena_) {
    size_t maxMsg = 0;
    for (const Step& s : plan_.steps) maxMsg = std::max(maxMsg, (size_t)s.length * es_);
    const size_t want = std::min<size_t>(maxSlices(), std::max<size_t>(1, (maxMsg + sliceBytes() - 1) / sliceBytes()));
    // above maxSlices() slices of sliceCapBytes() graph replay is as fast
    if (maxMsg <= (size_t)maxSlices() * sliceCapBytes()) {
      std::map<std::pair<int, int>, size_t> decl;  // (sender, slot) -> arena offset
      for (const Step& d : plan_.steps)
        if (d.kind == GLOO_HIP_STEP_DECL_RECV) decl[{d.peer, d.slot}] = d.dst_off;
      std::vector<Access> remote;
      bool ok = true;
      for (int peer : recvPeers) {
        const Plan theirs = planFor(planAlgo_, peer, P, count_, 0, 1, es_, maxSegmentBytes_, recvElems_);
        for (const Step& t : theirs.steps)
          if (t.kind == GLOO_HIP_STEP_SEND && t.peer == me) {
            auto it = decl.find({peer, t.slot});
            if (it == decl.end()) ok = false;
            else remote.push_back({kArena, it->second + t.dst_off, t.length});
          }
      }
      if (ok && slicedInterpSteps(plan_, (int)inputs_.size(), (int)ptrs_.size()) <= (size_t)kInterpMaxSteps &&
          sliceable(plan_, (int)inputs_.size(), (int)ptrs_.size(), remote))
        proposal = (int32_t)want;
    }
  }
  ArenaRecord rec;
  std::memset(&rec, 0, sizeof(rec));
  rec.interpSlices = proposal;
  rec.pid = ctx_->pid();
  rec.device = ctx_->device();
  rec.ptr = reinterpret_cast<uint64_t>(arena_);
  rec.bytes = arenaBytes;
  rec.deviceSignal = deviceSignal_ ? 1 : 0;
  if (!hostArena_) {
    // the first 8 bytes of the arena carry a nonce until the first message
    // lands; a peer that maps the arena over IPC reads it back (below)
    rec.nonce = arenaNonce();
    GLOO_AMD_HIP_CHECK(hipMemcpyAsync(arena_, &rec.nonce, sizeof(rec.nonce), hipMemcpyHostToDevice, stream_));
    GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
    if (ipcDiag()) {
      int times;
      {
        DiagLog& d = DiagLog::get();
        std::lock_guard<std::mutex> lk(d.m);
        times = d.exported[arena_]++;
      }
      std::fprintf(stderr, "[ipc-diag %d r%d inst%llu] export arena %p %zu B fine=%d nonce %llx (exported here %d times before): %s\n",
                   ctx_->pid(), me, (unsigned long long)inst_, (void*)arena_, arenaBytes, (int)fineArena_,
                   (unsigned long long)rec.nonce, times, diagProbe(arena_, stream_).c_str());
    }
  }
  rec.incarnation = ipc::incarnation();
  if (arenaSlab_) rec.slabBytes = arenaSlab_->bytes;
  if (mailbox_) {
    rec.hasMailbox = 1;
    rec.mailboxPtr = reinterpret_cast<uint64_t>(mailbox_);
    rec.mailboxBytes = mbBytes;
    rec.mailboxNonce = mbNonce;
    if (mailboxSlab_) {
      rec.mailboxSlabId = mailboxSlab_->id;
      rec.mailboxSlabBytes = mailboxSlab_->bytes;
    }
  }
  if (hostArena_) {
    rec.host = 1;
    GLOO_AMD_ENFORCE(arenaShm_->name.size() < sizeof(rec.shm), "shm name too long");
    std::memcpy(rec.shm, arenaShm_->name.c_str(), arenaShm_->name.size() + 1);
  } else if (arenaSlab_) {
    rec.slabId = arenaSlab_->id;  // exported once, when the pool allocated the slab
  }
  std::vector<char> blob(sizeof(rec));
  std::memcpy(blob.data(), &rec, sizeof(rec));
  GLOO_AMD_TRACE_PHASE("exchanging arena records");
  const std::vector<std::vector<char>> arenas = ctx_->allgather(strcat_("inst", inst_, "/arena"), blob);
  GLOO_AMD_TRACE_PHASE("arena records exchanged");

  // From here to "ready" a rank may fail on its own (a refused IPC mapping,
  // an allocation): it still joins the ready exchange with its reason, so
  // every rank of the collective construction fails together instead of
  // its peers timing out at the barrier and the ranks falling out of step.
  std::exception_ptr setupFailure;
  std::string setupReason;
  try {

  // Every plan peer's record: its mailbox (a channel uses mailboxes when
  // both ends signal from the device and have one — both ends decide alike),
  // and, for a peer this rank sends to, its inbox arena and the region the
  // peer declared there for our messages (its own plan).
  peerMailbox_.assign(P, nullptr);
  peerMailboxIpc_.assign(P, false);
  for (int peer : planPeers) {
    ArenaRecord pr;
    parseArena(arenas.at(peer), peer, &pr);
    if (mailbox_ && pr.deviceSignal && pr.hasMailbox) {
      if (pr.pid == ctx_->pid()) {
        peerMailbox_[peer] = reinterpret_cast<uint64_t*>(pr.mailboxPtr);
        if (pr.device != ctx_->device()) {
          hipError_t e = hipDeviceEnablePeerAccess(pr.device, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) GLOO_AMD_HIP_CHECK(e);
          (void)hipGetLastError();
        }
      } else {
        ipc::Remote rm;
        rm.pid = pr.pid;
        rm.incarnation = pr.incarnation;
        rm.id = pr.mailboxSlabId;
        void* p = ipc::import(rm, pr.mailboxBytes + 4096, ctx_->device());
        uint64_t seen = 0;
        GLOO_AMD_HIP_CHECK(hipMemcpyAsync(&seen, static_cast<char*>(p) + pr.mailboxBytes, sizeof(seen),
                                          hipMemcpyDeviceToHost, stream_));
        GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
        GLOO_AMD_ENFORCE(seen == pr.mailboxNonce, "rank ", me, ": the IPC mapping of rank ", peer, "'s mailbox (",
                         (void*)pr.mailboxPtr, " in pid ", pr.pid, ", mapped at ", p, ") ", kStaleImport, ": read ",
                         seen, ", expected ", pr.mailboxNonce);
        peerMailbox_[peer] = static_cast<uint64_t*>(p);
        peerMailboxIpc_[peer] = true;
      }
    }
    if (!sendPeers.count(peer)) continue;
    if (pr.host && pr.pid != ctx_->pid()) {
      // another process's host workspace: map the same pages here
      peerShm_.push_back(HostShm::open(std::string(pr.shm), pr.bytes));
      peers_[peer].base = static_cast<char*>(peerShm_.back()->dev);
    } else if (pr.host || pr.pid == ctx_->pid()) {
      // same process: registered portable (host) or peer-accessible (device)
      peers_[peer].base = reinterpret_cast<char*>(pr.ptr);
      if (pr.device != ctx_->device()) {
        hipError_t e = hipDeviceEnablePeerAccess(pr.device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) GLOO_AMD_HIP_CHECK(e);
        (void)hipGetLastError();
      }
    } else {
      // Another process's pool slab (ipc.h): mapped once, kept.  The mapping
      // must show the nonce the owner just wrote at the slab's start, and
      // span the arena; anything else is a hard error, never a silent
      // misdelivery.
      GLOO_AMD_TRACE_PHASE("importing rank ", peer, "'s arena slab ", pr.slabId, " (", pr.bytes, " B)");
      ipc::Remote rm;
      rm.pid = pr.pid;
      rm.incarnation = pr.incarnation;
      rm.id = pr.slabId;
      void* p = ipc::import(rm, pr.bytes, ctx_->device());
      GLOO_AMD_TRACE_PHASE("imported at ", p);
      uint64_t seen = 0;
      GLOO_AMD_HIP_CHECK(hipMemcpyAsync(&seen, p, sizeof(seen), hipMemcpyDeviceToHost, stream_));
      GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
      if (ipcDiag())
        std::fprintf(stderr, "[ipc-diag %d r%d inst%llu] import rank %d arena %p %llu B (pid %d) -> %p: seen %llx "
                     "want %llx%s%s\n", ctx_->pid(), me, (unsigned long long)inst_, peer, (void*)pr.ptr,
                     (unsigned long long)pr.bytes, pr.pid, p, (unsigned long long)seen,
                     (unsigned long long)pr.nonce, seen == pr.nonce ? "" : " MISMATCH: ",
                     seen == pr.nonce ? "" : diagProbe(p, stream_).c_str());
      peers_[peer].base = static_cast<char*>(p);
      peers_[peer].ipc = true;
      // (ipc::import maps the whole slab, at least pr.bytes, or raises)
      GLOO_AMD_ENFORCE(seen == pr.nonce, "rank ", me, ": the mapping of rank ", peer, "'s inbox arena (",
                       (void*)pr.ptr, ", ", pr.bytes, " B, slab ", pr.slabId, " of pid ", pr.pid, ", mapped at ", p,
                       ") ", kStaleImport, ": read ", seen, ", expected ", pr.nonce);
    }
    const Plan theirs = planFor(planAlgo_, peer, P, count_, 0, 1, es_, maxSegmentBytes_, recvElems_);
    for (const Step& d : theirs.steps)
      if (d.kind == GLOO_HIP_STEP_DECL_RECV && d.peer == me) {
        GLOO_AMD_ENFORCE((d.dst_off + d.length) * es_ <= pr.bytes, "peer region outside its arena");
        remoteRegion_[{peer, d.slot}] = d.dst_off;
      }
  }
  for (const Step& s : plan_.steps)
    if (s.kind == GLOO_HIP_STEP_SEND)
      GLOO_AMD_ENFORCE(remoteRegion_.count({s.peer, s.slot}), "rank ", s.peer, " declared no region for rank ",
                       me, " slot ", s.slot);
  // the sliced interpreter runs on every rank or on none
  int32_t agreed = proposal;
  for (int r = 0; r < P && agreed > 1; r++) {
    if (r == me) continue;
    ArenaRecord pr;
    parseArena(arenas.at(r), r, &pr);
    agreed = std::min(agreed, pr.interpSlices);
  }
  slices_ = agreed > 1 ? agreed : 1;
  assignSeqs();
  if (deviceSignal_) {
    (void)ctx_->counterDevicePtr(inst_, 0, 0, 0);  // register the control block now
    ctx_->errorWord(me).store(0);
    // Copy engine: a lone SEND is hipMemcpyAsync + signal ("memcpy", the
    // default) or the copy+signal kernel ("kernel"); a batch of consecutive
    // SENDs (one per peer) is one multi-destination copy kernel (default),
    // or with "memcpy" one hipMemcpyAsync per forked stream.
    const char* cp = std::getenv("GLOO_AMD_COPY");
    const std::string cmode = cp ? cp : "auto";
    kernelCopy_ = cmode == "kernel";
    autoCopy_ = cmode == "auto";
    batchKernelCopy_ = cmode != "memcpy";
    // Fold + forward (enqueue, FOLD): "0" keeps the fold and its SENDs apart.
    const char* fs = std::getenv("GLOO_AMD_FOLD_SEND");
    foldSend_ = !(fs && std::string(fs) == "0");
    // Completion protocol of the signalling kernels (GLOO_AMD_FWD_RELEASE)
    refreshFwdLean();
    // Workgroups per copy (executor.h): a few dozen saturate an xGMI link.
    // GLOO_AMD_COPY_BLOCKS overrides both the remote and the same-GPU size.
    if (const char* cb = std::getenv("GLOO_AMD_COPY_BLOCKS")) {
      copyBlocks_ = (unsigned)std::max(1, std::atoi(cb));
      copyBlocksLocal_ = copyBlocks_;
    }
    if (const char* cb = std::getenv("GLOO_AMD_COPY_BLOCKS_LOCAL")) copyBlocksLocal_ = (unsigned)std::max(1, std::atoi(cb));
    if (const char* cb = std::getenv("GLOO_AMD_COPY_OUT_BYTES")) copyOutKernelBytes_ = std::strtoull(cb, nullptr, 10);
    if (const char* cb = std::getenv("GLOO_AMD_COPY_OUT_BLOCKS")) copyOutBlocks_ = (unsigned)std::max(1, std::atoi(cb));
    if (const char* cs = std::getenv("GLOO_AMD_REDUCE_STORE")) reducePlain_ = std::string(cs) != "nt";
    if (const char* cs = std::getenv("GLOO_AMD_LOCAL_COPY_STORE"))
      localStore_ = std::string(cs) == "nt" ? kCopyStoreNT : std::string(cs) == "wt" ? kCopyStoreWT : kCopyStorePlain;
    const size_t tickets = std::max<size_t>(256, (size_t)P * GLOO_HIP_NUM_SLOTS * sizeof(unsigned));
    GLOO_AMD_HIP_ALLOC(hipMalloc(&ticket_, tickets));
    // zeroed on the executor's stream and complete before any copy kernel
    // (a plain hipMemset goes to the null stream, which a non-blocking
    // stream does not wait for)
    GLOO_AMD_HIP_CHECK(hipMemsetAsync(ticket_, 0, tickets, stream_));
    // Graph replay pays off where the host is the bottleneck: a plan with
    // steps that are not fused one-workgroup launches.  A mesh plan (a few
    // launches per call) whose messages reach GLOO_AMD_GRAPH_BYTES (default
    // 4 MiB) is device-bound instead: the host's eager enqueue stays ahead,
    // and eager measured 7-13 % faster than replay (HD 16 and 64 MiB per
    // rank, 2 and 4 ranks: DESIGN.md §4, profiles/round3/r3ah_*, r3ak_*).
    // The reference routes keep replay: their per-hop credit handshakes make
    // many launches per call, and eager lost there (HD 16 MiB per rank, 4
    // ranks: 149 vs 122 us, r3ax_*).  "1" / "0" force it.
    const char* gm = std::getenv("GLOO_AMD_GRAPH");
    const std::string gmode = gm ? gm : "auto";
    bool unfused = fuseBytes() == 0 || custom_;
    size_t maxMsg = 0;
    for (const Step& s : plan_.steps) {
      if ((s.kind == GLOO_HIP_STEP_SEND || s.kind == GLOO_HIP_STEP_REDUCE || s.kind == GLOO_HIP_STEP_COPY ||
           s.kind == GLOO_HIP_STEP_LOCAL_REDUCE || s.kind == GLOO_HIP_STEP_LOCAL_BCAST ||
           s.kind == GLOO_HIP_STEP_FOLD) &&
          s.length * es_ > fuseBytes())
        unfused = true;
      maxMsg = std::max(maxMsg, (size_t)s.length * es_);
    }
    const bool meshPlan = (planAlgo_ & GLOO_HIP_ALGO_MESH) || planAlgo_ == GLOO_HIP_ALGO_RING_CHUNKED_MESH;
    graphMode_ = gmode == "1" || (gmode == "auto" && unfused && !(meshPlan && maxMsg >= graphBytes()));
    if (interpMode_) GLOO_AMD_HIP_ALLOC(hipMalloc(&interpSteps_, kInterpMaxSteps * sizeof(InterpStep)));
    if (graphMode_) {
      GLOO_AMD_HIP_ALLOC(hipMalloc(&epoch_, sizeof(uint64_t)));
      GLOO_AMD_HIP_CHECK(hipMemsetAsync(epoch_, 0, sizeof(uint64_t), stream_));
    }
    GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  } catch (const std::exception& e) {
    setupFailure = std::current_exception();
    setupReason = e.what();
    if (setupReason.empty()) setupReason = "setup failed";
    if (setupReason.size() > 900) setupReason.resize(900);  // one bootstrap record
  }
  GLOO_AMD_TRACE_PHASE("ready: '", setupReason, "'");
  const auto ready = ctx_->allgather(strcat_("inst", inst_, "/ready"),
                                     std::vector<char>(setupReason.begin(), setupReason.end()));
  bool anyFailed = false;
  for (int r = 0; r < P; r++) anyFailed = anyFailed || !ready[r].empty();
  if (anyFailed) {
    // the destructor will not run: release what this rank set up.  Every
    // rank saw the same ready records and fails here together, so the
    // tear-down barrier (no arena is reused while a peer writes it) is
    // collective as in the destructor.
    release();
    if (setupFailure) std::rethrow_exception(setupFailure);
    for (int r = 0; r < P; r++)
      GLOO_AMD_ENFORCE(ready[r].empty(), "rank ", r, " could not set up its side of the collective: ",
                       std::string(ready[r].begin(), ready[r].end()));
  }
  if (arenaShm_) arenaShm_->unlink();  // every peer has mapped it by now
}

PlanExecutor::~PlanExecutor() { release(); }

void PlanExecutor::release() {
  try {
    quiesce();
    for (hipStream_t a : aux_) (void)hipStreamSynchronize(a);
    // the captured graph holds copy nodes into the peers' mapped arenas: it
    // goes before the mappings are closed, or a close leaves the import
    // alive and a later import of an equal handle (the peer's next arena of
    // the same size at the same address) was handed the old mapping
    if (graphExec_) (void)hipGraphExecDestroy(graphExec_);
    graphExec_ = nullptr;
    if (ctx_->size > 1) {
      // IPC imports stay mapped (ipc.h: the process-wide import cache);
      // nobody reuses or frees an arena a peer may still write
      for (auto& p : peers_) {
        if (!p.ipc) continue;
        ipc::unimport(p.base);
      }
      for (size_t q = 0; q < peerMailbox_.size(); q++)
        if (peerMailboxIpc_[q]) ipc::unimport(peerMailbox_[q]);
      peers_.clear();
      peerMailbox_.clear();
      ctx_->barrier(strcat_("inst", inst_, "/closed"));
      peerShm_.clear();
      if (arenaShm_) {
        arenaShm_.reset();
      } else if (arenaSlab_) {
        ipc::release(arenaSlab_);  // back to the pool, never freed
      } else if (arena_) {
        GLOO_AMD_HIP_RELEASE(hipFree(arena_));  // never exported
      }
      arenaSlab_ = nullptr;
      arena_ = nullptr;
      if (mailboxSlab_) {
        ipc::release(mailboxSlab_);
      } else if (mailbox_) {
        GLOO_AMD_HIP_RELEASE(hipFree(mailbox_));
      }
      mailboxSlab_ = nullptr;
      mailbox_ = nullptr;
    }
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
    events_.clear();
    for (hipEvent_t e : forkEvents_) (void)hipEventDestroy(e);
    forkEvents_.clear();
    for (hipStream_t a : aux_) (void)hipStreamDestroy(a);
    aux_.clear();
    if (epoch_) GLOO_AMD_HIP_RELEASE(hipFree(epoch_));
    epoch_ = nullptr;
    if (interpSteps_) GLOO_AMD_HIP_RELEASE(hipFree(interpSteps_));
    interpSteps_ = nullptr;
    if (ticket_) GLOO_AMD_HIP_RELEASE(hipFree(ticket_));
    ticket_ = nullptr;
    if (stamps_) GLOO_AMD_HIP_RELEASE(hipFree(stamps_));
    stamps_ = nullptr;
    for (char* p : outStage_)
      if (p) GLOO_AMD_HIP_RELEASE(hipFree(p));
    outStage_.clear();
    for (char* p : inStage_)
      if (p) GLOO_AMD_HIP_RELEASE(hipFree(p));
    inStage_.clear();
    if (ownedStream_) {
      (void)hipStreamSynchronize(ownedStream_);
      (void)hipStreamDestroy(ownedStream_);
    }
    ownedStream_ = nullptr;
    for (hipEvent_t e : sideEvents_) (void)hipEventDestroy(e);
    sideEvents_.clear();
    if (doneEvent_) (void)hipEventDestroy(doneEvent_);
    doneEvent_ = nullptr;
  } catch (...) {
    // teardown is best effort; never throw from a destructor
  }
  if (!released_) ctx_->releaseInstance(inst_);
  released_ = true;
}

void PlanExecutor::waitCounter(std::atomic<uint64_t>& c, uint64_t target, int peer, int slot) {
  // signed difference: a target below the counter (a previous-run credit in
  // the first run) is already met
  auto met = [&] { return (int64_t)(c.load(std::memory_order_acquire) - target) >= 0; };
  if (met()) return;
  const auto t0 = std::chrono::steady_clock::now();
  const auto deadline = t0 + ctx_->timeout();
  for (uint64_t i = 0;; i++) {
    if (met()) break;
    if (i < 4096) {
      __builtin_ia32_pause();
    } else if (i < 8192) {
      sched_yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if ((i & 255) == 255 && std::chrono::steady_clock::now() > deadline)
      throw IoException(strcat_("Timed out waiting for rank ", peer, " (slot ", slot, ") on rank ", ctx_->rank,
                                " after ", ctx_->timeout().count(), " ms"));
  }
  waitSeconds_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

hipStream_t PlanExecutor::auxStream(size_t k) {
  const size_t kMaxAux = 7;
  k %= kMaxAux;
  while (aux_.size() <= k) {
    hipStream_t a;
    GLOO_AMD_HIP_CHECK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    aux_.push_back(a);
  }
  return aux_[k];
}

hipEvent_t PlanExecutor::forkEvent(size_t k) {
  while (forkEvents_.size() <= k) {
    hipEvent_t e;
    GLOO_AMD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    forkEvents_.push_back(e);
  }
  return forkEvents_[k];
}

bool PlanExecutor::mailboxWith(int peer) const {
  return mailbox_ && peer >= 0 && peer < (int)peerMailbox_.size() && peerMailbox_[peer] != nullptr;
}

uint64_t* PlanExecutor::sigFlag(int peer, int slot) {
  if (mailboxWith(peer)) return peerMailbox_[peer] + ((size_t)ctx_->rank * GLOO_HIP_NUM_SLOTS + slot) * kMaxSlices;
  return ctx_->counterDevicePtr(inst_, ctx_->rank, peer, slot);
}

uint64_t* PlanExecutor::waitFlag(int peer, int slot) {
  if (mailboxWith(peer)) return mailbox_ + ((size_t)peer * GLOO_HIP_NUM_SLOTS + slot) * kMaxSlices;
  return ctx_->counterDevicePtr(inst_, peer, ctx_->rank, slot);
}

Seq PlanExecutor::seqOf(size_t i, uint64_t r, bool graph) const {
  const StepSeq& q = stepSeq_[i];
  return graph ? Seq{q.base, q.perRun} : Seq{q.base + r * q.perRun, 0};
}

void PlanExecutor::setStamping(bool on) {
  if (on == stamping_) return;
  dropGraph();  // the captured work differs with stamps
  stableRuns_ = 0;
  stamping_ = on;
  if (on && !stamps_) {
    // one slot per REDUCE / FOLD step, in step order, with its algorithmic
    // bytes: 2 reads + 1 write, or k source reads + 1 write
    stampBytes_.clear();
    stampCount_.clear();
    stampSlotOf_.clear();
    size_t srcs = 0;
    for (size_t i = 0; i < plan_.steps.size(); i++) {
      const Step& s = plan_.steps[i];
      if (s.kind == GLOO_HIP_STEP_FOLD_SRC) srcs++;
      if (s.kind != GLOO_HIP_STEP_REDUCE && s.kind != GLOO_HIP_STEP_FOLD) continue;
      // a one-source FOLD is a copy (the pipelined ring's allgather), not a reduction
      if (s.kind == GLOO_HIP_STEP_REDUCE || srcs >= 2) {
        stampSlotOf_[i] = (int)stampBytes_.size();
        stampBytes_.push_back((s.kind == GLOO_HIP_STEP_REDUCE ? 3.0 : srcs + 1.0) * s.length * es_);
        stampCount_.push_back(s.kind == GLOO_HIP_STEP_REDUCE ? 1 : srcs - 1);
      }
      if (s.kind == GLOO_HIP_STEP_FOLD) srcs = 0;
    }
    stampSlots_ = (int)stampBytes_.size();
    GLOO_AMD_HIP_ALLOC(hipMalloc(&stamps_, sizeof(uint64_t) * kStampSlotWords * std::max(1, stampSlots_)));
  }
}

void PlanExecutor::readStamps() {
  std::vector<uint64_t> h((size_t)kStampSlotWords * stampSlots_);
  if (h.empty()) return;
  GLOO_AMD_HIP_CHECK(hipMemcpy(h.data(), stamps_, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  for (int i = 0; i < stampSlots_; i++) {
    uint64_t ticks = 0;
    if (!stampSpan(&h[(size_t)kStampSlotWords * i], &ticks)) continue;  // not launched this run
    reduceSeconds_ += ticks * 1e-8;  // 100 MHz
    reduceBytes_ += stampBytes_[i];
    reduceCount_ += stampCount_[i];
  }
}

void PlanExecutor::run() {
  GLOO_AMD_HIP_CHECK(hipSetDevice(ctx_->device()));
  const int me = ctx_->rank;
  if (deviceSignal_ && ctx_->errorWord(me).load() != 0)
    throw IoException(strcat_("rank ", me, ": a device-side wait of a previous run timed out"));
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  GLOO_AMD_HIP_CHECK(hipStreamIsCapturing(stream_, &cs));
  GLOO_AMD_ENFORCE(cs == hipStreamCaptureStatusNone,
                   "run() on a stream under capture: the executor captures and replays its own graph");
  waitSeconds_ = 0;
  reduceSeconds_ = reduceBytes_ = 0;
  reduceCount_ = 0;
  replayed_ = false;
  // the caller's work on its other pointers' streams comes first
  for (size_t i = 0; i < sideStreams_.size(); i++) {
    GLOO_AMD_HIP_CHECK(hipEventRecord(sideEvents_[i], sideStreams_[i]));
    GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(stream_, sideEvents_[i], 0));
  }
  const uint64_t r = runs_ + 1;
  // sliced plans must run sliced on every rank (their flags are per slice);
  // profiling then reports no reduce events
  const bool interp = deviceSignal_ && interpMode_ && (!(profiling_ || stamping_) || slices_ > 1);
  if (interp && interpDirty_) buildInterp();
  const bool graphable = deviceSignal_ && graphMode_ && !profiling_;
  if (interp && interpCount_ > 0) {
    const uint64_t timeoutTicks = (uint64_t)ctx_->timeout().count() * 100000ull;  // 100 MHz realtime clock
    const size_t bytes = count_ * es_;
    // buffers on other GPUs of the process: the step list reads and writes
    // their local copies (buildInterp)
    for (size_t j = 0; anyRemote_ && j < inputs_.size(); j++)
      if (inRemote_[j]) GLOO_AMD_HIP_CHECK(hipMemcpyAsync(inStage_[j], inputs_[j], bytes, hipMemcpyDeviceToDevice, stream_));
    for (size_t j = 1; anyRemote_ && j < ptrs_.size(); j++)
      if (outRemote_[j]) GLOO_AMD_HIP_CHECK(hipMemcpyAsync(outStage_[j], ptrs_[j], bytes, hipMemcpyDeviceToDevice, stream_));
    checkRc(launchPlanInterp(op_, dtype_, interpSteps_, interpCount_, r, timeoutTicks, ctx_->errorWordDevicePtr(me),
                             slices_, stream_),
            "plan interpreter");
    for (size_t j = 1; anyRemote_ && j < ptrs_.size(); j++)
      if (outRemote_[j]) GLOO_AMD_HIP_CHECK(hipMemcpyAsync(ptrs_[j], outStage_[j], bytes, hipMemcpyDeviceToDevice, stream_));
  } else if (graphable && (graphExec_ || stableRuns_ >= 1)) {
    if (!graphExec_) tryCapture(r);  // sets the device epoch to r - 1
    if (graphExec_) {
      // a run enqueued eagerly since the last replay left the epoch behind
      if (epochRuns_ != r - 1) GLOO_AMD_HIP_CHECK(launchEpochSet(epoch_, r - 1, stream_));
      GLOO_AMD_HIP_CHECK(hipGraphLaunch(graphExec_, stream_));
      epochRuns_ = r;
      replayed_ = true;
    } else {
      enqueue(r, false);
    }
  } else {
    enqueue(r, false);
  }
  runs_ = r;
  stableRuns_++;
  if (!ownStream_) {
    // every stream of the caller is ordered after the collective, and later
    // host waits (teardown, a new stream) use this event, not the stream
    GLOO_AMD_HIP_CHECK(hipEventRecord(doneEvent_, stream_));
    donePending_ = true;
    for (hipStream_t t : sideStreams_) GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(t, doneEvent_, 0));
  }
  if (ownStream_ || profiling_ || stamping_) {
    const auto t0 = std::chrono::steady_clock::now();
    GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
    if (deviceSignal_) waitSeconds_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (deviceSignal_ && ctx_->errorWord(me).exchange(0) != 0)
      throw IoException(strcat_("Timed out on rank ", me, " waiting for a peer (device-side wait, ",
                                ctx_->timeout().count(), " ms)"));
  }
  if (stamping_ && !(interp && interpCount_ > 0)) readStamps();
  for (size_t i = 0; profiling_ && i + 1 < evUsed_; i += 2) {
    float ms = 0;
    GLOO_AMD_HIP_CHECK(hipEventElapsedTime(&ms, events_[i], events_[i + 1]));
    reduceSeconds_ += ms * 1e-3;
  }
}

void PlanExecutor::tryCapture(uint64_t r) {
  // The device epoch holds the number of runs already executed; the graph's
  // first node advances it, and every node derives its sequence numbers
  // from it.  Capture failures are not fatal: the plan keeps being enqueued
  // eagerly (graphError() says why).
  GLOO_AMD_HIP_CHECK(launchEpochSet(epoch_, r - 1, stream_));
  epochRuns_ = r - 1;
  GLOO_AMD_HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
  hipGraph_t g = nullptr;
  try {
    GLOO_AMD_HIP_CHECK(launchEpochBump(epoch_, stream_));
    enqueue(r, true);
  } catch (const std::exception& ex) {
    (void)hipStreamEndCapture(stream_, &g);
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    graphMode_ = false;
    graphError_ = ex.what();
    return;
  }
  hipError_t e = hipStreamEndCapture(stream_, &g);
  if (e == hipSuccess) e = hipGraphInstantiate(&graphExec_, g, nullptr, nullptr, 0);
  if (g) (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    graphExec_ = nullptr;
    graphMode_ = false;
    graphError_ = hipGetErrorString(e);
    (void)hipGetLastError();
  }
}

void PlanExecutor::buildInterp() {
  interpDirty_ = false;
  interpCount_ = 0;
  // Buffers on another GPU of the process: the step list runs over their
  // local staging copies (run() pulls them in before the launch and pushes
  // the broadcast outputs back after it), so the launch touches local HBM
  // only.  A sliced plan has no other route, its flags being per slice.
  auto outPtr = [&](size_t j) -> char* {
    return j < outRemote_.size() && outRemote_[j] ? outStage_[j] : static_cast<char*>(ptrs_[j]);
  };
  auto inPtr = [&](size_t j) -> const char* {
    return j < inRemote_.size() && inRemote_[j] ? static_cast<const char*>(inStage_[j])
                                                 : static_cast<const char*>(inputs_.at(j));
  };
  // a sliced plan's message sizes were vetted when the ranks agreed on it
  const size_t limit = slices_ > 1 ? SIZE_MAX : interpBytes();
  // a step operand: arena (the slab holding [off, +len)) or user buffer 0
  auto userOrArena = [&](bool arena, uint64_t off, uint64_t len) -> char* {
    return arena ? arenaAt(off, len) : userPtr(0) + off * es_;
  };
  auto sendSrc = [&](const Step& t) -> const char* {
    if (t.flags & GLOO_HIP_SRC_ARENA) return arenaAt(t.src_off, t.length);
    return (t.flags & GLOO_HIP_FROM_INPUTS ? inPtr(0) : userPtr(0)) + t.src_off * es_;
  };
  std::vector<InterpStep> v;
  auto push = [&](int kind) -> InterpStep& {
    v.emplace_back();
    InterpStep& t = v.back();
    std::memset(&t, 0, sizeof t);
    t.kind = kind;
    return t;
  };
  auto withSeq = [&](InterpStep& t, size_t i, uint64_t* flag) {
    t.flag = flag;
    t.base = stepSeq_[i].base;
    t.perRun = stepSeq_[i].perRun;
  };
  // dst = src[0] op src[1] ... (left fold); a copy for one source
  auto fold = [&](char* dst, const std::vector<const char*>& srcs, size_t n, int mode) {
    InterpStep& t = push(kInterpFold);
    t.dst = dst;
    t.nsrc = (int)srcs.size();
    t.mode = mode;
    for (size_t k = 0; k < srcs.size(); k++) t.src[k] = srcs[k];
    t.n = n;
  };
  // false: overlapping operands (a memmove), not an interpreter shape
  auto copy = [&](char* dst, const char* src, size_t elems) {
    const size_t bytes = elems * es_;
    if (dst == src || bytes == 0) return true;
    if (dst < src + bytes && src < dst + bytes) return false;
    InterpStep& t = push(kInterpCopy);
    t.dst = dst;
    t.src[0] = src;
    t.n = elems;
    return true;
  };
  auto fail = [&] {
    GLOO_AMD_ENFORCE(slices_ == 1, "a sliced interpreter plan with a step the interpreter cannot run");
    v.clear();
  };
  const std::vector<size_t> cuts = slices_ > 1 ? userCuts(plan_) : std::vector<size_t>();
  auto pieces = [&](const Step& t) { return cutRange(cuts, t.dst_off, t.length); };
  std::vector<const char*> foldSrcs;
  const std::vector<Step>& steps = plan_.steps;
  for (size_t i = 0; i < steps.size(); i++) {
    const Step& s = steps[i];
    const size_t bytes = s.length * es_;
    if (bytes > limit) return fail();
    switch (s.kind) {
      case GLOO_HIP_STEP_DECL_RECV:
      case GLOO_HIP_STEP_WAIT_SEND:
        break;
      case GLOO_HIP_STEP_SEND: {
        InterpStep& t = push(kInterpSend);
        t.dst = peerAt(s.peer, remoteRegion_.at({s.peer, s.slot}) + s.dst_off, s.length);
        t.src[0] = sendSrc(s);
        t.n = s.length;
        withSeq(t, i, sigFlag(s.peer, s.slot));
        break;
      }
      case GLOO_HIP_STEP_NOTIFY:
        withSeq(push(kInterpSignal), i, sigFlag(s.peer, s.slot));
        break;
      case GLOO_HIP_STEP_WAIT_RECV:
      case GLOO_HIP_STEP_WAIT_NOTIFY:
        withSeq(push(kInterpWait), i, waitFlag(s.peer, s.slot));
        break;
      case GLOO_HIP_STEP_REDUCE: {  // out = (in | out) op inbox
        const char* a = (s.flags & GLOO_HIP_FROM_INPUTS ? inPtr(0) : static_cast<const char*>(userPtr(0))) +
                        s.dst_off * es_;
        fold(userPtr(0) + s.dst_off * es_, {a, arenaAt(s.src_off, s.length)}, s.length, 0);
        break;
      }
      case GLOO_HIP_STEP_COPY:
        if (!copy(userOrArena(s.flags & GLOO_HIP_DST_ARENA, s.dst_off, s.length),
                  userOrArena(s.flags & GLOO_HIP_SRC_ARENA, s.src_off, s.length), s.length))
          return fail();
        break;
      case GLOO_HIP_STEP_LOCAL_REDUCE:  // as enqueue(): chained folds of <= GLOO_HIP_MAX_SRCS sources
        // sliced: one piece per range the other steps use (userCuts)
        for (const auto& pc : pieces(s)) {
          const size_t off = pc.first * es_, len = pc.second;
          const bool fromIn = s.flags & GLOO_HIP_FROM_INPUTS;
          const size_t nfrom = fromIn ? inputs_.size() : ptrs_.size();
          auto from = [&](size_t j) -> const char* { return (fromIn ? inPtr(j) : outPtr(j)) + off; };
          char* out0 = userPtr(0) + off;
          if (nfrom == 1) {
            if (!copy(out0, from(0), len)) return fail();
            continue;
          }
          std::vector<const char*> srcs;
          size_t j = 0;
          for (; j < nfrom && srcs.size() < GLOO_HIP_MAX_SRCS; j++) srcs.push_back(from(j));
          fold(out0, srcs, len, 0);
          while (j < nfrom) {
            srcs.assign(1, out0);
            for (; j < nfrom && srcs.size() < GLOO_HIP_MAX_SRCS; j++) srcs.push_back(from(j));
            fold(out0, srcs, len, 0);
          }
        }
        break;
      case GLOO_HIP_STEP_LOCAL_BCAST:
        for (const auto& pc : pieces(s))
          for (size_t j = 1; j < ptrs_.size(); j++)
            if (!copy(outPtr(j) + pc.first * es_, userPtr(0) + pc.first * es_, pc.second)) return fail();
        break;
      case GLOO_HIP_STEP_FOLD_SRC:
        foldSrcs.push_back(sendSrc(s));
        break;
      case GLOO_HIP_STEP_FOLD:
        GLOO_AMD_ENFORCE(!foldSrcs.empty() && foldSrcs.size() <= GLOO_HIP_MAX_SRCS, "bad fold");
        fold(userOrArena(s.flags & GLOO_HIP_DST_ARENA, s.dst_off, s.length), foldSrcs, s.length,
             s.flags & GLOO_HIP_FOLD_TREE ? 2 : s.flags & GLOO_HIP_FOLD_REVERSE ? 1 : 0);
        foldSrcs.clear();
        break;
      default:
        return fail();
    }
    if (v.size() > (size_t)kInterpMaxSteps) return fail();
  }
  if (v.empty()) return;
  // Batches (signal.h kInterpDefer): a run of waits polls every flag before
  // its one acquire and barrier, and a run of mutually independent data steps
  // (a mesh owner's sends to every peer, its copies out of the inboxes, the
  // credits after them) drains once and publishes its flags together — one
  // memory round trip per run instead of per step.  GLOO_AMD_INTERP_BATCH=0
  // keeps every step on its own.
  const char* ib = std::getenv("GLOO_AMD_INTERP_BATCH");
  if (!(ib && ib[0] == '0')) markInterpBatches(v.data(), v.size(), es_);
  // the bound the ranks agreed on (slicedInterpSteps) must cover what was
  // emitted; an under-count would have let an unrunnable plan be proposed
  GLOO_AMD_ENFORCE(slices_ == 1 || v.size() <= slicedInterpSteps(plan_, (int)inputs_.size(), (int)ptrs_.size()),
                   "sliced step list of ", v.size(), " entries exceeds its proposed bound");
  // an earlier launch may still read the list
  GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
  // on the stream the interpreter runs on (a null-stream copy is not ordered
  // before it), complete before `v` goes away
  GLOO_AMD_HIP_CHECK(
      hipMemcpyAsync(interpSteps_, v.data(), v.size() * sizeof(InterpStep), hipMemcpyHostToDevice, stream_));
  GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
  interpCount_ = (int)v.size();
}

void PlanExecutor::enqueue(uint64_t r, bool graph) {
  const int me = ctx_->rank;
  const uint64_t timeoutTicks = (uint64_t)ctx_->timeout().count() * 100000ull;  // 100 MHz realtime clock
  const uint64_t* epoch = graph ? epoch_ : nullptr;
  auto signal = [&](size_t i) {
    const Step& s = plan_.steps[i];
    if (deviceSignal_) {
      GLOO_AMD_HIP_CHECK(launchSignal(sigFlag(s.peer, s.slot), seqOf(i, r, graph), epoch,
                                      stream_));
    } else {
      enqueueBump(stream_, ctx_->counter(inst_, me, s.peer, s.slot));
    }
  };
  evUsed_ = 0;
  auto event = [&]() {
    if (evUsed_ == events_.size()) {
      hipEvent_t e;
      GLOO_AMD_HIP_CHECK(hipEventCreate(&e));
      events_.push_back(e);
    }
    return events_[evUsed_++];
  };
  // Small-message fusion (device signalling only): a plan's
  //   WAIT_* -> {REDUCE | COPY | SEND} -> [NOTIFY]   or a lone small SEND
  // becomes ONE one-workgroup launch (launchFusedSmall): below a few KiB a
  // hop costs dispatches, not bytes.  Off while profiling reduce kernels.
  const size_t kFuseBytes = fuseBytes();
  const bool fuse = deviceSignal_ && !profiling_ && kFuseBytes > 0 && !custom_;
  // a step operand: arena (the slab holding [off, +len)) or user buffer 0
  auto userOrArena = [&](bool arena, uint64_t off, uint64_t len) -> char* {
    return arena ? arenaAt(off, len) : userPtr(0) + off * es_;
  };
  // a SEND's source: the arena, input 0 (gloo::reduce's first segments) or output 0
  auto sendSrc = [&](const Step& t) -> const char* {
    if (t.flags & GLOO_HIP_SRC_ARENA) return arenaAt(t.src_off, t.length);
    return (t.flags & GLOO_HIP_FROM_INPUTS ? static_cast<const char*>(inputs_.at(0)) : userPtr(0)) +
           t.src_off * es_;
  };
  const std::vector<Step>& steps = plan_.steps;
  auto sendDst = [&](const Step& t) {
    return peerAt(t.peer, remoteRegion_[{t.peer, t.slot}] + t.dst_off, t.length);
  };
  auto isWaitKind = [](int k) { return k == GLOO_HIP_STEP_WAIT_RECV || k == GLOO_HIP_STEP_WAIT_NOTIFY; };
  std::vector<const void*> foldSrcs;
  if (stamping_) checkRc(launchStampInit(stamps_, stampSlots_, stream_), "stamp init");
  // the stamp slot of the next REDUCE / FOLD launch (none when not stamping)
  struct StampScope {
    explicit StampScope(uint64_t* slot) : prev(setLaunchStamp(slot)) {}
    ~StampScope() { setLaunchStamp(prev); }
    uint64_t* prev;
  };
  // the store flavour of this plan's REDUCE launches (signal.h)
  struct ReduceStoreScope {
    explicit ReduceStoreScope(bool plain) : prev(setReducePlainStores(plain)) {}
    ~ReduceStoreScope() { setReducePlainStores(prev); }
    bool prev;
  } reduceStores(reducePlain_);
  auto slotOf = [&](size_t step) -> uint64_t* {
    if (!stamping_) return nullptr;
    auto it = stampSlotOf_.find(step);
    return it == stampSlotOf_.end() ? nullptr : stamps_ + (size_t)kStampSlotWords * it->second;
  };
  for (size_t i = 0; i < steps.size(); i++) {
    const Step& s = steps[i];
    // A run of consecutive SENDs (a mesh schedule's sends to every peer):
    // all in flight at once.
    if (s.kind == GLOO_HIP_STEP_SEND && i + 1 < steps.size() && steps[i + 1].kind == GLOO_HIP_STEP_SEND) {
      size_t j = i;
      while (j < steps.size() && steps[j].kind == GLOO_HIP_STEP_SEND) j++;
      {
        // one ticket counter and flag per (peer, slot): a batch sharing a
        // channel would interleave tickets and publish out of order
        std::set<std::pair<int, int>> chans;
        for (size_t k = i; k < j; k++)
          GLOO_AMD_ENFORCE(chans.insert({steps[k].peer, steps[k].slot}).second, "a SEND batch repeats channel (peer ",
                           steps[k].peer, ", slot ", steps[k].slot, ")");
      }
      if (deviceSignal_ && batchKernelCopy_) {
        for (size_t b = i; b < j; b += kMaxCopyEntries) {
          CopyDesc d[kMaxCopyEntries];
          int nd = 0;
          for (size_t k = b; k < std::min(j, b + kMaxCopyEntries); k++) {
            const Step& t = steps[k];
            const size_t bytes = t.length * es_;
            d[nd++] = CopyDesc{sendDst(t), sendSrc(t), bytes,
                               sigFlag(t.peer, t.slot), seqOf(k, r, graph),
                               ticket_ + (size_t)t.peer * GLOO_HIP_NUM_SLOTS + t.slot,
                               copySignalGrid(bytes, copyBlocksFor(t.peer))};
          }
          checkRc(launchCopySignalMulti(d, nd, epoch, stream_), "copy_signal_kernel (batch)");
        }
      } else {
        // fork: one hipMemcpyAsync + arrival signal per auxiliary stream, joined
        // back before anything later on the rank's stream
        hipEvent_t fork = forkEvent(0);
        GLOO_AMD_HIP_CHECK(hipEventRecord(fork, stream_));
        for (size_t k = i; k < j; k++) {
          const Step& t = steps[k];
          hipStream_t a = auxStream(k - i);
          GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(a, fork, 0));
          if (t.length)
            GLOO_AMD_HIP_CHECK(hipMemcpyAsync(sendDst(t), sendSrc(t), t.length * es_, hipMemcpyDeviceToDevice, a));
          if (deviceSignal_) {
            GLOO_AMD_HIP_CHECK(launchSignal(sigFlag(t.peer, t.slot), seqOf(k, r, graph),
                                            epoch, a));
          } else {
            enqueueBump(a, ctx_->counter(inst_, me, t.peer, t.slot));
          }
          hipEvent_t join = forkEvent(1 + (k - i));
          GLOO_AMD_HIP_CHECK(hipEventRecord(join, a));
          GLOO_AMD_HIP_CHECK(hipStreamWaitEvent(stream_, join, 0));
        }
      }
      i = j - 1;
      continue;
    }
    // A run of consecutive local COPYs with disjoint operands (a mesh
    // schedule's results out of the inboxes): one multi-copy launch.
    if (s.kind == GLOO_HIP_STEP_COPY && i + 1 < steps.size() && steps[i + 1].kind == GLOO_HIP_STEP_COPY &&
        deviceSignal_) {
      size_t j = i;
      std::vector<std::pair<char*, const char*>> ops;
      std::vector<size_t> lens;
      for (; j < steps.size() && steps[j].kind == GLOO_HIP_STEP_COPY && ops.size() < (size_t)kMaxCopyEntries; j++) {
        const Step& t = steps[j];
        ops.push_back({userOrArena(t.flags & GLOO_HIP_DST_ARENA, t.dst_off, t.length),
                       userOrArena(t.flags & GLOO_HIP_SRC_ARENA, t.src_off, t.length)});
        lens.push_back(t.length * es_);
      }
      bool disjoint = true;
      for (size_t a = 0; a < ops.size(); a++)
        for (size_t b = 0; b < ops.size(); b++) {
          const char* d = ops[a].first;
          const char* q = ops[b].second;
          if (d < q + lens[b] && q < d + lens[a]) disjoint = false;
          if (a != b && d < ops[b].first + lens[b] && ops[b].first < d + lens[a]) disjoint = false;
        }
      if (disjoint) {
        CopyDesc d[kMaxCopyEntries];
        int nd = 0;
        for (size_t k = 0; k < ops.size(); k++)
          if (lens[k]) d[nd++] = CopyDesc{ops[k].first, ops[k].second, lens[k], nullptr, Seq{}, nullptr,
                                          copySignalGrid(lens[k], copyOutBlocks_)};
        if (nd) checkRc(launchCopySignalMulti(d, nd, epoch, stream_, localStore_), "copy kernel (local batch)");
        i = j - 1;
        continue;
      }
    }
    // A run of consecutive waits: one launch polls them all.
    if (deviceSignal_ && isWaitKind(s.kind) && i + 1 < steps.size() && isWaitKind(steps[i + 1].kind)) {
      size_t j = i;
      std::vector<const uint64_t*> flags;
      std::vector<Seq> targets;
      for (; j < steps.size() && isWaitKind(steps[j].kind); j++) {
        flags.push_back(waitFlag(steps[j].peer, steps[j].slot));
        targets.push_back(seqOf(j, r, graph));
      }
      GLOO_AMD_HIP_CHECK(launchWaitMulti(flags.data(), targets.data(), (int)flags.size(), epoch, timeoutTicks,
                                         ctx_->errorWordDevicePtr(me), stream_));
      i = j - 1;
      continue;
    }
    if (fuse) {
      const bool isWait = s.kind == GLOO_HIP_STEP_WAIT_RECV || s.kind == GLOO_HIP_STEP_WAIT_NOTIFY;
      const Step* t = isWait && i + 1 < steps.size() ? &steps[i + 1] : &s;
      // (a three-operand REDUCE, out = in op inbox, is not a fused shape)
      const bool body = (t->kind == GLOO_HIP_STEP_REDUCE && !(t->flags & GLOO_HIP_FROM_INPUTS)) ||
                        t->kind == GLOO_HIP_STEP_COPY || t->kind == GLOO_HIP_STEP_SEND;
      if (body && t->length * es_ <= kFuseBytes && (isWait || t->kind == GLOO_HIP_STEP_SEND)) {
        int op = 0;
        char* dst = nullptr;
        const char* src = nullptr;
        if (t->kind == GLOO_HIP_STEP_REDUCE) {
          op = op_;
          dst = userPtr(0) + t->dst_off * es_;
          src = arenaAt(t->src_off, t->length);
        } else if (t->kind == GLOO_HIP_STEP_COPY) {
          dst = userOrArena(t->flags & GLOO_HIP_DST_ARENA, t->dst_off, t->length);
          src = userOrArena(t->flags & GLOO_HIP_SRC_ARENA, t->src_off, t->length);
        } else {
          dst = peerAt(t->peer, remoteRegion_[{t->peer, t->slot}] + t->dst_off, t->length);
          src = sendSrc(*t);
        }
        const size_t bytes = t->length * es_;
        const bool overlap = dst < src + bytes && src < dst + bytes && dst != src;
        if (!(t->kind == GLOO_HIP_STEP_COPY && overlap)) {
          const uint64_t* wf = nullptr;
          Seq wt;
          if (isWait) {
            wt = seqOf(i, r, graph);
            wf = waitFlag(s.peer, s.slot);
          }
          uint64_t* sf = nullptr;
          Seq sv;
          size_t consumed = isWait ? 2 : 1;
          if (t->kind == GLOO_HIP_STEP_SEND) {
            sv = seqOf(isWait ? i + 1 : i, r, graph);
            sf = sigFlag(t->peer, t->slot);
          } else if (isWait && i + 2 < steps.size() && steps[i + 2].kind == GLOO_HIP_STEP_NOTIFY) {
            const Step& nt = steps[i + 2];
            sv = seqOf(i + 2, r, graph);
            sf = sigFlag(nt.peer, nt.slot);
            consumed = 3;
          }
          checkRc(launchFusedSmall(op, dtype_, dst, src, t->length, wf, wt, timeoutTicks, ctx_->errorWordDevicePtr(me),
                                   sf, sv, epoch, stream_),
                  "fused step");
          i += consumed - 1;
          continue;
        }
      }
    }
    switch (s.kind) {
      case GLOO_HIP_STEP_DECL_RECV:
        break;
      case GLOO_HIP_STEP_SEND: {
        char* dst = peerAt(s.peer, remoteRegion_[{s.peer, s.slot}] + s.dst_off, s.length);
        const char* src = sendSrc(s);
        // GLOO_AMD_COPY=auto: a lone SEND of >= 16 MiB to a rank on this
        // same GPU goes to the copy kernel with 256 workgroups, which moves
        // HBM -> HBM faster than the blit engine from 16 MiB up (one MI355X:
        // 8.1 vs 9.7 us at 16 MiB, 22.0 vs 26.0 us at 64 MiB kernel time,
        // profiles/round2/r2d_rocprof_copy_engines_segments.csv); below that,
        // and over xGMI, hipMemcpyAsync + signal inside a captured graph
        const bool bigLocal = autoCopy_ && s.length * es_ >= (16u << 20) && peers_[s.peer].device == ctx_->device();
        // eager (not captured): hipMemcpyAsync into an IPC mapping is the slow
        // path of an eager enqueue, and the copy kernel signals without a
        // write-back since round 3; graph memcpy nodes stay faster
        // (profiles/round3/r3ag_latency_ab_release_and_copy_engine.jsonl)
        const bool eagerKernel = autoCopy_ && !graph;
        if (kernelCopy_ || bigLocal || eagerKernel) {
          const unsigned grid = copySignalGrid(s.length * es_, bigLocal ? 256u : copyBlocksFor(s.peer));
          checkRc(launchCopySignal(dst, src, s.length * es_, sigFlag(s.peer, s.slot),
                                   seqOf(i, r, graph), ticket_ + (size_t)s.peer * GLOO_HIP_NUM_SLOTS + s.slot, epoch,
                                   grid, stream_),
                  "copy_signal_kernel");
          break;
        }
        if (s.length) GLOO_AMD_HIP_CHECK(hipMemcpyAsync(dst, src, s.length * es_, hipMemcpyDeviceToDevice, stream_));
        signal(i);
        break;
      }
      case GLOO_HIP_STEP_WAIT_RECV:
      case GLOO_HIP_STEP_WAIT_NOTIFY: {
        if (deviceSignal_) {
          GLOO_AMD_HIP_CHECK(launchWait(waitFlag(s.peer, s.slot), seqOf(i, r, graph), epoch,
                                        timeoutTicks, ctx_->errorWordDevicePtr(me), stream_));
        } else {
          waitCounter(ctx_->counter(inst_, s.peer, me, s.slot), seqOf(i, r, false).base, s.peer, s.slot);
        }
        break;
      }
      case GLOO_HIP_STEP_REDUCE: {
        if (profiling_) GLOO_AMD_HIP_CHECK(hipEventRecord(event(), stream_));
        StampScope stamp(slotOf(i));
        if (s.flags & GLOO_HIP_FROM_INPUTS) {  // out = in op inbox (gloo/reduce.cc:180-184)
          checkRc(gloo_hip_reduce3(op_, dtype_, userPtr(0) + s.dst_off * es_,
                                   static_cast<const char*>(inputs_.at(0)) + s.dst_off * es_,
                                   arenaAt(s.src_off, s.length), s.length, stream_),
                  "gloo_hip_reduce3");
        } else {
          checkRc(gloo_hip_reduce(op_, dtype_, userPtr(0) + s.dst_off * es_, arenaAt(s.src_off, s.length), s.length,
                                  stream_),
                  "gloo_hip_reduce");
        }
        if (profiling_) {
          GLOO_AMD_HIP_CHECK(hipEventRecord(event(), stream_));
          reduceBytes_ += 3.0 * s.length * es_;
          reduceCount_++;
        }
        break;
      }
      case GLOO_HIP_STEP_COPY: {
        char* dst = userOrArena(s.flags & GLOO_HIP_DST_ARENA, s.dst_off, s.length);
        const char* src = userOrArena(s.flags & GLOO_HIP_SRC_ARENA, s.src_off, s.length);
        const size_t bytes = s.length * es_;
        if (deviceSignal_ && bytes >= copyOutKernelBytes_ && bytes > 0 && (dst + bytes <= src || src + bytes <= dst)) {
          const CopyDesc d{dst, src, bytes, nullptr, Seq{}, nullptr, copySignalGrid(bytes, copyOutBlocks_)};
          checkRc(launchCopySignalMulti(&d, 1, epoch, stream_, localStore_), "copy kernel (local)");
          break;
        }
        deviceMove(dst, src, bytes, stream_);
        break;
      }
      case GLOO_HIP_STEP_NOTIFY:
        signal(i);
        break;
      case GLOO_HIP_STEP_WAIT_SEND:
        // stream order already puts every later use of the buffer after the
        // copy; only host-side waiting needs the explicit drain
        if (!deviceSignal_) GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
        break;
      case GLOO_HIP_STEP_LOCAL_REDUCE: {
        // out[0][range] = ((src0 op src1) op src2) ... with src = the
        // separate inputs (FROM_INPUTS; one input = a copy) or the outputs;
        // one fused pass per GLOO_HIP_MAX_SRCS sources.
        const size_t off = s.dst_off * es_;
        const bool fromInputs = s.flags & GLOO_HIP_FROM_INPUTS;
        std::vector<void*> from = fromInputs ? inputs_ : ptrs_;
        if (anyRemote_) {
          const std::vector<bool>& remote = fromInputs ? inRemote_ : outRemote_;
          const std::vector<char*>& stage = fromInputs ? inStage_ : outStage_;
          for (size_t j = 0; j < from.size(); j++)
            if (remote[j]) {  // pull the range over the peer link into local HBM
              GLOO_AMD_HIP_CHECK(hipMemcpyAsync(stage[j] + off, static_cast<const char*>(from[j]) + off,
                                                s.length * es_, hipMemcpyDeviceToDevice, stream_));
              from[j] = stage[j];
            }
        }
        char* out0 = userPtr(0) + off;
        if (from.size() == 1) {
          deviceMove(out0, static_cast<const char*>(from[0]) + off, s.length * es_, stream_);
          break;
        }
        std::vector<const void*> srcs;
        size_t j = 0;
        for (; j < from.size() && srcs.size() < GLOO_HIP_MAX_SRCS; j++)
          srcs.push_back(static_cast<const char*>(from[j]) + off);
        checkRc(gloo_hip_reduce_multi(op_, dtype_, out0, srcs.data(), (int)srcs.size(), s.length, stream_),
                "gloo_hip_reduce_multi");
        while (j < from.size()) {
          srcs.assign(1, out0);
          for (; j < from.size() && srcs.size() < GLOO_HIP_MAX_SRCS; j++)
            srcs.push_back(static_cast<const char*>(from[j]) + off);
          checkRc(gloo_hip_reduce_multi(op_, dtype_, out0, srcs.data(), (int)srcs.size(), s.length, stream_),
                  "gloo_hip_reduce_multi");
        }
        break;
      }
      case GLOO_HIP_STEP_FOLD_SRC:  // the arena, input 0 (gloo::reduce's contribution) or output 0
        foldSrcs.push_back(sendSrc(s));
        break;
      case GLOO_HIP_STEP_FOLD: {
        // one pass over every source, in the plan's order (plan.cc FOLD)
        GLOO_AMD_ENFORCE(!foldSrcs.empty() && foldSrcs.size() <= GLOO_HIP_MAX_SRCS, "bad fold");
        if (profiling_) GLOO_AMD_HIP_CHECK(hipEventRecord(event(), stream_));
        const int mode = s.flags & GLOO_HIP_FOLD_TREE ? 2 : s.flags & GLOO_HIP_FOLD_REVERSE ? 1 : 0;
        // Fold + forward: the SENDs right after a fold that ship its result
        // unchanged (a mesh owner's return of its finished range) ride in the
        // fold's own pass, and its last workgroup signals them and the NOTIFY
        // credits that follow.  Device signalling only; off while the reduce
        // kernels are timed with events (they need a pure fold between two
        // markers).  Device stamps time the fused launch itself, forward
        // stores included (stamp_end waits for them), so what ships is what
        // is measured; the slot's bytes stay the fold's (k + 1) * n * s.
        if (foldSend_ && deviceSignal_ && !custom_ && !profiling_ && s.length > 0 &&
            !(s.flags & GLOO_HIP_DST_ARENA)) {
          char* fdst = userPtr(0) + s.dst_off * es_;
          FwdDesc fwd[kMaxCopyEntries];
          int nf = 0;
          size_t j = i + 1;
          for (; j < steps.size() && nf < kMaxCopyEntries; j++) {
            const Step& t = steps[j];
            if (t.kind != GLOO_HIP_STEP_SEND || (t.flags & (GLOO_HIP_SRC_ARENA | GLOO_HIP_FROM_INPUTS)) ||
                t.src_off != s.dst_off || t.length != s.length)
              break;
            fwd[nf++] = FwdDesc{sendDst(t), sigFlag(t.peer, t.slot), seqOf(j, r, graph)};
          }
          // every SEND of the run must be taken, or the rest would still
          // re-read the result; a partial run stays unfused
          const bool sendsTaken = j == steps.size() || steps[j].kind != GLOO_HIP_STEP_SEND;
          // credits right after (a reduce-scatter owner's NOTIFYs: the fold has
          // consumed the senders' inboxes) go out from the same last workgroup
          // as data-free entries, once every read of the fold is complete
          if (sendsTaken)
            for (; j < steps.size() && nf < kMaxCopyEntries && steps[j].kind == GLOO_HIP_STEP_NOTIFY; j++)
              fwd[nf++] = FwdDesc{nullptr, sigFlag(steps[j].peer, steps[j].slot), seqOf(j, r, graph)};
          if (nf > 0 && sendsTaken) {
            const Step& t0 = steps[i + 1];
            StampScope stamp(slotOf(i));
            checkRc(launchFoldSend(op_, dtype_, fdst, foldSrcs.data(), (int)foldSrcs.size(), s.length, mode, fwd,
                                   nf, ticket_ + (size_t)t0.peer * GLOO_HIP_NUM_SLOTS + t0.slot, epoch, stream_),
                    "fold+forward");
            foldSendUsed_ = true;
            foldSrcs.clear();
            i = j - 1;
            break;
          }
        }
        {
          StampScope stamp(slotOf(i));
          checkRc(launchFold(op_, dtype_, userOrArena(s.flags & GLOO_HIP_DST_ARENA, s.dst_off, s.length),
                             foldSrcs.data(), (int)foldSrcs.size(), s.length, mode, stream_),
                  "fold");
        }
        if (profiling_) {
          GLOO_AMD_HIP_CHECK(hipEventRecord(event(), stream_));
          if (foldSrcs.size() >= 2) {
            reduceBytes_ += (foldSrcs.size() + 1.0) * s.length * es_;
            reduceCount_ += foldSrcs.size() - 1;
          } else {
            evUsed_ -= 2;  // a one-source fold is a copy: not a reduce kernel to time
          }
        }
        foldSrcs.clear();
        break;
      }
      case GLOO_HIP_STEP_LOCAL_BCAST:
        for (size_t j = 1; j < ptrs_.size(); j++)
          GLOO_AMD_HIP_CHECK(hipMemcpyAsync(userPtr(j) + s.dst_off * es_, userPtr(0) + s.dst_off * es_,
                                            s.length * es_, hipMemcpyDeviceToDevice, stream_));
        break;
      default:
        throw EnforceNotMet(strcat_("unknown plan step ", s.kind));
    }
  }
}

}  // namespace gloo_amd

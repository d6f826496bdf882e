// executor.cc — see executor.h: construction (plan choice, the rank exchange,
// arenas, mailboxes, imports) and teardown.  Runs: executor_run.cc.
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
#include "executor_internal.h"

namespace gloo_amd {

using namespace exec;  // executor_internal.h

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

// The environment knob that chooses which plan a collective executes
// (INTEGRATION.md §4): GLOO_AMD_MESH.  It is read here and nowhere else;
// every rank must read it alike, and the "where" exchange carries it with a
// fingerprint of the plan it produces, so a rank-inconsistent choice is
// refused on every rank instead of running mismatched step lists.
struct RouteKnobs {
  bool mesh = true;  // GLOO_AMD_MESH: derived mesh plans (mesh.cc) where P allows
  int32_t bits() const { return mesh ? 1 : 0; }
};
RouteKnobs routeKnobs() {
  const char* e = std::getenv("GLOO_AMD_MESH");
  RouteKnobs k;
  k.mesh = !(e && e[0] == '0');
  return k;
}
std::string knobText(int32_t bits) { return strcat_("GLOO_AMD_MESH=", bits & 1 ? 1 : 0); }

// The plan `algo` executes as, given the knob.  A custom op is called as the
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
  if (mesh && algo == GLOO_HIP_ALGO_RING_CHUNKED) planAlgo = GLOO_HIP_ALGO_RING_CHUNKED_MESH;
  if (mesh && (algo == GLOO_HIP_ALGO_HALVING_DOUBLING || algo == GLOO_HIP_ALGO_REDUCE_SCATTER || isNewStyle(algo) ||
               algo == GLOO_HIP_ALGO_BCUBE))
    planAlgo = algo | GLOO_HIP_ALGO_MESH;
  // Ring-chunked on its ring route (the mesh off, or P > 8): three inboxes
  // per channel, so each round reduces and forwards in one pass (plan.cc
  // planRingChunkedPipe; the reference's bytes; 3.4 % faster than the
  // literal two-inbox order at 256 MiB per rank).
  if (planAlgo == GLOO_HIP_ALGO_RING_CHUNKED && !custom) planAlgo = GLOO_HIP_ALGO_RING_CHUNKED_PIPE;
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

}  // namespace

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

// This rank's proposal for the sliced interpreter (executor.h): one
// workgroup per sliceBytes() of its largest message, if its own plan and the
// messages its peers write into its arena slice consistently (sliceable); 0
// otherwise.  All ranks then take the smallest proposal, so they agree.
int32_t PlanExecutor::proposeSlices(const std::set<int>& recvPeers, int sliceCap) {
  const int me = ctx_->rank, P = ctx_->size;
  int32_t proposal = 0;
  if (interpMode_ && mailbox_ && !anyRemote_ && !hostArena_) {
    size_t maxMsg = 0;
    for (const Step& s : plan_.steps) maxMsg = std::max(maxMsg, (size_t)s.length * es_);
    const size_t want = std::min<size_t>(sliceCap, std::max<size_t>(1, (maxMsg + sliceBytes() - 1) / sliceBytes()));
    // above sliceCap slices of sliceCapBytes() graph replay is as fast
    if (maxMsg <= (size_t)sliceCap * sliceCapBytes()) {
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
  return proposal;
}

// Every plan peer's record: its mailbox (a channel uses mailboxes when both
// ends signal from the device and have one — both ends decide alike), and,
// for a peer this rank sends to, its inbox arena and the region the peer
// declared there for our messages (its own plan).
void PlanExecutor::mapPeers(const std::vector<std::vector<char>>& arenas, const std::set<int>& planPeers,
                            const std::set<int>& sendPeers) {
  const int me = ctx_->rank, P = ctx_->size;
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
          // a pool slab (the peer also talks to other processes): VMM access
          if (pr.mailboxSlabId) ipc::grantAccess(reinterpret_cast<void*>(pr.mailboxPtr), ctx_->device());
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
        // a pool slab (the peer also talks to other processes): VMM access
        if (!pr.host && pr.slabId) ipc::grantAccess(reinterpret_cast<void*>(pr.ptr), ctx_->device());
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
}

// Device signalling: the ticket counters, the completion word, and whether
// runs replay a hipGraph.  (The copy engines, fold + forward, copy grids and
// store flavours are fixed: executor.h, each from a measured A/B.)
void PlanExecutor::configureDeviceLaunches() {
  const int me = ctx_->rank, P = ctx_->size;
  (void)me;
  (void)ctx_->counterDevicePtr(inst_, 0, 0, 0);  // register the control block now
  ctx_->errorWord(me).store(0);
  const size_t tickets = std::max<size_t>(256, (size_t)P * GLOO_HIP_NUM_SLOTS * sizeof(unsigned));
  GLOO_AMD_HIP_ALLOC(hipMalloc(&ticket_, tickets));
  // zeroed on the executor's stream and complete before any copy kernel
  // (a plain hipMemset goes to the null stream, which a non-blocking
  // stream does not wait for)
  GLOO_AMD_HIP_CHECK(hipMemsetAsync(ticket_, 0, tickets, stream_));
  // Graph replay pays off where the host is the bottleneck: a plan with
  // steps that are not fused one-workgroup launches.  A mesh plan (a few
  // launches per call) whose messages reach graphBytes() (4 MiB) is
  // device-bound instead: the host's eager enqueue stays ahead,
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
  if (ownStream_) {
    GLOO_AMD_HIP_ALLOC(hipHostMalloc(reinterpret_cast<void**>(&hostDone_), 64,
                                     hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
    __atomic_store_n(hostDone_, 0, __ATOMIC_RELEASE);
    GLOO_AMD_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hostDoneDev_), hostDone_, 0));
    if (interpMode_) {
      GLOO_AMD_HIP_ALLOC(hipMalloc(&doneTicket_, 64));
      GLOO_AMD_HIP_CHECK(hipMemsetAsync(doneTicket_, 0, 64, stream_));
    }
  }
  if (graphMode_) {
    GLOO_AMD_HIP_ALLOC(hipMalloc(&epoch_, sizeof(uint64_t)));
    GLOO_AMD_HIP_CHECK(hipMemsetAsync(epoch_, 0, sizeof(uint64_t), stream_));
  }
  GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
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
  try {
    plan_ = planFor(planAlgo_, me, P, count_, (int)inputs_.size(), (int)ptrs_.size(), es_, maxSegmentBytes_,
                    recvElems_);
  } catch (const std::runtime_error&) {
    // AllreduceBcube has a mesh form only where every rank ends with the same
    // expression trees (P a power of the base, counts of at least P or so;
    // mesh.cc throws otherwise): the reference route then, decided alike on
    // every rank since the derivation depends only on (P, count, base)
    if (planAlgo_ != (GLOO_HIP_ALGO_BCUBE | GLOO_HIP_ALGO_MESH)) throw;
    planAlgo_ = GLOO_HIP_ALGO_BCUBE;
    plan_ = planFor(planAlgo_, me, P, count_, (int)inputs_.size(), (int)ptrs_.size(), es_, maxSegmentBytes_,
                    recvElems_);
  }
  GLOO_AMD_HIP_CHECK(hipSetDevice(ctx_->device()));
  classifyPointers();
  inst_ = ctx_->acquireInstance();
  GLOO_AMD_HIP_CHECK(hipSetDevice(ctx_->device()));
  GLOO_AMD_HIP_CHECK(hipEventCreateWithFlags(&doneEvent_, hipEventDisableTiming));
  if (stream) {
    stream_ = stream;
  } else {
    // The executor's own stream (one stream per context was shared
    // by every algorithm given none, so two algorithms run from two threads
    // in different orders on two ranks queued each one's device-side waits
    // behind the other's; the reference gives each op its stream,
    // gloo/cuda.h:102-105)
    GLOO_AMD_HIP_CHECK(hipStreamCreateWithFlags(&ownedStream_, hipStreamNonBlocking));
    stream_ = ownedStream_;
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
    int64_t gpu;  // the GPU's PCI location: ranks of any process on one GPU share it
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
    Where w{ctx_->pid(), ctx_->device(), knobs.bits(), planAlgo_, callHash, exchangeHash(plan_), gpuLocation(ctx_->device())};
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
      GLOO_AMD_ENFORCE(false, "rank-inconsistent collective: ", why, ". The plan-selecting knob (GLOO_AMD_MESH) "
                       "and the call's arguments must be equal on every rank");
    }
  }
  peers_.resize(P);
  bool sharesDeviceInProcess = false;
  for (int peer : planPeers) {
    const Where& w = where.at(peer);
    peers_[peer].pid = w.pid;
    peers_[peer].device = w.device;
    if (w.pid == ctx_->pid() && w.device == ctx_->device()) sharesDeviceInProcess = true;
    if (w.pid != ctx_->pid()) crossProcess_ = true;
  }
  // Stream-ordered device-side signals, unless another rank of this process
  // shares this GPU: those ranks wait on the host (their launches need not
  // be co-resident)
  deviceSignal_ = !sharesDeviceInProcess;
  // Any peer that writes this rank's inboxes — another GPU (over xGMI),
  // another process (through its own mapping), or another rank of this
  // process on this same GPU (its own stream) — writes them in fine-grained
  // memory, so no stale cache line can be read on the receiving side.
  // Two measurements with coarse-grained inboxes on one MI355X:
  //  - two processes: after an executor of the same size had run, the
  //    importer read the previous contents through its mapping even after a
  //    device synchronise (bench.py config-3 variants back to back);
  //  - twelve ranks as threads (BCUBE, GPUTEST_r05, seen once): the wrong
  //    value is exactly what rank 8's phase-1 fold of the SECOND run gives if
  //    it read arena element 5 as it stood at the end of the first run (rank
  //    10's phase-2 message, which shares that offset) instead of rank 9's
  //    new phase-1 message the host counter had announced
  //    (tests/test_newstyle_plan.py::test_bcube_p12_stale_inbox_read_explains_r05);
  //    the protocol orders that read, and isolated probes of the cache and
  //    host-function paths did not reproduce it.
  // A plan reuses arena offsets for different messages of one run, so a
  // line cached by one step's read is wrong for a later step's.
  GLOO_AMD_ENFORCE(workspace == GLOO_HIP_WORKSPACE_DEVICE || workspace == GLOO_HIP_WORKSPACE_HOST,
                   "unknown workspace ", workspace);
  hostArena_ = workspace == GLOO_HIP_WORKSPACE_HOST;
  fineArena_ = !hostArena_ && !recvPeers.empty();

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
  if (deviceSignal_) {
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
  // rank's proposal for the sliced form (proposeSlices).
  {
    const char* im = std::getenv("GLOO_AMD_INTERP");
    const char* gm = std::getenv("GLOO_AMD_GRAPH");
    interpMode_ = deviceSignal_ && !(im && std::string(im) == "0") && !(gm && std::string(gm) == "1") &&
                  interpBytes() > 0 && !custom_;
  }
  // The sliced interpreter's slices spin until their peer slices run, so
  // every launch of the ranks on one GPU must be resident at once.  Measured
  // on one MI355X (256 CUs): 2 ranks x 128 slices and 8 x 32 ran, 4 x 128
  // timed out in every rank's device wait (profiles/round5/r5at_slices_p2.jsonl).
  // So the ranks sharing this GPU split its CUs: at most CUs / ranks slices
  // each (below GLOO_AMD_INTERP_MAX_SLICES), the same on every rank of the GPU.
  int ranksHere = 0;
  for (int r = 0; r < P; r++) ranksHere += where[r].gpu == where[me].gpu;
  const int32_t proposal = proposeSlices(recvPeers, coResidentSlices(ctx_->device(), ranksHere));
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

  mapPeers(arenas, planPeers, sendPeers);
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
  if (deviceSignal_) configureDeviceLaunches();
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
    if (doneTicket_) GLOO_AMD_HIP_RELEASE(hipFree(doneTicket_));
    doneTicket_ = nullptr;
    if (hostDone_) GLOO_AMD_HIP_RELEASE(hipHostFree(hostDone_));
    hostDone_ = hostDoneDev_ = nullptr;
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

}  // namespace gloo_amd

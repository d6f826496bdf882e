// executor.h — runs one rank's plan on its GPU.
//
// The device-side twin of the reference's GPU algorithms
// (gloo/cuda_allreduce_ring_chunked.cc:130-273 and friends) with the inboxes
// in device memory (the CudaDeviceWorkspace flavour, gloo/cuda_workspace.h:20-31)
// on every rank:
//   SEND        hipMemcpyAsync into the peer's inbox (IPC-mapped or same
//               process), over xGMI when the peer is another GPU, then a
//               stream-ordered host function bumps the arrival counter;
//   WAIT_*      host waits on the control-block counter (bounded by the
//               context timeout -> IoException);
//   REDUCE      the HIP chunk-reduce kernel on the rank's stream, reading the
//               local inbox from HBM (never a peer's memory);
//   NOTIFY      stream-ordered counter bump, i.e. only after every reduction
//               enqueued before it has finished reading the inbox.
// Only the wait steps block the host; copies and kernels stay asynchronous,
// so a rank's chunk reductions queue back to back on its stream.
//
// Device signalling (default whenever no other rank shares this rank's GPU
// inside the same process): SEND / NOTIFY become a one-wave signal kernel
// writing the channel's next sequence number, WAIT_* a one-wave wait kernel
// (signal.h) — the whole plan is enqueued without a single host round trip.
// Within one process, ranks that share a GPU share its hardware queues, where
// a spinning wait could block the very signal it waits for; those ranks keep
// the host-side waits.  Both styles write the same monotonically increasing
// sequence numbers, so they interoperate.
//
// hipGraph replay (device signalling; GLOO_AMD_GRAPH=auto, the default, for
// plans with unfused steps, except mesh plans with messages of 4 MiB or
// more; =1 always): once a plan has run with the same buffers, the next run() captures the whole
// enqueue — epoch bump, waits, copies, reductions, signals — into a hipGraph
// and every later run() is ONE hipGraphLaunch.  Sequence numbers are
// replayable (signal.h: base + epoch * perRun with a device-side run epoch),
// so the graph never needs its kernel arguments updated.  New buffers
// (setBuffers) drop the graph; profiling runs are enqueued eagerly.
//
// Workspace (gloo/cuda_workspace.h:20-31): DEVICE inboxes in HBM (default),
// or HOST inboxes in pinned host memory shared by the node's ranks (POSIX shm
// registered with hipHostRegister), the placement of a transport that
// receives from a socket/NIC.  Peers write HOST inboxes over PCIe; REDUCE
// reads them in place (zero-copy) and accumulates into the device buffer.
//
// Copy engine of a SEND (device signalling): copy_signal_kernel, one launch
// that copies and publishes the arrival itself, in an eager enqueue and for
// batches; hipMemcpyAsync + signal kernel inside a captured graph (the
// PlanExecutor members below say why, with the measurements).
//
// One-launch interpreter (device signalling, GLOO_AMD_INTERP, default on):
// when every message of the plan is at most the fuse limit
// (GLOO_AMD_FUSE_BYTES, 64 KiB) and no operand lives on another GPU of this
// process, the steps are resolved once into a device-resident InterpStep
// list (signal.h) and every run() is ONE one-workgroup launch walking it —
// a small allreduce costs its cross-rank hops, not a kernel boundary each.
// Larger plans (messages up to GLOO_AMD_INTERP_MAX_SLICES (32) x
// 2 x GLOO_AMD_INTERP_SLICE_BYTES) run SLICED when every rank's plan allows
// it: one workgroup per GLOO_AMD_INTERP_SLICE_BYTES (32 KiB) of the largest
// message, at most the cap (also at most the GPU's CUs / the ranks on it),
// each running the whole plan on its slice of every step with its own flag
// words (signal.h).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <map>
#include <set>
#include <string>
#include <memory>
#include <utility>
#include <vector>

#include "gloo_amd/common.h"
#include "gloo_amd/context.h"
#include "gloo_amd/ipc.h"
#include "gloo_amd/plan.h"
#include "gloo_amd/signal.h"

namespace gloo_amd {

class PlanExecutor {
 public:
  // stream == nullptr: the executor owns a stream and run() returns with the
  // outputs complete (synchronizeDeviceOutputs_, gloo/cuda_allreduce_ring_chunked.cc:52).
  // Otherwise work is enqueued on `stream` and the caller synchronises
  // (docs/cuda.md:6-13 of the reference).
  PlanExecutor(std::shared_ptr<Context> ctx, int algo, int op, int dtype,
               const std::vector<void*>& ptrs, size_t count, const std::vector<int>& recvElems,
               hipStream_t stream, const std::vector<void*>& inputs = {}, size_t maxSegmentBytes = 0,
               int workspace = 0 /* GLOO_HIP_WORKSPACE_DEVICE */);

  // Function-style calls (gloo::allreduce(opts)) reuse one executor for a
  // given option set and rebind the buffers before each run.
  void setBuffers(const std::vector<void*>& inputs, const std::vector<void*>& outputs);
  // ... and to the call's stream (nullptr: the executor's own stream, and
  // run() returns with the outputs complete).  Work on the new stream is
  // ordered after everything this executor queued before.
  void setStream(hipStream_t stream);
  // One stream per output pointer, the reference's `streams` argument
  // (gloo/cuda_allreduce_ring_chunked.cc:55-67, GLOO_ENFORCE_EQ(streams.size(),
  // ptrs.size())): run() orders its use of pointer i after the work already
  // queued on streams[i] (docs/cuda.md:7-11) and, on return, every
  // streams[i] is ordered after the collective, so the caller synchronises
  // with any of them.  The plan itself runs on streams[0].  Empty: the
  // executor's own stream, and run() returns with the outputs complete.
  // The executor never holds a caller's stream past run(): later waits use
  // an event it owns, so a caller may destroy its streams between calls.
  void setStreams(const std::vector<hipStream_t>& streams);
  ~PlanExecutor();

  template <typename... Args>
  static std::unique_ptr<PlanExecutor> create(Args&&... args) {
    return std::unique_ptr<PlanExecutor>(new PlanExecutor(std::forward<Args>(args)...));
  }
  PlanExecutor(const PlanExecutor&) = delete;
  PlanExecutor& operator=(const PlanExecutor&) = delete;

  void run();

  const Plan& plan() const { return plan_; }
  int planAlgorithm() const { return planAlgo_; }
  hipStream_t stream() const { return stream_; }
  bool deviceSignalling() const { return deviceSignal_; }
  bool fineGrainedArena() const { return fineArena_; }
  bool hostArena() const { return hostArena_; }
  bool foldSendUsed() const { return foldSendUsed_; }
  // True when the last run() was a replay of the captured hipGraph (a run
  // with profiling events on is enqueued eagerly even while a graph exists).
  bool graphed() const { return replayed_; }
  // True once run() executes the plan as one interpreter launch.
  bool interpreted() const { return interpMode_ && interpCount_ > 0; }
  // Workgroups of that launch: > 1 when every rank runs the plan sliced.
  int interpSlices() const { return slices_; }
  // run() on the executor's own stream: it returns with the outputs complete
  // (through the device-published done word); otherwise on the caller's
  bool ownStream() const { return ownStream_; }
  // Why graph capture was abandoned (empty if it was not).
  const std::string& graphError() const { return graphError_; }
  // Host time spent blocked in WAIT steps during the last run(), seconds.
  double lastWaitSeconds() const { return waitSeconds_; }
  // When enabled, every REDUCE of run() is bracketed by HIP events; after the
  // run: summed kernel seconds and algorithmic bytes (3 * n * sizeof(T)).
  void setProfiling(bool on) { profiling_ = on; }
  // Device stamps instead (reduce.hip stamp_begin / stamp_end): every REDUCE
  // and FOLD kernel of a run records its first-workgroup start and
  // last-workgroup end on the GPU's constant clock, which also works inside a
  // replayed hipGraph (events around the steps would force eager runs).
  // After each run the same accessors report the summed kernel durations.
  // A fused fold + forward launch is stamped as it ships (its forward stores
  // inside the span); its bytes count as the fold's.
  void setStamping(bool on);
  double lastReduceSeconds() const { return reduceSeconds_; }
  double lastReduceBytes() const { return reduceBytes_; }
  size_t lastReduceCount() const { return reduceCount_; }

 private:
  // Pointers into an arena, by element offset.
  char* arenaAt(uint64_t elems, uint64_t) const { return arena_ + elems * es_; }
  char* peerAt(int peer, uint64_t elems, uint64_t) const { return peers_[peer].base + elems * es_; }
  struct Peer {
    char* base = nullptr;
    bool ipc = false;
    int pid = -1;
    int device = -1;
  };
  void waitCounter(std::atomic<uint64_t>& c, uint64_t target, int peer, int slot);
  // Enqueue run `r` (1-based) of the plan.  graph: sequence numbers read the
  // device epoch (a capture); otherwise they are computed on the host.
  void enqueue(uint64_t r, bool graph);
  void tryCapture(uint64_t r);
  void dropGraph();
  // Resolve the plan into interpSteps_ for the current buffers; interpCount_
  // = 0 if some step is not an interpreter shape (the plan runs enqueued).
  void buildInterp();
  Seq seqOf(size_t step, uint64_t r, bool graph) const;
  // Where a device-side signal to `peer` lands / a device-side wait for
  // `peer` polls: the receiver's device mailbox when both ends have one,
  // else the counter in the node's host control block.
  bool mailboxWith(int peer) const;
  uint64_t* sigFlag(int peer, int slot);
  uint64_t* waitFlag(int peer, int slot);
  hipStream_t auxStream(size_t k);
  hipEvent_t forkEvent(size_t k);
  char* userPtr(int j) const { return static_cast<char*>(ptrs_[j]); }

  std::shared_ptr<Context> ctx_;
  int algo_, op_, dtype_;
  bool custom_ = false;  // op_ is a registered custom reduction (gloo_hip_register_op)
  int planAlgo_;  // the plan executed (RING_CHUNKED may run as RING_CHUNKED_MESH)
  size_t es_;
  std::vector<void*> ptrs_;     // outputs (the reference's ptrs_ / out)
  std::vector<void*> inputs_;   // separate inputs (new-style allreduce), may be empty
  size_t count_;
  size_t maxSegmentBytes_ = 0;
  std::vector<int> recvElems_;
  // Local pointers on other GPUs of this process (the reference's
  // multi-GPU-per-process form, gloo/cuda_collectives_native.h:22-146):
  // their ranges are pulled into local staging buffers by peer copies before
  // the fused local fold, and the broadcast pushes back by peer copies.
  std::vector<bool> outRemote_, inRemote_;
  std::vector<char*> outStage_, inStage_;
  bool anyRemote_ = false;
  void classifyPointers();
  // construction phases (executor.cc)
  int32_t proposeSlices(const std::set<int>& recvPeers, int sliceCap);
  void mapPeers(const std::vector<std::vector<char>>& arenas, const std::set<int>& planPeers,
                const std::set<int>& sendPeers);
  void configureDeviceLaunches();
  Plan plan_;
  uint64_t inst_;
  char* arena_ = nullptr;       // device-visible address of this rank's inboxes
  bool crossProcess_ = false;   // a plan peer lives in another process: arena and mailbox are IPC pool slabs
  ipc::Slab* arenaSlab_ = nullptr;
  ipc::Slab* mailboxSlab_ = nullptr;
  size_t arenaBytes_ = 0;       // its allocated size (whole 2 MiB granules)
  bool hostArena_ = false;      // inboxes in shared pinned host memory (HOST workspace)
  struct HostShm;
  std::unique_ptr<HostShm> arenaShm_;
  std::vector<std::unique_ptr<HostShm>> peerShm_;
  hipStream_t stream_ = nullptr;
  bool ownStream_ = false;            // stream_ is the executor's own: run() returns with outputs complete
  hipStream_t ownedStream_ = nullptr;  // the stream runs use when given none: the executor's own
  std::vector<hipStream_t> sideStreams_;  // the caller's streams of pointers 1.. (setStreams)
  std::vector<hipEvent_t> sideEvents_;
  hipEvent_t doneEvent_ = nullptr;     // recorded on stream_ at the end of a run on a caller's stream
  bool donePending_ = false;           // ... and not yet waited for on the host
  // Host-wait for everything this executor has queued, without touching a
  // caller's stream (it may be gone).
  void quiesce();
  // Tear-down (collective when P > 1): the destructor, and a construction
  // that failed on any rank (every rank fails together at the ready point).
  void release();
  bool released_ = false;
  std::vector<Peer> peers_;
  std::map<std::pair<int, int>, uint64_t> remoteRegion_;  // (peer, slot) -> elts into peer arena
  // Sequence numbers.  Channel (peer, slot) carries perRun messages per run;
  // the j-th message of run r on it has number
  //   baseline + (r - 1) * perRun + j + 1 = base + r * perRun
  // with base = baseline + j + 1 - perRun precomputed per step (StepSeq).
  struct StepSeq {
    uint64_t base = 0, perRun = 0;
  };
  std::vector<StepSeq> stepSeq_;
  uint64_t runs_ = 0;          // runs enqueued so far
  uint64_t* epoch_ = nullptr;  // device: the run being executed (graph replay)
  hipGraphExec_t graphExec_ = nullptr;
  bool replayed_ = false;      // the last run() launched graphExec_
  bool graphMode_ = false;
  uint64_t epochRuns_ = 0;     // the device epoch once the work queued so far has run
  uint64_t stableRuns_ = 0;    // runs since the buffers last changed
  std::string graphError_;
  bool deviceSignal_ = false;  // stream-ordered signal/wait kernels instead of host waits
  bool interpMode_ = false;            // the interpreter may run this plan
  bool interpDirty_ = true;            // interpSteps_ predates the current buffers
  InterpStep* interpSteps_ = nullptr;  // device copy of the resolved steps
  // A run on the executor's own stream publishes its completion here (the
  // interpreter's done signal, or a signal kernel behind an eager or replayed
  // run) and run() spins on it instead of synchronising the stream: a launch + stream synchronise costs 10.3 µs on
  // MI355X, a kernel's own store seen by a spinning host 7.4 µs
  // (tools/launch_probe, profiles/round5/r5ac_*).
  uint64_t* hostDone_ = nullptr;     // coherent pinned host memory
  uint64_t* hostDoneDev_ = nullptr;  // ... its device address
  unsigned* doneTicket_ = nullptr;   // device: the workgroups' ticket counter
  bool spinSkip_ = false;            // the last run outlasted the spin window: synchronise instead
  int interpCount_ = 0;
  int slices_ = 1;                     // workgroups of the (sliced) interpreter, agreed by all ranks
  uint64_t* mailbox_ = nullptr;           // this rank's incoming counters, (sender, slot), fine-grained HBM
  std::vector<uint64_t*> peerMailbox_;    // peers' mailboxes (nullptr: that channel uses the host block)
  std::vector<bool> peerMailboxIpc_;
  bool fineArena_ = false;     // inbox arena in fine-grained (cross-device coherent) memory
  // Fixed launch choices, each from a measured A/B (the knobs
  // that switched them are gone):
  //  - a SEND in an eager enqueue, a batch of SENDs to several peers, and a
  //    lone same-GPU SEND of 16 MiB or more run on the copy+signal kernel; a
  //    lone SEND inside a captured graph is hipMemcpyAsync + signal kernel;
  //  - workgroups per copy: 64 to a peer on another GPU (a few dozen saturate
  //    an xGMI link), 128 to a peer on this GPU (ranks sharing a GPU run
  //    their copies concurrently and whole-chip grids convoy: HD 16 MiB per
  //    rank 45.4-47.1 vs 47.2-48.2 us at 2 ranks against 64, 64 MiB
  //    226-230 vs 240-247 us at 4 ranks, profiles/round4/r4j_*);
  //  - a local COPY (a mesh result out of its inbox) runs on the copy kernel
  //    with at most 256 workgroups and plain stores (up to 11 % per call
  //    faster than the blit, and than `nt`, profiles/round5/r5o_*);
  //  - REDUCE steps store plain (HD on the reference route 3-4 % faster per
  //    call at 64 and 256 MiB per rank, profiles/round5/r5u_*);
  //  - a FOLD's result SENDs ride in the fold's pass (launchFoldSend).
  static constexpr unsigned kCopyBlocksRemote = 64;
  static constexpr unsigned kCopyBlocksLocal = 128;
  static constexpr unsigned kCopyOutBlocks = 256;
  unsigned copyBlocksFor(int peer) const {
    return peers_[peer].device == ctx_->device() ? kCopyBlocksLocal : kCopyBlocksRemote;
  }
  bool foldSendUsed_ = false;    // ... and some enqueue did so
  unsigned* ticket_ = nullptr;   // copy_signal_kernel tickets, one counter per (peer, slot)
  std::vector<hipStream_t> aux_;        // forked SEND batches (memcpy engine)
  std::vector<hipEvent_t> forkEvents_;
  double waitSeconds_ = 0;
  bool profiling_ = false;
  bool stamping_ = false;
  uint64_t* stamps_ = nullptr;    // 2 x stampSlots_ device words: (start min, end max) per reduce step
  int stampSlots_ = 0;
  std::vector<double> stampBytes_;  // algorithmic bytes per slot
  std::vector<size_t> stampCount_;  // chunk reductions per slot (a k-source fold counts k - 1, as with events)
  std::map<size_t, int> stampSlotOf_;  // plan step -> slot
  void readStamps();
  std::vector<hipEvent_t> events_;
  size_t evUsed_ = 0;
  double reduceSeconds_ = 0, reduceBytes_ = 0;
  size_t reduceCount_ = 0;
};

}  // namespace gloo_amd

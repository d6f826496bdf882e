// signal.h — stream-ordered cross-rank signalling kernels (internal).
//
// A rank's chunk exchange is a sequence of (copy, signal) on the sender's
// stream and (wait, reduce) on the receiver's stream.  These kernels make
// both ends stream-ordered, so a whole plan is enqueued — and captured into
// a hipGraph — without host round trips:
//   signal: system-scope release, then the flag word := value
//   wait:   poll the flag (relaxed) until >= target (signed difference, so a
//           target below the counter is met at once), sleeping between polls;
//           ONE system-scope acquire after the match; give up after
//           `timeoutTicks` of the 100 MHz realtime counter and set *err (the
//           host raises IoException).
// Flags are 64-bit counters in the node's shared control block, registered
// with hipHostRegister so every GPU of every rank can address them.
//
// Replayable sequence numbers: every value a kernel waits for or writes is
//   Seq{base, perRun}.value(epoch) = base + epoch * perRun   (mod 2^64)
// where `epoch` is the rank-local run counter in device memory that the
// first node of each run increments (launchEpochBump).  A captured plan can
// therefore be replayed unchanged: run r computes its own targets.  With a
// null epoch pointer the value is `base` (host-computed).
#pragma once

#include <algorithm>

#include <hip/hip_runtime_api.h>

#include "gloo_amd.h"

#include <cstdint>

namespace gloo_amd {

struct Seq {
  uint64_t base = 0;
  uint64_t perRun = 0;
};

hipError_t launchEpochBump(uint64_t* epoch, hipStream_t stream);            // *epoch += 1
hipError_t launchEpochSet(uint64_t* epoch, uint64_t value, hipStream_t stream);  // *epoch = value
hipError_t launchSignal(uint64_t* flag, Seq value, const uint64_t* epoch, hipStream_t stream);
hipError_t launchWait(const uint64_t* flag, Seq target, const uint64_t* epoch, uint64_t timeoutTicks,
                      uint32_t* err, hipStream_t stream);
// Diagnosis: out[0..3] = the word at p by a plain load, a system-scope
// atomic load, a non-temporal load after a system-scope acquire, and a plain
// load again (out: host-visible memory).
hipError_t launchProbe(const uint64_t* p, uint64_t* out, hipStream_t stream);

// One-workgroup fused step for small messages (reduce.hip): optionally wait
// for `*waitFlag >= wait`, then dst[i] = dst[i] op src[i] (op 0: copy), then
// optionally signal `*sigFlag = sig`.  Returns a gloo_hip status.
int launchFusedSmall(int op, int dtype, void* dst, const void* src, size_t n, const uint64_t* waitFlag, Seq wait,
                     uint64_t timeoutTicks, uint32_t* err, uint64_t* sigFlag, Seq sig, const uint64_t* epoch,
                     hipStream_t stream);

// Peer copy + fused arrival signal (reduce.hip): `grid` workgroups copy
// `bytes` from src (local) to dst (a peer's inbox); the workgroup that takes
// the launch's last ticket resets the counter (zero between launches; one
// counter per channel, launches on it stream-ordered) and publishes *flag =
// seq.  copySignalGrid() sizes the grid (capped at maxBlocks: a link, not
// HBM, bounds a peer copy).
unsigned copySignalGrid(size_t bytes, unsigned maxBlocks);
int launchCopySignal(void* dst, const void* src, size_t bytes, uint64_t* flag, Seq seq, unsigned* ticketCounter,
                     const uint64_t* epoch, unsigned grid, hipStream_t stream);

// Up to kMaxCopyEntries such copies in ONE launch, all in flight together
// (a mesh schedule's sends to every peer: one xGMI link each).
constexpr int kMaxCopyEntries = 8;
struct CopyDesc {
  void* dst;
  const void* src;
  size_t bytes;
  uint64_t* flag;    // nullptr: a plain copy, no arrival signal
  Seq seq;
  unsigned* ticket;  // this entry's ticket counter (zero at launch)
  unsigned blocks;   // copySignalGrid(bytes, ...)
};
// The stores of a flag-less (local) entry.  `nt` streams the bytes past the
// die's Infinity Cache; plain stores leave them there for the next reader.
// A collective's copy-out is re-read by the caller's next use of its buffer
// (and by the next call's fold), and plain stores made the HD call 3-11 %
// faster (profiles/round5/r5n_*, r5o_*).  Signalled entries
// (sends) keep `nt` / write-through.
enum CopyStore { kCopyStoreNT = 0, kCopyStoreWT = 1, kCopyStorePlain = 2 };
int launchCopySignalMulti(const CopyDesc* d, int n, const uint64_t* epoch, hipStream_t stream,
                          CopyStore localStore = kCopyStoreNT);

// Wait for several flags in one launch (one lane per flag), then ONE
// system-scope acquire.  n <= kMaxWaitEntries.
constexpr int kMaxWaitEntries = 16;
hipError_t launchWaitMulti(const uint64_t* const* flags, const Seq* targets, int n, const uint64_t* epoch,
                           uint64_t timeoutTicks, uint32_t* err, hipStream_t stream);

// One-launch plan interpreter (reduce.hip) for plans whose every message is
// small: a workgroup walks a precompiled step list — copies, sends (copy,
// drain, one system-scope release, flag store), signals, waits (one lane
// polls, one acquire, barrier) and folds — with a workgroup barrier between
// steps.  A small allreduce becomes a single kernel: its device time is the
// cross-rank hops, not the kernel boundaries between them.  Sequence values
// are base + run * perRun (the eager numbering).  A wait that times out sets
// *err and ends the workgroup.
//
// Sliced form (`slices` > 1 workgroups): workgroup g runs the WHOLE list on
// slice g of every step — elements [lo, hi) with q = ceil(n / slices) rounded
// up to 16 bytes, lo = min(n, g q), hi = min(n, lo + q) — and signals / waits
// on its own flag word `flag + g`.  The slices never meet inside the launch
// (no grid barrier): every rank slices every message alike, so slice g of a
// message is produced, sent, received and consumed by workgroups g alone.  The
// executor proves per plan that each step reads exactly the ranges earlier
// steps or peers wrote (executor_modes.cc sliceable) before choosing it.
enum { kInterpCopy = 0, kInterpSend = 1, kInterpSignal = 2, kInterpWait = 3, kInterpFold = 4 };
struct InterpStep {
  int32_t kind;       // kInterp*
  int32_t mode;       // FOLD: 0 left fold, 1 reverse (acc = s op acc), 2 balanced tree
  int32_t nsrc;       // FOLD: sources
  int32_t flags;      // kInterpDefer: the next step is independent of this one (executor_run.cc buildInterp)
  uint64_t* flag;     // SEND / SIGNAL: the flag written; WAIT: the flag polled (slice 0's)
  uint64_t base, perRun;
  char* dst;
  const char* src[8]; // COPY / SEND: src[0]; FOLD: the sources in order
  uint64_t n;         // elements
};
constexpr int kInterpMaxSteps = 512;
// InterpStep.flags: this step and the next form one batch.  A WAIT then only
// polls (the batch's last wait takes the one acquire and the barrier); a data
// step's memory operations are not drained before the next step, and the
// flags of the batch's SENDs / SIGNALs are published together after the
// batch's last step drains.  Set only where the next step of the same kind
// (wait after wait; data or signal after data or signal) touches no byte this
// one writes and writes no byte it reads.
constexpr int kInterpDefer = 1;
// Sets kInterpDefer on v[0..n) (executor.cc): step i is deferred when step
// i+1 is of the same class (wait / non-wait) and touches nothing that any
// step of the open batch (every step since the last non-deferred one) writes,
// and writes nothing any of them reads.  `es` = bytes per element of `n`.
void markInterpBatches(InterpStep* v, size_t n, size_t es);
// Flag words per (sender, slot) in a device mailbox: one per slice.
constexpr int kMaxSlices = 256;
// done / doneTicket (both or neither): the workgroup that finishes last
// stores `run` into *done (system scope, after every workgroup's release) and
// resets *doneTicket (zero between launches), so a host that owns the stream
// can spin on *done (coherent host memory) instead of synchronising it.
int launchPlanInterp(int op, int dtype, const InterpStep* steps, int nsteps, uint64_t run, uint64_t timeoutTicks,
                     uint32_t* err, int slices, hipStream_t stream, uint64_t* done = nullptr,
                     unsigned* doneTicket = nullptr);

// Multi-source fold in one pass, k <= GLOO_HIP_MAX_SRCS.  mode 0: left fold
// acc = acc op s_j; 1: reverse, acc = s_j op acc; 2: balanced pairwise tree
// over the sources in order (k a power of two).  Returns a gloo_hip status.
// Device-side timing of the reduce kernels (reduce_vec_kernel,
// reduce_multi_vec_kernel): while a stamp slot is set on the calling thread,
// each of those launches folds its first workgroup start into the slot's
// begin shards (min) and its last workgroup end into its end shards (max),
// 100 MHz clock ticks; the kernel's span is max(end shards) - min(begin
// shards) (stampSpan).  A slot is kStampSlotWords words: kStampShards begin
// words, then kStampShards end words, one per kStampLineWords-word (128-B)
// line.  setLaunchStamp returns the previous slot; launchStampInit resets k
// consecutive slots (begin ~0, end 0).
constexpr int kStampShards = 64;
constexpr int kStampLineWords = 16;
constexpr int kStampSlotWords = 2 * kStampShards * kStampLineWords;
inline bool stampSpan(const uint64_t* slot, uint64_t* ticks) {
  uint64_t b = ~0ull, e = 0;
  for (int i = 0; i < kStampShards; i++) {
    b = std::min(b, slot[i * kStampLineWords]);
    e = std::max(e, slot[(kStampShards + i) * kStampLineWords]);
  }
  if (e == 0 || e < b) return false;  // not launched (a fused or empty step)
  *ticks = e - b;
  return true;
}
uint64_t* setLaunchStamp(uint64_t* slot);
// The stores of the element-wise reduce kernels launched on this thread
// (gloo_hip_reduce / reduce3) and multi-source folds (gloo_hip_reduce_multi,
// launchFold): `nt` (default, the chunk-reduce of the headline bench streams
// past the Infinity Cache) or plain (a plan's REDUCE, FOLD or local fold into a
// buffer that is re-read soon).  Returns the previous setting.
bool setReducePlainStores(bool plain);
int launchStampInit(uint64_t* stamps, int k, hipStream_t stream);

// Registered custom reductions (gloo_hip_register_op): op codes
// GLOO_HIP_CUSTOM + i.  customOp fills fn/user and returns true for a
// registered code.
bool isBuiltinOp(int op);
bool customOp(int op, gloo_hip_custom_fn* fn, void** user);

int launchFold(int op, int dtype, void* dst, const void* const* srcs, int k, size_t n, int mode,
               hipStream_t stream);

// Fold + forward (reduce.hip fold_send_kernel): the fold above, with each
// result tile also stored to every fwd[r].dst (peers' inboxes; any
// element-aligned address) in the same pass; the workgroup taking the launch's
// last ticket publishes every non-null fwd[r].flag = seq (epoch-scaled, as
// launchCopySignal).  An entry with dst == nullptr is a credit: its flag is
// published once every read of the fold is complete, and no data moves.
// Built-in ops only.  Returns a gloo_hip status.
struct FwdDesc {
  void* dst;
  uint64_t* flag;
  Seq seq;
};
int launchFoldSend(int op, int dtype, void* dst, const void* const* srcs, int k, size_t n, int mode,
                   const FwdDesc* fwd, int nf, unsigned* ticket, const uint64_t* epoch, hipStream_t stream);

}  // namespace gloo_amd

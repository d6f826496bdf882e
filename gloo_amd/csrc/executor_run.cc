// executor_run.cc — see executor.h: a run of the plan (eager enqueue, graph
// capture and replay, the one-launch and sliced interpreters) and the
// buffer / stream rebinding between runs.  Construction: executor.cc.
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

void bumpCounter(void* p) { static_cast<std::atomic<uint64_t>*>(p)->fetch_add(1, std::memory_order_acq_rel); }

void enqueueBump(hipStream_t s, std::atomic<uint64_t>& c) {
  GLOO_AMD_HIP_CHECK(hipLaunchHostFunc(s, bumpCounter, &c));
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
    if (!ownedStream_) {
      // on the rank's device, whatever device the calling thread has current
      int prev = -1;
      GLOO_AMD_HIP_CHECK(hipGetDevice(&prev));
      if (prev != ctx_->device()) GLOO_AMD_HIP_CHECK(hipSetDevice(ctx_->device()));
      const hipError_t e = hipStreamCreateWithFlags(&ownedStream_, hipStreamNonBlocking);
      if (prev != ctx_->device()) (void)hipSetDevice(prev);
      GLOO_AMD_HIP_CHECK(e);
    }
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
  if (!ownStream_) {  // (the executor's own stream is never the caller's to capture)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    GLOO_AMD_HIP_CHECK(hipStreamIsCapturing(stream_, &cs));
    GLOO_AMD_ENFORCE(cs == hipStreamCaptureStatusNone,
                     "run() on a stream under capture: the executor captures and replays its own graph");
  }
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
  bool spinDone = false;  // this run publishes its completion to hostDone_
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
    spinDone = ownStream_ && doneTicket_ && !anyRemote_ && !profiling_ && !stamping_;
    checkRc(launchPlanInterp(op_, dtype_, interpSteps_, interpCount_, r, timeoutTicks, ctx_->errorWordDevicePtr(me),
                             slices_, stream_, spinDone ? hostDoneDev_ : nullptr, spinDone ? doneTicket_ : nullptr),
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
  // eager or replayed: one signal kernel behind the run stores its number
  // into hostDone_ after a system-scope release (a launch of 0.8 µs on the host
  // against the stream synchronise's 3 µs, launch_probe)
  if (ownStream_ && hostDone_ && !spinDone && !profiling_ && !stamping_) {
    GLOO_AMD_HIP_CHECK(launchSignal(hostDoneDev_, Seq{r, 0}, nullptr, stream_));
    spinDone = true;
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
    // the run's device-published completion word (the interpreter's last
    // workgroup, or the signal kernel behind an eager or replayed run), spun
    // on for up to 2 ms: the stream's completion signal reaches a
    // synchronising host about 3 µs later.  A run that takes longer, or an
    // interpreter whose wait timed out (it ends without the store), falls
    // back to the stream synchronise.
    // (Runs that outlast the window skip the spin until a run is short again,
    // so long collectives do not burn 2 ms of a core each.)
    bool seen = false;
    for (uint32_t i = 0; spinDone && !spinSkip_ && !seen; i++) {
      seen = __atomic_load_n(hostDone_, __ATOMIC_ACQUIRE) >= r;
      if (seen) break;
      __builtin_ia32_pause();
      if ((i & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
    }
    if (!seen) {
      GLOO_AMD_HIP_CHECK(hipStreamSynchronize(stream_));
      if (spinDone) spinSkip_ = std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(1);
    }
    if (deviceSignal_) waitSeconds_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (deviceSignal_ && ctx_->errorWord(me).exchange(0) != 0) {
      // workgroups that timed out left without their done ticket
      if (doneTicket_) (void)hipMemsetAsync(doneTicket_, 0, 64, stream_);
      throw IoException(strcat_("Timed out on rank ", me, " waiting for a peer (device-side wait, ",
                                ctx_->timeout().count(), " ms)"));
    }
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
  // memory round trip per run instead of per step.  (On one GPU it measured
  // within 1 us of the unbatched form; the round trips
  // it removes are the ones over xGMI.)
  markInterpBatches(v.data(), v.size(), es_);
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
  } reduceStores(true);
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
      if (deviceSignal_) {
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
                                          copySignalGrid(lens[k], kCopyOutBlocks)};
        if (nd) checkRc(launchCopySignalMulti(d, nd, epoch, stream_, kCopyStorePlain), "copy kernel (local batch)");
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
        // A lone SEND of >= 16 MiB to a rank on this
        // same GPU goes to the copy kernel with 256 workgroups, which moves
        // HBM -> HBM faster than the blit engine from 16 MiB up (one MI355X:
        // 8.1 vs 9.7 us at 16 MiB, 22.0 vs 26.0 us at 64 MiB kernel time,
        // profiles/round2/r2d_rocprof_copy_engines_segments.csv); below that,
        // and over xGMI, hipMemcpyAsync + signal inside a captured graph
        const bool bigLocal = deviceSignal_ && s.length * es_ >= (16u << 20) && peers_[s.peer].device == ctx_->device();
        // eager (not captured): hipMemcpyAsync into an IPC mapping is the slow
        // path of an eager enqueue, and the copy kernel signals without a
        // write-back since round 3; graph memcpy nodes stay faster
        // (profiles/round3/r3ag_latency_ab_release_and_copy_engine.jsonl)
        const bool eagerKernel = deviceSignal_ && !graph;
        if (bigLocal || eagerKernel) {
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
        if (deviceSignal_ && bytes > 0 && (dst + bytes <= src || src + bytes <= dst)) {
          const CopyDesc d{dst, src, bytes, nullptr, Seq{}, nullptr, copySignalGrid(bytes, kCopyOutBlocks)};
          checkRc(launchCopySignalMulti(&d, 1, epoch, stream_, kCopyStorePlain), "copy kernel (local)");
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
        if (deviceSignal_ && !custom_ && !profiling_ && s.length > 0 &&
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
      case GLOO_HIP_STEP_LOCAL_BCAST: {
        // Output 0 to every other output in ONE pass that reads it once: a
        // one-source fold into output 1 that forwards each tile to outputs
        // 2.. (launchFoldSend; no flags), or the local copy kernel for a
        // single destination.  (k - 1 copies read it k - 1 times: HD with 4
        // pointers of 64 MiB per rank spent 65 % of its time in the local
        // passes, profiles/round6/r6f/multi_pointer_p2.jsonl.)  Outputs on
        // other GPUs of the process keep the peer copies.
        const size_t off = s.dst_off * es_, bytes = s.length * es_;
        if (bytes == 0 || ptrs_.size() < 2) break;
        if (!anyRemote_ && !custom_) {
          const void* src0 = userPtr(0) + off;
          for (size_t j0 = 1; j0 < ptrs_.size(); j0 += 1 + kMaxCopyEntries) {
            const size_t j1 = std::min(ptrs_.size(), j0 + 1 + kMaxCopyEntries);
            if (j1 - j0 == 1) {
              const CopyDesc d{userPtr(j0) + off, src0, bytes, nullptr, Seq{}, nullptr,
                               copySignalGrid(bytes, kCopyOutBlocks)};
              checkRc(launchCopySignalMulti(&d, 1, epoch, stream_, kCopyStorePlain), "copy kernel (broadcast)");
              continue;
            }
            FwdDesc fwd[kMaxCopyEntries];
            int nf = 0;
            for (size_t j = j0 + 1; j < j1; j++) fwd[nf++] = FwdDesc{userPtr(j) + off, nullptr, Seq{}};
            checkRc(launchFoldSend(op_, dtype_, userPtr(j0) + off, &src0, 1, s.length, 0, fwd, nf, nullptr, epoch,
                                   stream_),
                    "broadcast (one-source fold + forwards)");
          }
          break;
        }
        for (size_t j = 1; j < ptrs_.size(); j++)
          GLOO_AMD_HIP_CHECK(hipMemcpyAsync(userPtr(j) + off, userPtr(0) + off, bytes, hipMemcpyDeviceToDevice, stream_));
        break;
      }
      default:
        throw EnforceNotMet(strcat_("unknown plan step ", s.kind));
    }
  }
}

}  // namespace gloo_amd

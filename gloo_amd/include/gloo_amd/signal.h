// signal.h — stream-ordered cross-rank signalling kernels (internal).
//
// A rank's chunk exchange is a sequence of (copy, signal) on the sender's
// stream and (wait, reduce) on the receiver's stream.  These two one-wave
// kernels make both ends stream-ordered, so a whole plan is enqueued without
// host round trips:
//   signal: system-scope release, then the flag word := value
//   wait:   poll the flag (system-scope acquire) until >= target, sleeping
//           between polls; give up after `timeout_ticks` of the 100 MHz
//           realtime counter and set *err (the host raises IoException).
// Flags are 64-bit counters in the node's shared control block, registered
// with hipHostRegister so every GPU of every rank can address them.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace gloo_amd {

hipError_t launchSignal(uint64_t* flag, uint64_t value, hipStream_t stream);
hipError_t launchWait(const uint64_t* flag, uint64_t target, uint64_t timeoutTicks, uint32_t* err,
                      hipStream_t stream);

// One-workgroup fused step for small messages (reduce.hip): optionally wait
// for `waitFlag >= waitTarget`, then dst[i] = dst[i] op src[i] (op 0: copy),
// then optionally signal `*sigFlag = sigValue`.  Returns a gloo_hip status.
int launchFusedSmall(int op, int dtype, void* dst, const void* src, size_t n, const uint64_t* waitFlag,
                     uint64_t waitTarget, uint64_t timeoutTicks, uint32_t* err, uint64_t* sigFlag,
                     uint64_t sigValue, hipStream_t stream);

// Peer copy + fused arrival signal (reduce.hip): `grid` workgroups copy
// `bytes` from src (local) to dst (a peer's inbox); the workgroup that takes
// ticket ticketBase + grid - 1 publishes *flag = seq.  copySignalGrid() sizes
// the grid (capped at maxBlocks: a link, not HBM, bounds a peer copy).
unsigned copySignalGrid(size_t bytes, unsigned maxBlocks);
int launchCopySignal(void* dst, const void* src, size_t bytes, uint64_t* flag, uint64_t seq, unsigned* ticket,
                     unsigned ticketBase, unsigned grid, hipStream_t stream);

}  // namespace gloo_amd

// plan.cc — per-rank schedules of Gloo's reducing algorithms.
//
// Each planner restates one reference algorithm (constructor + run()) as the
// ordered list of steps that rank `rank` performs: one-sided sends into a
// peer's registered inbox region, waits for arrivals, the per-chunk
// reductions, copies and the notification handshakes that guard inbox reuse.
// Offsets, lengths, peers and ORDER are the reference's, so executing a plan
// reproduces the reference's association order bit for bit.  Nothing here
// touches HIP: the same plans drive the device executor (executor.hip) and
// the CPU simulation in tests/.
//
// Inbox regions live in a per-rank "arena" laid out exactly like the
// reference's receive buffers (inbox_[2], recvBuf_, recvBufDist_, outbox_).

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

#include "gloo_amd.h"
#include "gloo_amd/plan.h"
#include "gloo_amd/mesh.h"

namespace gloo_amd {

namespace {

Step mk(int kind, int peer = -1, int slot = 0, int flags = 0, uint64_t dst = 0, uint64_t src = 0,
        uint64_t len = 0) {
  Step s;
  s.kind = kind;
  s.peer = peer;
  s.slot = slot;
  s.flags = flags;
  s.dst_off = dst;
  s.src_off = src;
  s.length = len;
  return s;
}

// floor(log2(x)) as the reference computes it through <cmath> log2 + an
// integer conversion (gloo/allreduce_halving_doubling.h:76 `steps_(log2(P))`).
uint32_t ilog2(uint64_t x) { return static_cast<uint32_t>(std::log2(static_cast<double>(x))); }

// gloo/allreduce_halving_doubling.h:23-33 and gloo/reduce_scatter.h:50-62.
uint32_t reverseLastNBits(uint32_t ctr, uint32_t n) {
  uint32_t bitMask = 1, reversed = 0;
  while (bitMask < (static_cast<uint32_t>(1) << n)) {
    reversed <<= 1;
    if (ctr & bitMask) reversed |= 1;
    bitMask <<= 1;
  }
  return reversed;
}

// Binary-block decomposition for non-power-of-two P
// (gloo/allreduce_halving_doubling.h:39-64, gloo/reduce_scatter.h:21-48).
struct Blocks {
  uint32_t offsetToMyBinaryBlock = 0, myBinaryBlockSize = 0, stepsWithinBlock = 0;
  uint32_t rankInBinaryBlock = 0, nextSmallerBlockSize = 0, nextLargerBlockSize = 0;
};

Blocks binaryBlocks(int rank, int size) {
  Blocks b;
  uint32_t offset = size, blockSize = 1, currentBlockSize = 0, prevBlockSize = 0;
  do {
    if (size & blockSize) {
      prevBlockSize = currentBlockSize;
      currentBlockSize = blockSize;
      offset -= blockSize;
      if (b.myBinaryBlockSize != 0) {
        b.nextLargerBlockSize = currentBlockSize;
        break;
      }
      if (offset <= (uint32_t)rank) {
        b.offsetToMyBinaryBlock = offset;
        b.myBinaryBlockSize = currentBlockSize;
        b.nextSmallerBlockSize = prevBlockSize;
      }
    }
    blockSize <<= 1;
  } while (offset != 0);
  b.stepsWithinBlock = ilog2(b.myBinaryBlockSize);
  b.rankInBinaryBlock = rank % b.myBinaryBlockSize;
  return b;
}

// The in-block recursive-halving geometry shared by allreduce HD and
// reduce-scatter HD (gloo/allreduce_halving_doubling.h:107-157,
// gloo/reduce_scatter.h:155-203).
struct HDGeometry {
  uint64_t steps = 0, chunkSize = 0;
  std::vector<int> dest;
  std::vector<uint64_t> sendOffsets, recvOffsets, sendCounts, recvCounts, regionOff;
  uint64_t bufferOffset = 0;    // arena offset after the in-block regions
  uint64_t stepChunkSize = 0;   // value after the loop
};

HDGeometry hdGeometry(int rank, int size, uint64_t count, const Blocks& bl) {
  HDGeometry g;
  g.steps = ilog2(size);
  const uint64_t chunks = 1ull << g.steps;
  g.chunkSize = (count + chunks - 1) / chunks;
  uint64_t bitmask = 1;
  uint64_t stepChunkSize = g.chunkSize << (g.steps - 1);
  uint64_t sendOffset = 0, recvOffset = 0, bufferOffset = 0;
  for (uint32_t i = 0; i < bl.stepsWithinBlock; i++) {
    const int destRank = rank ^ (int)bitmask;
    g.dest.push_back(destRank);
    const uint64_t so = sendOffset + ((destRank & bitmask) ? stepChunkSize : 0);
    const uint64_t ro = recvOffset + ((rank & bitmask) ? stepChunkSize : 0);
    g.sendOffsets.push_back(so);
    g.recvOffsets.push_back(ro);
    g.sendCounts.push_back(so < count ? std::min(stepChunkSize, count - so) : 0);
    g.recvCounts.push_back(ro < count ? std::min(stepChunkSize, count - ro) : 0);
    g.regionOff.push_back(bufferOffset);
    bufferOffset += stepChunkSize;
    if (rank & bitmask) {
      sendOffset += stepChunkSize;
      recvOffset += stepChunkSize;
    }
    bitmask <<= 1;
    stepChunkSize >>= 1;
  }
  g.bufferOffset = bufferOffset;
  g.stepChunkSize = stepChunkSize;
  return g;
}

// ---------------------------------------------------------------------------
// AllreduceRingChunked (gloo/allreduce_ring_chunked.h:22-236), GPU twin
// gloo/cuda_allreduce_ring_chunked.cc:130-273.
// ---------------------------------------------------------------------------
Plan planRingChunked(int rank, int size, uint64_t count, int nptrs) {
  Plan p;
  if (count == 0) return p;                                   // run() :84-86
  const uint64_t chunks = 2ull * size;                        // ctor :32
  const uint64_t chunkSize = std::max<uint64_t>(256, (count + chunks - 1) / chunks);  // :37
  const int left = (size + rank - 1) % size, right = (rank + 1) % size;
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count));  // :89-91
  if (size == 1) {                                            // :93-99
    if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
    return p;
  }
  p.arena = 2 * chunkSize;  // inbox_[0], inbox_[1] registered with chunkBytes_ (:58-59)
  for (int i = 0; i < 2; i++)
    p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, left, i, 0, i * chunkSize, 0, chunkSize));

  auto span = [&](uint64_t chunkOffset, uint64_t& offset, uint64_t& length) {
    offset = chunkOffset * chunkSize;
    length = chunkSize;
    if (offset + length <= count) {
    } else if (offset < count) {
      length = count - offset;
    } else {
      length = 0;
    }
  };
  auto copyChunkAtOffset = [&](uint64_t chunkOffset) {     // :215-236
    uint64_t offset = (chunkOffset % chunks) * chunkSize, length = chunkSize;
    if (offset + length <= count) {
    } else if (offset < count) {
      length = count - offset;
    } else {
      offset = 0;  // out-of-range chunk still puts 1 element on the wire
      length = 1;
    }
    p.steps.push_back(mk(GLOO_HIP_STEP_SEND, right, (int)(chunkOffset & 1), 0, 0, offset, length));
  };
  auto chunkAt = [&](uint64_t round) {                      // :124-126
    return (uint64_t)((2 * (uint64_t)rank) - (round & ~1ull) + (round & 1ull) + chunks) % chunks;
  };

  copyChunkAtOffset(2 * rank);                              // :102-103
  copyChunkAtOffset(2 * rank + 1);
  for (uint64_t round = 2; round < chunks; round++) {       // :106-158
    const uint64_t co = chunkAt(round);
    uint64_t offset, length;
    span(co, offset, length);
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, left, (int)(co & 1)));
    if (length > 0)
      p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, offset,
                           (co & 1) * chunkSize, length));
    p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, left, GLOO_HIP_SLOT_NOTIFY));
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, right, GLOO_HIP_SLOT_NOTIFY));
    copyChunkAtOffset(co);
  }
  for (uint64_t round = 0; round < chunks - 2; round++) {   // :163-200
    const uint64_t co = chunkAt(round);
    uint64_t offset, length;
    span(co, offset, length);
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, left, (int)(co & 1)));
    if (length > 0)
      p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, offset,
                           (co & 1) * chunkSize, length));
    if (round < chunks - 4) {
      p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, left, GLOO_HIP_SLOT_NOTIFY));
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, right, GLOO_HIP_SLOT_NOTIFY));
      copyChunkAtOffset(co);
    }
  }
  p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, left, GLOO_HIP_SLOT_NOTIFY));      // :205-206
  p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, right, GLOO_HIP_SLOT_NOTIFY));
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
  return p;
}

// ---------------------------------------------------------------------------
// AllreduceRingChunked's own ring route, pipelined: the reference's chunks,
// hops, association and operand order (so its bytes), with each round's
// reduce and the send of its result in ONE pass.
//
// In the reference a round is wait(left) -> reduce -> notify(left) ->
// wait(right's credit) -> send (:141-157): the send re-reads the reduced
// chunk after a kernel boundary, and a pass that reduced and forwarded at
// once would have to wait for the right's credit first.  With the
// reference's two inboxes that order deadlocks (the credit a round waits
// for is the right's credit of the SAME round, tests/test_fold_forward_plan.py).
// With THREE inboxes per channel it cannot: message m goes to the right's
// inbox m % 3 and waits only for the right's credit of message m - 3, which
// the right sends one round earlier, so no credit chain wraps around the
// ring.  Each round is then
//     WAIT_RECV(left) [WAIT_NOTIFY(right)] FOLD(local, inbox) SEND(right) NOTIFY(left)
// and the executor runs FOLD + SEND + NOTIFY as one fold_send launch: every
// tile is reduced, stored locally and into the right's inbox in the same
// pass, and the last workgroup publishes the arrival and the credit.  The
// allgather rounds are the same with a one-source FOLD (a copy).  Every
// consumed message is credited (M per run), the first three sends of a run
// wait for nothing, and the run ends waiting for the credits of its last
// three messages (the reference's trailing notify/wait pair, :205-206), so
// runs need no other barrier.  Messages of a run: M = 2 + (2P - 2) + (2P - 4).
// ---------------------------------------------------------------------------
Plan planRingChunkedPipe(int rank, int size, uint64_t count, int nptrs) {
  Plan p;
  if (count == 0) return p;
  const uint64_t chunks = 2ull * size;
  const uint64_t chunkSize = std::max<uint64_t>(256, (count + chunks - 1) / chunks);
  const int left = (size + rank - 1) % size, right = (rank + 1) % size;
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count));
  if (size == 1) {
    if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
    return p;
  }
  static const int kSlot[3] = {0, 1, 3};  // data slots; GLOO_HIP_SLOT_NOTIFY (2) carries the credits
  p.arena = 3 * chunkSize;
  for (int i = 0; i < 3; i++)
    p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, left, kSlot[i], 0, i * chunkSize, 0, chunkSize));
  auto span = [&](uint64_t chunkOffset, uint64_t& offset, uint64_t& length) {
    offset = chunkOffset * chunkSize;
    length = chunkSize;
    if (offset + length > count) length = offset < count ? count - offset : 0;
  };
  uint64_t sent = 0, consumed = 0;
  // SEND of chunk `co` (:215-236, the 1-element dummy for an empty chunk),
  // after the right's credit of message sent - 3
  auto send = [&](uint64_t co) {
    uint64_t offset = (co % chunks) * chunkSize, length = chunkSize;
    if (offset + length <= count) {
    } else if (offset < count) {
      length = count - offset;
    } else {
      offset = 0;
      length = 1;
    }
    p.steps.push_back(mk(GLOO_HIP_STEP_SEND, right, kSlot[sent % 3], 0, 0, offset, length));
    sent++;
  };
  auto credit = [&] {
    if (sent >= 3) p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, right, GLOO_HIP_SLOT_NOTIFY));
  };
  auto chunkAt = [&](uint64_t round) {
    return (uint64_t)((2 * (uint64_t)rank) - (round & ~1ull) + (round & 1ull) + chunks) % chunks;
  };
  // one round: take the next message from the left into chunk co (reduce:
  // local op incoming, or copy), then forward the result (forward = false:
  // the last allgather rounds send nothing)
  auto round = [&](uint64_t co, bool reduce, bool forward) {
    uint64_t offset, length;
    span(co, offset, length);
    const int in = kSlot[consumed % 3];
    const uint64_t inOff = (consumed % 3) * chunkSize;
    consumed++;
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, left, in));
    if (forward) credit();
    if (length > 0) {
      if (reduce) p.steps.push_back(mk(GLOO_HIP_STEP_FOLD_SRC, -1, 0, 0, 0, offset, length));
      p.steps.push_back(mk(GLOO_HIP_STEP_FOLD_SRC, -1, 0, GLOO_HIP_SRC_ARENA, 0, inOff, length));
      p.steps.push_back(mk(GLOO_HIP_STEP_FOLD, -1, 0, 0, offset, 0, length));
    }
    if (forward) send(co);
    p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, left, GLOO_HIP_SLOT_NOTIFY));
  };
  send(2 * rank);                                           // :102-103
  send(2 * rank + 1);
  for (uint64_t r = 2; r < chunks; r++) round(chunkAt(r), true, true);            // :106-158
  for (uint64_t r = 0; r < chunks - 2; r++) round(chunkAt(r), false, r < chunks - 4);  // :163-200
  for (int i = 0; i < 3; i++) p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, right, GLOO_HIP_SLOT_NOTIFY));
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
  return p;
}

// ---------------------------------------------------------------------------
// AllreduceRingChunked's result, mesh data movement.
//
// In the ring (planRingChunked above) the chunk pair q = {2q, 2q+1} starts
// on rank q (copyChunkAtOffset(2 * rank), :102-103) and every later rank
// q+1, q+2, ... reduces `local op incoming` (fn_->call(&ptrs_[0][offset],
// inbox, ...), :148-151) on its still-untouched local chunk, so the ring
// finishes the pair on rank o = q-1 with
//     x_{q+P-1} op ( ... op (x_{q+2} op (x_{q+1} op x_q)))
// and broadcasts it.  Here every rank sends its raw pair straight to o, all
// pairs at once (one xGMI link per peer on an 8-GPU node), o evaluates the
// same expression in one pass (FOLD, REVERSE: acc = s_k op acc, s_0 = x_q),
// and sends the result to every rank: 2 hops instead of 2(P-1), every link
// busy, identical bits.
//
// Arena: RS[p] = [2p * cs, +2cs) receives p's raw pair of MY range,
//        AG[p] = [2(P+p) * cs, +2cs) receives owner p's finished range.
// Inbox reuse needs no extra handshake: my next-run RS send to p is stream-
// ordered after my WAIT on p's AG message, which p sends after its FOLD;
// p's next AG send needs my next RS data, sent after my COPY out of AG[p].
// ---------------------------------------------------------------------------
Plan planRingChunkedMesh(int rank, int size, uint64_t count, int nptrs) {
  if (size > GLOO_HIP_MAX_SRCS) throw std::invalid_argument("mesh ring-chunked needs size <= 8");
  Plan p;
  if (count == 0) return p;
  const uint64_t chunks = 2ull * size;
  const uint64_t cs = std::max<uint64_t>(256, (count + chunks - 1) / chunks);
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count));
  if (size == 1) {
    if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
    return p;
  }
  // owner o finishes pair q = o + 1: elements [2q*cs, min(count, (2q+2)*cs))
  auto range = [&](int owner, uint64_t& off, uint64_t& len) {
    const uint64_t q = (uint64_t)((owner + 1) % size);
    off = 2 * q * cs;
    const uint64_t end = std::min<uint64_t>(count, off + 2 * cs);
    len = off < end ? end - off : 0;
  };
  p.arena = 4ull * size * cs;
  uint64_t myOff, myLen;
  range(rank, myOff, myLen);
  for (int d = 1; d < size; d++) {
    const int peer = (rank + d) % size;
    uint64_t o, l;
    range(peer, o, l);
    if (myLen) p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, peer, GLOO_HIP_SLOT_DATA0, 0, 2ull * peer * cs, 0, 2 * cs));
    if (l) p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, peer, GLOO_HIP_SLOT_DATA1, 0, 2ull * (size + peer) * cs, 0,
                                2 * cs));
  }
  // reduce-scatter: my raw piece of every other owner's range, all at once
  for (int d = 1; d < size; d++) {
    const int peer = (rank + d) % size;
    uint64_t o, l;
    range(peer, o, l);
    if (l) p.steps.push_back(mk(GLOO_HIP_STEP_SEND, peer, GLOO_HIP_SLOT_DATA0, 0, 0, o, l));
  }
  if (myLen) {
    for (int d = 1; d < size; d++)
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, (rank + d) % size, GLOO_HIP_SLOT_DATA0));
    // s_0 = x_q, s_1 = x_{q+1}, ..., s_{P-1} = x_o (local, in place)
    const int q = (rank + 1) % size;
    for (int k = 0; k < size; k++) {
      const int src = (q + k) % size;
      if (src == rank)
        p.steps.push_back(mk(GLOO_HIP_STEP_FOLD_SRC, -1, 0, 0, 0, myOff, myLen));
      else
        p.steps.push_back(mk(GLOO_HIP_STEP_FOLD_SRC, src, 0, GLOO_HIP_SRC_ARENA, 0, 2ull * src * cs, myLen));
    }
    p.steps.push_back(mk(GLOO_HIP_STEP_FOLD, -1, 0, GLOO_HIP_FOLD_REVERSE, myOff, 0, myLen));
    // allgather: the finished range to every rank, all at once
    for (int d = 1; d < size; d++)
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, (rank + d) % size, GLOO_HIP_SLOT_DATA1, 0, 0, myOff, myLen));
  }
  for (int d = 1; d < size; d++) {
    const int peer = (rank + d) % size;
    uint64_t o, l;
    range(peer, o, l);
    if (l) p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, peer, GLOO_HIP_SLOT_DATA1));
  }
  for (int d = 1; d < size; d++) {
    const int peer = (rank + d) % size;
    uint64_t o, l;
    range(peer, o, l);
    if (l) p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, o, 2ull * (size + peer) * cs, l));
  }
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
  return p;
}

// ---------------------------------------------------------------------------
// AllreduceHalvingDoubling (gloo/allreduce_halving_doubling.h:67-362), GPU
// twin gloo/cuda_allreduce_halving_doubling.cc:246-410.
// ---------------------------------------------------------------------------
Plan planHalvingDoubling(int rank, int size, uint64_t count, int nptrs) {
  Plan p;
  if (count == 0) return p;                                             // run() :226-228
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count));
  if (size == 1) {
    if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
    return p;
  }
  const Blocks bl = binaryBlocks(rank, size);                           // :102
  HDGeometry g = hdGeometry(rank, size, count, bl);                     // :107-157
  const uint32_t swb = bl.stepsWithinBlock;
  p.arena = g.chunkSize << g.steps;                                     // recvBuf_ (:80)
  for (uint32_t i = 0; i < swb; i++)
    p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, g.dest[i], GLOO_HIP_SLOT_DATA0, 0, g.regionOff[i],
                         0, g.chunkSize << (g.steps - 1) >> i));
  uint64_t ctorBufferOffset = g.bufferOffset;
  int smallDest = -1;
  bool smallRecv = false;
  if (bl.nextSmallerBlockSize != 0) {                                   // :159-175
    const uint32_t offsetToSmallerBlock = bl.offsetToMyBinaryBlock + bl.myBinaryBlockSize;
    smallDest = offsetToSmallerBlock + bl.rankInBinaryBlock % bl.nextSmallerBlockSize;
    const uint64_t itemCount = g.recvCounts[swb - 1];
    if (itemCount > 0) {
      smallRecv = true;
      p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, smallDest, GLOO_HIP_SLOT_DATA0, 0,
                           ctorBufferOffset, 0, itemCount));
    }
  }
  std::vector<int> largeDest;
  uint64_t sendCountToLargerBlock = 0;
  const uint64_t totalItemsToSend = swb > 0 ? g.recvCounts[swb - 1] : count;
  if (bl.nextLargerBlockSize != 0) {                                    // :176-222
    const uint32_t offsetToLargerBlock = bl.offsetToMyBinaryBlock - bl.nextLargerBlockSize;
    const uint32_t numSR = bl.nextLargerBlockSize / bl.myBinaryBlockSize;
    sendCountToLargerBlock = g.stepChunkSize >> (static_cast<uint64_t>(ilog2(numSR)) - 1);
    const uint32_t srcOrdinal = reverseLastNBits(bl.rankInBinaryBlock, ilog2(bl.myBinaryBlockSize));
    uint32_t destOrdinal = srcOrdinal * numSR;
    for (uint32_t i = 0; i < numSR; i++) {
      const int d = offsetToLargerBlock + reverseLastNBits(destOrdinal, ilog2(bl.nextLargerBlockSize));
      largeDest.push_back(d);
      if (sendCountToLargerBlock * i < totalItemsToSend) {
        const uint64_t toSend = std::min(sendCountToLargerBlock, totalItemsToSend - sendCountToLargerBlock * i);
        p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, d, GLOO_HIP_SLOT_DATA0, 0, ctorBufferOffset, 0, toSend));
        ctorBufferOffset += toSend;
      }
      destOrdinal++;
    }
  }
  p.arena = std::max<uint64_t>(p.arena, ctorBufferOffset);

  // run() :225-362
  uint64_t bufferOffset = 0;
  uint64_t numItems = swb > 0 ? g.chunkSize << (g.steps - 1) : count;
  for (uint32_t i = 0; i < swb; i++) {                                  // :244-259
    if (g.sendOffsets[i] < count)
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, g.dest[i], GLOO_HIP_SLOT_DATA0, 0, 0, g.sendOffsets[i],
                           g.sendCounts[i]));
    if (g.recvOffsets[i] < count) {
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, g.dest[i], GLOO_HIP_SLOT_DATA0));
      p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, g.recvOffsets[i],
                           bufferOffset, g.recvCounts[i]));
    }
    bufferOffset += numItems;
    p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, g.dest[i], GLOO_HIP_SLOT_NOTIFY));
    numItems >>= 1;
  }
  if (bl.nextSmallerBlockSize != 0 && smallRecv) {                      // :266-273
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, smallDest, GLOO_HIP_SLOT_DATA0));
    p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, g.recvOffsets[swb - 1],
                         bufferOffset, g.recvCounts[swb - 1]));
  }
  if (bl.nextLargerBlockSize != 0 && totalItemsToSend != 0) {           // :277-309
    const uint64_t offset = swb > 0 ? g.recvOffsets[swb - 1] : 0;
    const uint32_t numSR = bl.nextLargerBlockSize / bl.myBinaryBlockSize;
    for (uint32_t i = 0; i < numSR; i++)
      if (sendCountToLargerBlock * i < totalItemsToSend)
        p.steps.push_back(mk(GLOO_HIP_STEP_SEND, largeDest[i], GLOO_HIP_SLOT_DATA0, 0, 0,
                             offset + i * sendCountToLargerBlock,
                             std::min(sendCountToLargerBlock, totalItemsToSend - sendCountToLargerBlock * i)));
    for (uint32_t i = 0; i < numSR; i++)
      if (sendCountToLargerBlock * i < totalItemsToSend)
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, largeDest[i], GLOO_HIP_SLOT_DATA0));
    p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, offset, bufferOffset,
                         totalItemsToSend));
  }
  bool sentToSmallerBlock = false;                                      // :312-321
  if (bl.nextSmallerBlockSize != 0) {
    if (g.recvOffsets[swb - 1] < count) {
      sentToSmallerBlock = true;
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, smallDest, GLOO_HIP_SLOT_DATA0, 0, 0,
                           g.recvOffsets[swb - 1], g.recvCounts[swb - 1]));
    }
  }
  numItems = g.chunkSize << (g.steps - swb);                            // :324-346
  for (int i = (int)swb - 1; i >= 0; i--) {
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, g.dest[i], GLOO_HIP_SLOT_NOTIFY));
    if (g.recvOffsets[i] < count)
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, g.dest[i], GLOO_HIP_SLOT_DATA0, 0, 0, g.recvOffsets[i],
                           g.recvCounts[i]));
    bufferOffset -= numItems;
    if (g.sendOffsets[i] < count) {
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, g.dest[i], GLOO_HIP_SLOT_DATA0));
      p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, g.sendOffsets[i],
                           bufferOffset, g.sendCounts[i]));
    }
    numItems <<= 1;
    p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, g.dest[i], GLOO_HIP_SLOT_NOTIFY));
  }
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));  // :349-352
  for (int i = (int)swb - 1; i >= 0; i--)                               // :357-359
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, g.dest[i], GLOO_HIP_SLOT_NOTIFY));
  if (sentToSmallerBlock)                                               // :364-366
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_SEND, smallDest, GLOO_HIP_SLOT_DATA0));
  return p;
}

// ---------------------------------------------------------------------------
// AllreduceRing (gloo/allreduce_ring.h:21-113), GPU twin
// gloo/cuda_allreduce_ring.cc:73-121.  Arena = [inbox_ | outbox_].
// ---------------------------------------------------------------------------
Plan planRing(int rank, int size, uint64_t count, int nptrs) {
  Plan p;
  if (count == 0) return p;
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count));
  if (size > 1) {
    const int left = (size + rank - 1) % size, right = (rank + 1) % size;
    const uint64_t inbox = 0, outbox = count;
    p.arena = 2 * count;
    p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, left, GLOO_HIP_SLOT_DATA0, 0, inbox, 0, count));
    p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_DST_ARENA, outbox, 0, count));  // :78
    for (int round = 0; round < size - 1; round++) {
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, right, GLOO_HIP_SLOT_DATA0, GLOO_HIP_SRC_ARENA, 0, outbox, count));
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, left, GLOO_HIP_SLOT_DATA0));
      p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, 0, inbox, count));
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_SEND, right, GLOO_HIP_SLOT_DATA0));
      if (round < size - 2)
        p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA | GLOO_HIP_DST_ARENA, outbox,
                             inbox, count));
      p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, left, GLOO_HIP_SLOT_NOTIFY));
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, right, GLOO_HIP_SLOT_NOTIFY));
    }
  }
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
  return p;
}

// AllreduceLocal (gloo/allreduce_local.cc:28-37).
Plan planLocal(int, int, uint64_t count, int nptrs) {
  Plan p;
  if (nptrs > 1 && count > 0) {
    p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count));
    p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
  }
  return p;
}

// ---------------------------------------------------------------------------
// AllreduceBcube (gloo/allreduce_bcube.h:265-699), GPU twin CudaAllreduceBcube
// (gloo/cuda_allreduce_bcube.cc:49-215).  Ranks form groups of `base` whose
// members are `base^step` apart; each step reduce-scatters the group's range
// among its members, the all-gather walks the steps back.  The geometry is
// the reference's Node / Group bookkeeping restated (its int arithmetic, the
// count-0 -> 1 rule and the wrap `ptrOffset %= count`), so small or uneven
// counts take the reference's ranges too.  The reference tests P = base^k
// only (gloo/test/allreduce_test.cc:271-299).
// ---------------------------------------------------------------------------
struct BcubeNode {
  std::vector<std::vector<int>> peers;  // per step, self excluded
  std::vector<int> numElems, ptrOffset;
};

// computeSteps (gloo/allreduce_bcube.h:528-532): float logarithms, as there.
int bcubeSteps(int nodes, int base) {
  const float lg2n = std::log2(nodes);
  const float lg2p = std::log2(base);
  return (int)std::ceil(lg2n / lg2p);
}

// setupNodes / updateGroupNodes / Group (gloo/allreduce_bcube.h:163-250,
// 646-699).
std::vector<BcubeNode> bcubeNodes(int nodes, int base, int count, int steps) {
  std::vector<BcubeNode> all(nodes);
  for (auto& n : all) {
    n.peers.resize(steps);
    n.numElems.assign(steps, 0);
    n.ptrOffset.assign(steps, 0);
  }
  // (64-bit where the reference's int arithmetic could overflow for huge
  // bases or counts; equal results wherever it does not)
  int64_t peerDistance = 1;
  for (int step = 0; step < steps; ++step) {
    for (int rank = 0; rank < nodes; ++rank) {
      const BcubeNode& first = all[rank];
      if (!first.peers[step].empty()) continue;  // only nodes without peers start a group
      std::vector<int> group;
      for (int64_t i = 0; i < base && rank + i * peerDistance < nodes; ++i) group.push_back((int)(rank + i * peerDistance));
      int64_t ptrOffset = step == 0 ? 0 : first.ptrOffset[step - 1];
      const int groupCount = step == 0 ? count : first.numElems[step - 1];
      const int numElems = std::max(groupCount, (int)group.size());
      const int sz = (int)group.size();
      int each = numElems / sz;
      const int rem = numElems % sz;
      if (each == 0) each = 1;
      for (int i = 0; i < sz; ++i) {
        BcubeNode& node = all[group[i]];
        for (int peer : group)
          if (peer != group[i]) node.peers[step].push_back(peer);
        const int n = i != sz - 1 ? each : each + rem;
        node.numElems[step] = n;
        node.ptrOffset[step] = (int)ptrOffset;
        ptrOffset += n;
        ptrOffset %= count;
      }
    }
    peerDistance *= base;
  }
  return all;
}

// Arena: one inbox per (step, peer), sized max(mine, the peer's) as the
// reference's recvBufs_ (:300-308); a peer meets this rank in one step only.
// Notifications: the reference's (one per reduce-scatter receive, one per
// step-0 all-gather receive, waited for before each all-gather send and at the
// end) plus one per all-gather receive of the later steps, waited for at the
// end.  A plan runs repeatedly on asynchronous streams, and nothing else
// orders a step-s peer's next-run reduce-scatter send (s > 0) after this
// rank's copy out of the same inbox: the reference's final wait covers the
// step-0 peers only.  Data and order are the reference's, so the results are
// too.
Plan planBcube(int rank, int size, uint64_t count64, int nptrs, int base) {
  Plan p;
  if (count64 == 0) return p;                                          // run() :348-351
  if (count64 > (uint64_t)std::numeric_limits<int>::max())
    throw std::invalid_argument("AllreduceBcube counts elements in int");
  const int count = (int)count64;
  // CudaAllreduceBcube takes `context->base ? context->base : 2`
  // (gloo/cuda_allreduce_bcube.cc:57); a base
  // of 1 would divide by log2(1) = 0 in computeSteps, so it plans as 2 too
  if (base < 2) base = 2;
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count64));  // :352-355
  if (size == 1) {                                                      // :357-363
    if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count64));
    return p;
  }
  const int steps = bcubeSteps(size, base);
  const std::vector<BcubeNode> all = bcubeNodes(size, base, count, steps);
  const BcubeNode& me = all[rank];
  std::vector<std::vector<uint64_t>> inbox(steps);                      // ctor :296-320
  for (int step = 0; step < steps; ++step)
    for (int peer : me.peers[step]) {
      const uint64_t n = (uint64_t)std::max(me.numElems[step], all[peer].numElems[step]);
      inbox[step].push_back(p.arena);
      p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, peer, GLOO_HIP_SLOT_DATA0, 0, p.arena, 0, n));
      p.arena += n;
    }
  for (int step = 0; step < steps; ++step) {                           // reduce-scatter :365-391
    for (int dest : me.peers[step])
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, dest, GLOO_HIP_SLOT_DATA0, 0, 0,
                           (uint64_t)all[dest].ptrOffset[step], (uint64_t)all[dest].numElems[step]));
    for (size_t j = 0; j < me.peers[step].size(); ++j) {
      const int src = me.peers[step][j];
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, src, GLOO_HIP_SLOT_DATA0));
      p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, (uint64_t)me.ptrOffset[step],
                           inbox[step][j], (uint64_t)me.numElems[step]));
      p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, src, GLOO_HIP_SLOT_NOTIFY));  // :389
    }
  }
  for (int step = steps - 1; step >= 0; --step) {                      // all-gather :395-429
    for (int dest : me.peers[step]) {
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, dest, GLOO_HIP_SLOT_NOTIFY));  // :404
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, dest, GLOO_HIP_SLOT_DATA0, 0, 0, (uint64_t)me.ptrOffset[step],
                           (uint64_t)me.numElems[step]));
    }
    for (size_t j = 0; j < me.peers[step].size(); ++j) {
      const int src = me.peers[step][j];
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, src, GLOO_HIP_SLOT_DATA0));
      p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, (uint64_t)all[src].ptrOffset[step],
                           inbox[step][j], (uint64_t)all[src].numElems[step]));
      p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, src, GLOO_HIP_SLOT_NOTIFY));  // :419-424 (step 0 there)
    }
  }
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count64));  // :431-434
  for (int step = 0; step < steps; ++step)                             // :441-443 (+ the later steps)
    for (int peer : me.peers[step]) p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, peer, GLOO_HIP_SLOT_NOTIFY));
  return p;
}

// ---------------------------------------------------------------------------
// ReduceScatterHalvingDoubling (gloo/reduce_scatter.h:112-442).
// Arena = [recvBuf_ (chunkSize << steps) | recvBufDist_ (count)].
// ---------------------------------------------------------------------------
struct DistMap {
  int rank;
  uint64_t offset, itemCount;
};

// gloo/reduce_scatter.h:72-110
void distributionMap(int size, uint64_t srcOffset, uint64_t srcCount, const std::vector<int>& recvCounts,
                     bool reorder, std::vector<DistMap>& out) {
  if (srcCount == 0) return;
  uint64_t destOffset = 0;
  const int n = reorder ? 1 << (int)ilog2(size) : size;
  int start = 0;
  for (; start < n; ++start) {
    if (destOffset + (uint64_t)(int64_t)recvCounts[start] > srcOffset) break;
    destOffset += recvCounts[start];
  }
  destOffset = srcOffset - destOffset;
  uint64_t totalCount = srcCount;
  for (int i = start; i < n; ++i) {
    int64_t recvCount = recvCounts[i];
    if (destOffset != 0) {
      recvCount -= (int64_t)destOffset;
      destOffset = 0;
    }
    const int r = reorder ? (int)reverseLastNBits(i, ilog2(size)) : i;
    uint64_t rc = (uint64_t)recvCount;
    rc = rc < totalCount ? rc : totalCount;
    out.push_back({r, srcOffset, rc});
    srcOffset += rc;
    totalCount -= rc;
    if (totalCount == 0) break;
  }
}

Plan planReduceScatter(int rank, int size, uint64_t count, int nptrs, const std::vector<int>& recvElems) {
  Plan p;
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count));
  if (size == 1) {                                                       // run() :337-343
    if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
    return p;
  }
  const Blocks bl = binaryBlocks(rank, size);
  HDGeometry g = hdGeometry(rank, size, count, bl);
  const uint32_t swb = bl.stepsWithinBlock;
  const uint64_t distBase = g.chunkSize << g.steps;
  p.arena = distBase + count;
  for (uint32_t i = 0; i < swb; i++)
    p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, g.dest[i], GLOO_HIP_SLOT_DATA0, 0, g.regionOff[i], 0,
                         g.chunkSize << (g.steps - 1) >> i));
  int smallDest = -1;
  bool smallRecv = false;
  if (bl.nextSmallerBlockSize != 0) {                                    // :206-220
    smallDest = bl.offsetToMyBinaryBlock + bl.myBinaryBlockSize + bl.rankInBinaryBlock % bl.nextSmallerBlockSize;
    const uint64_t itemCount = g.recvCounts[swb - 1];
    if (itemCount > 0) {
      smallRecv = true;
      p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, smallDest, GLOO_HIP_SLOT_DATA0, 0, g.bufferOffset, 0,
                           itemCount));
    }
  }
  std::vector<int> largeDest;
  uint64_t sendCountToLargerBlock = 0;
  if (bl.nextLargerBlockSize != 0) {                                     // :221-247
    const uint32_t offsetToLargerBlock = bl.offsetToMyBinaryBlock - bl.nextLargerBlockSize;
    const uint32_t numSR = bl.nextLargerBlockSize / bl.myBinaryBlockSize;
    sendCountToLargerBlock = g.stepChunkSize >> (static_cast<uint64_t>(ilog2(numSR)) - 1);
    const uint32_t srcOrdinal = reverseLastNBits(bl.rankInBinaryBlock, ilog2(bl.myBinaryBlockSize));
    uint32_t destOrdinal = srcOrdinal * numSR;
    for (uint32_t i = 0; i < numSR; i++) {
      largeDest.push_back(offsetToLargerBlock + reverseLastNBits(destOrdinal, ilog2(bl.nextLargerBlockSize)));
      destOrdinal++;
    }
  }
  std::vector<DistMap> distSend, distRecv;                               // :255-327
  if (bl.nextLargerBlockSize == 0 && swb > 0)
    distributionMap(size, g.recvOffsets[swb - 1], g.recvCounts[swb - 1], recvElems, false, distSend);
  if (recvElems[rank] > 0) {
    std::vector<int> srcCounts;
    uint64_t rem = count;
    for (int i = 0; i < size; ++i) {
      srcCounts.push_back((int)std::min(g.chunkSize, rem));
      rem = rem > g.chunkSize ? rem - g.chunkSize : 0;
    }
    uint64_t offset = 0;
    for (int i = 0; i < rank; ++i) offset += recvElems[i];
    distributionMap(size, offset, recvElems[rank], srcCounts, true, distRecv);
    for (const auto& d : distRecv)
      if (d.rank != rank)
        p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, d.rank, GLOO_HIP_SLOT_DIST, 0, distBase + d.offset, 0,
                             d.itemCount));
  }

  // run() :329-442
  uint64_t bufferOffset = 0;
  uint64_t numItems = swb > 0 ? g.chunkSize << (g.steps - 1) : count;
  for (uint32_t i = 0; i < swb; i++) {
    if (g.sendOffsets[i] < count)
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, g.dest[i], GLOO_HIP_SLOT_DATA0, 0, 0, g.sendOffsets[i],
                           g.sendCounts[i]));
    if (g.recvOffsets[i] < count) {
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, g.dest[i], GLOO_HIP_SLOT_DATA0));
      p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, g.recvOffsets[i], bufferOffset,
                           g.recvCounts[i]));
    }
    bufferOffset += numItems;
    p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, g.dest[i], GLOO_HIP_SLOT_NOTIFY));
    numItems >>= 1;
  }
  if (bl.nextSmallerBlockSize != 0 && smallRecv) {
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, smallDest, GLOO_HIP_SLOT_DATA0));
    p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, g.recvOffsets[swb - 1],
                         bufferOffset, g.recvCounts[swb - 1]));
  }
  const uint64_t totalItemsToSend = swb > 0 ? g.recvCounts[swb - 1] : count;
  if (bl.nextLargerBlockSize != 0 && totalItemsToSend != 0) {
    const uint64_t offset = swb > 0 ? g.recvOffsets[swb - 1] : 0;
    const uint32_t numSR = bl.nextLargerBlockSize / bl.myBinaryBlockSize;
    for (uint32_t i = 0; i < numSR; i++)
      if (sendCountToLargerBlock * i < totalItemsToSend)
        p.steps.push_back(mk(GLOO_HIP_STEP_SEND, largeDest[i], GLOO_HIP_SLOT_DATA0, 0, 0,
                             offset + i * sendCountToLargerBlock,
                             std::min(sendCountToLargerBlock, totalItemsToSend - sendCountToLargerBlock * i)));
  }
  for (const auto& d : distSend)
    if (d.rank != rank)
      p.steps.push_back(mk(GLOO_HIP_STEP_SEND, d.rank, GLOO_HIP_SLOT_DIST, 0, 0, d.offset, d.itemCount));
  bufferOffset = 0;
  for (const auto& d : distRecv) {
    if (d.rank != rank) {
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, d.rank, GLOO_HIP_SLOT_DIST));
      p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, bufferOffset, distBase + d.offset,
                           d.itemCount));
      p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, d.rank, GLOO_HIP_SLOT_DIST_NOTIFY));
    } else if (rank != 0) {  // data already in place for rank 0 (:418-425)
      p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, 0, bufferOffset, d.offset, d.itemCount));
    }
    bufferOffset += d.itemCount;
  }
  if (nptrs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
  for (uint32_t i = 0; i < swb; i++)                                     // :432-439
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, g.dest[i], GLOO_HIP_SLOT_NOTIFY));
  for (const auto& d : distSend)
    if (d.rank != rank)
      p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, d.rank, GLOO_HIP_SLOT_DIST_NOTIFY));
  return p;
}

// ---------------------------------------------------------------------------
// New-style gloo::allreduce(opts), RING (gloo/allreduce.cc:97-392).
// The reference's two-sided unbound buffers are restated one-sidedly: posting
// a receive becomes a credit (NOTIFY) to the sender, which waits for it
// before writing (WAIT_NOTIFY + SEND); the reduce-scatter receives land in
// two segment inboxes (tmp, :219-226), the allgather receives in two more and
// are copied to out[0] at their offset (the reference receives in place).
// Arena = [tmp0 | tmp1 | ag0 | ag1], one segment each.
// ---------------------------------------------------------------------------
Plan planAllreduceRing(int rank, int size, uint64_t count, const NewStyleOptions& o) {
  Plan p;
  if (count == 0) return p;                                             // :98-100
  const uint64_t es = o.elemSize;
  const bool localReduce = o.ninputs > 0 || o.noutputs > 1;
  const int fromInputs = o.ninputs > 0 ? GLOO_HIP_FROM_INPUTS : 0;
  auto reduceInputs = [&](uint64_t off, uint64_t len) {                 // :42-84
    if (localReduce) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, fromInputs, off, 0, len));
  };
  auto broadcastOutputs = [&](uint64_t off, uint64_t len) {             // :89-98
    if (o.noutputs > 1) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, off, 0, len));
  };
  if (size == 1) {                                                      // :125-129
    reduceInputs(0, count);
    broadcastOutputs(0, count);
    return p;
  }
  const uint64_t totalBytes = count * es;
  const uint64_t maxSegmentBytes = es * std::max<uint64_t>(1, (o.maxSegmentBytes ? o.maxSegmentBytes : 1024 * 1024) / es);
  auto roundUp = [](uint64_t v, uint64_t m) { return v % m == 0 ? v : v + m - v % m; };
  const uint64_t numSegments =
      roundUp(std::max<uint64_t>((totalBytes + (maxSegmentBytes - 1)) / maxSegmentBytes, (uint64_t)size * 2),
              (uint64_t)size);                                          // :202-207
  const uint64_t nspr = numSegments / size;
  const uint64_t segBytes = roundUp((totalBytes + numSegments - 1) / numSegments, es);  // :211-212
  const uint64_t seg = segBytes / es;  // elements
  const int recvRank = (size + rank + 1) % size, sendRank = (size + rank - 1) % size;  // :158-159
  p.arena = 4 * seg;
  p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, recvRank, GLOO_HIP_SLOT_DATA0, 0, 0, 0, seg));
  p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, recvRank, GLOO_HIP_SLOT_DATA1, 0, seg, 0, seg));
  p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, recvRank, GLOO_HIP_SLOT_AUX0, 0, 2 * seg, 0, seg));
  p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, recvRank, GLOO_HIP_SLOT_AUX1, 0, 3 * seg, 0, seg));
  struct Off {
    uint64_t sendOffset, recvOffset;
    int64_t sendLength, recvLength;
  };
  auto offsets = [&](uint64_t i, int sendShift, int recvShift) {        // :231-257, :312-335
    Off r;
    r.sendOffset = ((((uint64_t)rank + sendShift) * nspr + i) * seg) % (numSegments * seg);
    r.recvOffset = ((((uint64_t)rank + recvShift) * nspr + i) * seg) % (numSegments * seg);
    r.sendLength = std::min<int64_t>((int64_t)seg, (int64_t)count - (int64_t)r.sendOffset);
    r.recvLength = std::min<int64_t>((int64_t)seg, (int64_t)count - (int64_t)r.recvOffset);
    return r;
  };
  const uint64_t iters = numSegments - nspr + 2;
  for (uint64_t i = 0; i < iters; i++) {                                // reduce/scatter :268-306
    const int buf = (int)(i & 1);
    if (i >= 2) {
      const Off prev = offsets(i - 2, 1, 2);
      if (prev.recvLength > 0) {
        reduceInputs(prev.recvOffset, prev.recvLength);
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, recvRank, GLOO_HIP_SLOT_DATA0 + buf));
        p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, prev.recvOffset, buf * seg,
                             prev.recvLength));
      }
    }
    if (i < numSegments - nspr) {
      const Off cur = offsets(i, 1, 2);
      if (cur.recvLength > 0) p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, recvRank, GLOO_HIP_SLOT_NOTIFY));
      if (cur.sendLength > 0) {
        if (i < nspr) reduceInputs(cur.sendOffset, cur.sendLength);
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, sendRank, GLOO_HIP_SLOT_NOTIFY));
        p.steps.push_back(mk(GLOO_HIP_STEP_SEND, sendRank, GLOO_HIP_SLOT_DATA0 + buf, 0, 0, cur.sendOffset,
                             cur.sendLength));
      }
    }
  }
  for (uint64_t i = 0; i < iters; i++) {                                // allgather :345-377
    const int buf = (int)(i & 1);
    if (i >= 2) {
      const Off prev = offsets(i - 2, 0, 1);
      if (prev.recvLength > 0) {
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, recvRank, GLOO_HIP_SLOT_AUX0 + buf));
        p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, prev.recvOffset, (2 + buf) * seg,
                             prev.recvLength));
        broadcastOutputs(prev.recvOffset, prev.recvLength);
      }
    }
    if (i < numSegments - nspr) {
      const Off cur = offsets(i, 0, 1);
      if (cur.recvLength > 0) p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, recvRank, GLOO_HIP_SLOT_AUX_NOTIFY));
      if (cur.sendLength > 0) {
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, sendRank, GLOO_HIP_SLOT_AUX_NOTIFY));
        p.steps.push_back(mk(GLOO_HIP_STEP_SEND, sendRank, GLOO_HIP_SLOT_AUX0 + buf, 0, 0, cur.sendOffset,
                             cur.sendLength));
        if (i < nspr) broadcastOutputs(cur.sendOffset, cur.sendLength);
      }
    }
  }
  return p;
}

// ---------------------------------------------------------------------------
// New-style gloo::allreduce(opts), BCUBE (gloo/allreduce.cc:397-669).
// The group of every step is computed exactly as the reference does
// (:466-503).  Reduce-scatter receives land in `tmp` at i * chunkLength
// (:529-533) and are folded into out[myChunk] in group order, out = out op
// tmp_i (:580-592) — one FOLD pass over all of them when they fit in one
// launch.  Allgather receives (the reference's in-place out->recv, :622-626)
// land in a second arena region laid out like `out` and are copied there.
// Posting a receive is a credit to the sender, as in the ring; messages of
// length 0 are skipped on both sides (both compute the same length).
// Arena = [tmp: bufferLength (:507-511) | allgather: count].
// ---------------------------------------------------------------------------
std::vector<uint64_t> groupSizePerStep(uint64_t size, uint64_t n) {  // :397-408
  std::vector<uint64_t> out;
  while (size % n == 0) {
    out.push_back(n);
    size /= n;
  }
  if (size > 1) out.push_back(size);
  return out;
}

Plan planAllreduceBcube(int rank, int size, uint64_t count, const NewStyleOptions& o) {
  Plan p;
  if (count == 0) return p;                                             // :98-100
  const bool localReduce = o.ninputs > 0 || o.noutputs > 1;
  const int fromInputs = o.ninputs > 0 ? GLOO_HIP_FROM_INPUTS : 0;
  auto reduceInputs = [&](uint64_t off, uint64_t len) {                 // :42-84
    if (localReduce && len) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, fromInputs, off, 0, len));
  };
  auto broadcastOutputs = [&](uint64_t off, uint64_t len) {             // :89-98
    if (o.noutputs > 1 && len) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, off, 0, len));
  };
  if (size == 1) {                                                      // :125-129
    reduceInputs(0, count);
    broadcastOutputs(0, count);
    return p;
  }
  struct Group {
    uint64_t bufferOffset = 0, bufferLength = 0, chunkLength = 0, myChunkOffset = 0, myChunkLength = 0;
    std::vector<int> ranks;
    // length of member i's chunk (:542-548, :615-621)
    uint64_t lengthOf(size_t i) const {
      const int64_t rest = (int64_t)bufferLength - (int64_t)(i * chunkLength);
      return std::min<uint64_t>(chunkLength, (uint64_t)std::max<int64_t>(0, rest));
    }
    uint64_t offsetOf(size_t i) const { return bufferOffset + i * chunkLength; }
  };
  std::vector<Group> groups;
  {
    uint64_t peerDistance = 1, bufferOffset = 0, bufferLength = count;
    for (const uint64_t groupSize : groupSizePerStep((uint64_t)size, 2)) {
      Group g;
      const uint64_t groupRank = ((uint64_t)rank / peerDistance) % groupSize;
      const uint64_t baseRank = (uint64_t)rank - groupRank * peerDistance;
      for (uint64_t i = 0; i < groupSize; i++) g.ranks.push_back((int)(baseRank + i * peerDistance));
      g.bufferOffset = bufferOffset;
      g.bufferLength = bufferLength;
      g.chunkLength = (bufferLength + groupSize - 1) / groupSize;
      g.myChunkOffset = bufferOffset + groupRank * g.chunkLength;
      g.myChunkLength = g.lengthOf(groupRank);
      groups.push_back(g);
      peerDistance *= groupSize;
      bufferOffset = g.myChunkOffset;
      bufferLength = g.myChunkLength;
    }
  }
  uint64_t tmpLength = count;                                            // :507-511
  for (const Group& g : groups) tmpLength = std::max<uint64_t>(tmpLength, g.ranks.size() * g.chunkLength);
  const uint64_t agBase = tmpLength;
  p.arena = tmpLength + count;
  // Every peer appears in exactly one step (members of a step's group differ
  // from this rank in that step's mixed-radix digit only), so one region per
  // (peer, slot) is enough.
  for (const Group& g : groups)
    for (size_t i = 0; i < g.ranks.size(); i++) {
      const int peer = g.ranks[i];
      if (peer == rank) continue;
      if (g.myChunkLength)
        p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, peer, GLOO_HIP_SLOT_DATA0, 0, i * g.chunkLength, 0,
                             g.myChunkLength));
      if (g.lengthOf(i))
        p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, peer, GLOO_HIP_SLOT_AUX0, 0, agBase + g.offsetOf(i), 0,
                             g.lengthOf(i)));
    }
  // Reduce/scatter (:519-593).
  for (size_t step = 0; step < groups.size(); step++) {
    const Group& g = groups[step];
    for (int peer : g.ranks)                                             // tmp->recv (:524-534)
      if (peer != rank && g.myChunkLength) p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, peer, GLOO_HIP_SLOT_NOTIFY));
    if (step == 0)                                                       // :549-554
      for (size_t i = 0; i < g.ranks.size(); i++)
        if (g.ranks[i] != rank) reduceInputs(g.offsetOf(i), g.lengthOf(i));
    // credits first, then every send in one batch (one launch, all links)
    for (size_t i = 0; i < g.ranks.size(); i++)
      if (g.ranks[i] != rank && g.lengthOf(i))
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, g.ranks[i], GLOO_HIP_SLOT_NOTIFY));
    for (size_t i = 0; i < g.ranks.size(); i++)                          // out->send (:555-559)
      if (g.ranks[i] != rank && g.lengthOf(i))
        p.steps.push_back(mk(GLOO_HIP_STEP_SEND, g.ranks[i], GLOO_HIP_SLOT_DATA0, 0, 0, g.offsetOf(i), g.lengthOf(i)));
    if (g.myChunkLength)                                                 // :563-570
      for (int peer : g.ranks)
        if (peer != rank) p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, peer, GLOO_HIP_SLOT_DATA0));
    if (step == 0) reduceInputs(g.myChunkOffset, g.myChunkLength);      // :574-577
    if (g.myChunkLength == 0) continue;
    // out = ((out op tmp_0) op tmp_1) ... over the peers in group order (:580-592)
    if (g.ranks.size() <= (size_t)GLOO_HIP_MAX_SRCS) {
      p.steps.push_back(mk(GLOO_HIP_STEP_FOLD_SRC, -1, 0, 0, 0, g.myChunkOffset, g.myChunkLength));
      for (size_t i = 0; i < g.ranks.size(); i++)
        if (g.ranks[i] != rank)
          p.steps.push_back(mk(GLOO_HIP_STEP_FOLD_SRC, -1, 0, GLOO_HIP_SRC_ARENA, 0, i * g.chunkLength,
                               g.myChunkLength));
      p.steps.push_back(mk(GLOO_HIP_STEP_FOLD, -1, 0, 0, g.myChunkOffset, 0, g.myChunkLength));
    } else {
      for (size_t i = 0; i < g.ranks.size(); i++)
        if (g.ranks[i] != rank)
          p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA, g.myChunkOffset, i * g.chunkLength,
                               g.myChunkLength));
    }
  }
  broadcastOutputs(groups.back().myChunkOffset, groups.back().myChunkLength);  // :599-603
  // Allgather (:605-668).
  for (auto it = groups.rbegin(); it != groups.rend(); ++it) {
    const Group& g = *it;
    for (size_t i = 0; i < g.ranks.size(); i++)                          // out->recv (:610-627)
      if (g.ranks[i] != rank && g.lengthOf(i))
        p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, g.ranks[i], GLOO_HIP_SLOT_AUX_NOTIFY));
    if (g.myChunkLength) {                                               // out->send (:630-640)
      for (int peer : g.ranks)
        if (peer != rank) p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, peer, GLOO_HIP_SLOT_AUX_NOTIFY));
      for (int peer : g.ranks)
        if (peer != rank)
          p.steps.push_back(mk(GLOO_HIP_STEP_SEND, peer, GLOO_HIP_SLOT_AUX0, 0, 0, g.myChunkOffset, g.myChunkLength));
    }
    for (size_t i = 0; i < g.ranks.size(); i++)                          // :643-650
      if (g.ranks[i] != rank && g.lengthOf(i))
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, g.ranks[i], GLOO_HIP_SLOT_AUX0));
    for (size_t i = 0; i < g.ranks.size(); i++)
      if (g.ranks[i] != rank && g.lengthOf(i))
        p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, g.offsetOf(i), agBase + g.offsetOf(i),
                             g.lengthOf(i)));
    for (size_t i = 0; i < g.ranks.size(); i++)                          // :653-667
      if (g.ranks[i] != rank) broadcastOutputs(g.offsetOf(i), g.lengthOf(i));
  }
  return p;
}

// ---------------------------------------------------------------------------
// New-style gloo::reduce(opts) (gloo/reduce.cc:21-247).  A ring
// reduce-scatter over two segment inboxes (tmp, :124-134) — out = in op tmp
// (:180-184), the first numSegmentsPerRank sends read `in` (:206-210) — then
// every rank's reduced chunk goes to the root (:221-246), landing in an arena
// region laid out like `out` and copied there.  REDUCE / SEND carry
// GLOO_HIP_FROM_INPUTS when a separate input exists.
// Arena = [tmp0 | tmp1 | (root only) gather: numSegments segments].
// ---------------------------------------------------------------------------
Plan planReduce(int rank, int size, uint64_t count, const NewStyleOptions& o) {
  Plan p;
  if (count == 0) return p;                                             // :22-24
  if (o.root < 0 || o.root >= size) throw std::invalid_argument("root out of range");  // :32
  const int fromIn = o.ninputs > 0 ? GLOO_HIP_FROM_INPUTS : 0;
  if (size == 1) {                                                      // :54-59
    if (fromIn) p.steps.push_back(mk(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, GLOO_HIP_FROM_INPUTS, 0, 0, count));
    return p;
  }
  auto roundUp = [](uint64_t v, uint64_t m) { return v % m == 0 ? v : v + m - v % m; };
  const uint64_t es = o.elemSize;
  const uint64_t totalBytes = count * es;
  const uint64_t maxSegmentSize = es * ((o.maxSegmentBytes ? o.maxSegmentBytes : 1024 * 1024) / es);  // :90-91
  if (maxSegmentSize == 0) throw std::invalid_argument("maxSegmentSize below one element");
  const uint64_t P = (uint64_t)size;
  const uint64_t segmentBytes =
      roundUp(std::min<uint64_t>((totalBytes + (P * 2 - 1)) / (P * 2), maxSegmentSize), es);  // :95-101
  const uint64_t numSegments =
      roundUp(std::max<uint64_t>((totalBytes + (segmentBytes - 1)) / segmentBytes, P * 2), P);  // :113-117
  const uint64_t nspr = numSegments / P;                                // :120
  const uint64_t seg = segmentBytes / es;                               // elements
  const uint64_t chunk = nspr * seg;                                    // :121
  const int recvRank = (size + rank + 1) % size, sendRank = (size + rank - 1) % size;  // :34-43
  const uint64_t gatherBase = 2 * seg;
  p.arena = 2 * seg + (rank == o.root ? numSegments * seg : 0);
  p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, recvRank, GLOO_HIP_SLOT_DATA0, 0, 0, 0, seg));
  p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, recvRank, GLOO_HIP_SLOT_DATA1, 0, seg, 0, seg));
  auto chunkLength = [&](int r) {                                       // :227-229, :239-241
    return std::min<int64_t>((int64_t)chunk, (int64_t)count - (int64_t)((uint64_t)r * chunk));
  };
  if (rank == o.root)
    for (int r = 0; r < size; r++)
      if (r != rank && chunkLength(r) > 0)
        p.steps.push_back(mk(GLOO_HIP_STEP_DECL_RECV, r, GLOO_HIP_SLOT_DIST, 0, gatherBase + (uint64_t)r * chunk, 0,
                             (uint64_t)chunkLength(r)));
  struct Off {
    uint64_t sendOffset, recvOffset;
    int64_t sendLength, recvLength;
  };
  auto offsets = [&](uint64_t i) {                                      // :138-169
    Off r;
    r.sendOffset = ((((uint64_t)rank + 1) * nspr + i) * seg) % (numSegments * seg);
    r.recvOffset = ((((uint64_t)rank + 2) * nspr + i) * seg) % (numSegments * seg);
    r.sendLength = std::min<int64_t>((int64_t)seg, (int64_t)count - (int64_t)r.sendOffset);
    r.recvLength = std::min<int64_t>((int64_t)seg, (int64_t)count - (int64_t)r.recvOffset);
    return r;
  };
  for (uint64_t i = 0; i < numSegments; i++) {                          // :171-213
    const int buf = (int)(i & 1);
    if (i >= 2) {
      const Off prev = offsets(i - 2);
      if (prev.recvLength > 0) {
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, recvRank, GLOO_HIP_SLOT_DATA0 + buf));
        p.steps.push_back(mk(GLOO_HIP_STEP_REDUCE, -1, 0, GLOO_HIP_SRC_ARENA | fromIn, prev.recvOffset, buf * seg,
                             (uint64_t)prev.recvLength));
      }
    }
    if (i + 2 < numSegments) {
      const Off cur = offsets(i);
      if (cur.recvLength > 0) p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, recvRank, GLOO_HIP_SLOT_NOTIFY));
      if (cur.sendLength > 0) {
        p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, sendRank, GLOO_HIP_SLOT_NOTIFY));
        p.steps.push_back(mk(GLOO_HIP_STEP_SEND, sendRank, GLOO_HIP_SLOT_DATA0 + buf, i < nspr ? fromIn : 0, 0,
                             cur.sendOffset, (uint64_t)cur.sendLength));
      }
    }
  }
  if (rank == o.root) {                                                 // :221-237
    for (int r = 0; r < size; r++)
      if (r != rank && chunkLength(r) > 0) p.steps.push_back(mk(GLOO_HIP_STEP_NOTIFY, r, GLOO_HIP_SLOT_DIST_NOTIFY));
    for (int r = 0; r < size; r++)
      if (r != rank && chunkLength(r) > 0) p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_RECV, r, GLOO_HIP_SLOT_DIST));
    for (int r = 0; r < size; r++)
      if (r != rank && chunkLength(r) > 0)
        p.steps.push_back(mk(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, (uint64_t)r * chunk,
                             gatherBase + (uint64_t)r * chunk, (uint64_t)chunkLength(r)));
  } else if (chunkLength(rank) > 0) {                                   // :238-246
    p.steps.push_back(mk(GLOO_HIP_STEP_WAIT_NOTIFY, o.root, GLOO_HIP_SLOT_DIST_NOTIFY));
    p.steps.push_back(mk(GLOO_HIP_STEP_SEND, o.root, GLOO_HIP_SLOT_DIST, 0, 0, (uint64_t)rank * chunk,
                         (uint64_t)chunkLength(rank)));
  }
  return p;
}

}  // namespace

Plan makeNewStylePlan(int algo, int rank, int size, uint64_t count, const NewStyleOptions& o) {
  if (size < 1 || rank < 0 || rank >= size) throw std::invalid_argument("bad rank/size");
  if (o.noutputs < 1 || o.ninputs < 0 || o.elemSize == 0) throw std::invalid_argument("bad options");
  if ((algo & ~GLOO_HIP_ALGO_MESH) == GLOO_HIP_ALGO_REDUCE && (o.ninputs > 1 || o.noutputs != 1))
    throw std::invalid_argument("gloo::reduce takes one input and one output");
  if (algo & GLOO_HIP_ALGO_MESH) {
    const int base = algo & ~GLOO_HIP_ALGO_MESH;
    if (base == GLOO_HIP_ALGO_REDUCE && (o.root < 0 || o.root >= size)) throw std::invalid_argument("root out of range");
    return makeMeshPlan(base, rank, size, count, o.noutputs, {}, &o);
  }
  switch (algo) {
    case GLOO_HIP_ALGO_ALLREDUCE_RING: return planAllreduceRing(rank, size, count, o);
    case GLOO_HIP_ALGO_ALLREDUCE_BCUBE: return planAllreduceBcube(rank, size, count, o);
    case GLOO_HIP_ALGO_REDUCE: return planReduce(rank, size, count, o);
  }
  throw std::invalid_argument("not a new-style algorithm");
}

Plan makePlan(int algo, int rank, int size, uint64_t count, int nptrs, const std::vector<int>& recvElems) {
  if (size < 1 || rank < 0 || rank >= size) throw std::invalid_argument("bad rank/size");
  if (nptrs < 1) throw std::invalid_argument("need at least one pointer");
  if (algo & GLOO_HIP_ALGO_MESH) {
    const int base = algo & ~GLOO_HIP_ALGO_MESH;
    if (base == GLOO_HIP_ALGO_REDUCE_SCATTER && (int)recvElems.size() != size)
      throw std::invalid_argument("recvElems must have size entries");
    return makeMeshPlan(base, rank, size, count, nptrs, recvElems);
  }
  switch (algo) {
    case GLOO_HIP_ALGO_RING_CHUNKED: return planRingChunked(rank, size, count, nptrs);
    case GLOO_HIP_ALGO_RING_CHUNKED_MESH: return planRingChunkedMesh(rank, size, count, nptrs);
    case GLOO_HIP_ALGO_RING_CHUNKED_PIPE: return planRingChunkedPipe(rank, size, count, nptrs);
    case GLOO_HIP_ALGO_HALVING_DOUBLING: return planHalvingDoubling(rank, size, count, nptrs);
    case GLOO_HIP_ALGO_RING: return planRing(rank, size, count, nptrs);
    case GLOO_HIP_ALGO_LOCAL: return planLocal(rank, size, count, nptrs);
    case GLOO_HIP_ALGO_BCUBE: return planBcube(rank, size, count, nptrs, recvElems.empty() ? 2 : recvElems[0]);
    case GLOO_HIP_ALGO_REDUCE_SCATTER:
      if ((int)recvElems.size() != size) throw std::invalid_argument("recvElems must have size entries");
      return planReduceScatter(rank, size, count, nptrs, recvElems);
  }
  throw std::invalid_argument("unknown algorithm");
}

}  // namespace gloo_amd

extern "C" int gloo_hip_plan(int algo, int rank, int size, size_t count, int nptrs, const int* recv_elems,
                             gloo_hip_step_t* steps, size_t capacity, size_t* nsteps, size_t* arena_elems) {
  return gloo_hip_plan_ex(algo, rank, size, count, 0, nptrs, 4, 0, recv_elems, steps, capacity, nsteps,
                          arena_elems);
}

extern "C" int gloo_hip_plan_ex(int algo, int rank, int size, size_t count, int ninputs, int noutputs,
                                size_t elem_size, size_t max_segment_bytes, const int* recv_elems,
                                gloo_hip_step_t* steps, size_t capacity, size_t* nsteps, size_t* arena_elems) {
  try {
    std::vector<int> re;
    if ((algo & ~GLOO_HIP_ALGO_MESH) == GLOO_HIP_ALGO_REDUCE_SCATTER) {
      if (!recv_elems) return GLOO_HIP_EINVAL_ARG;
      re.assign(recv_elems, recv_elems + size);
    }
    if ((algo & ~GLOO_HIP_ALGO_MESH) == GLOO_HIP_ALGO_BCUBE && recv_elems) re.assign(recv_elems, recv_elems + 1);  // {base}
    gloo_amd::Plan p;
    if (gloo_amd::isNewStyle(algo)) {
      gloo_amd::NewStyleOptions o;
      o.ninputs = ninputs;
      o.noutputs = noutputs;
      o.elemSize = elem_size;
      o.maxSegmentBytes = max_segment_bytes;
      if ((algo & ~GLOO_HIP_ALGO_MESH) == GLOO_HIP_ALGO_REDUCE) {
        if (!recv_elems) return GLOO_HIP_EINVAL_ARG;  // recv_elems[0] = root
        o.root = recv_elems[0];
      }
      p = gloo_amd::makeNewStylePlan(algo, rank, size, count, o);
    } else {
      p = gloo_amd::makePlan(algo, rank, size, count, noutputs, re);
    }
    if (nsteps) *nsteps = p.steps.size();
    if (arena_elems) *arena_elems = p.arena;
    if (steps) {
      if (capacity < p.steps.size()) return GLOO_HIP_EINVAL_ARG;
      if (!p.steps.empty()) std::memcpy(steps, p.steps.data(), p.steps.size() * sizeof(gloo_hip_step_t));
    }
    return GLOO_HIP_OK;
  } catch (const std::exception&) {
    return GLOO_HIP_EINVAL_ARG;
  }
}

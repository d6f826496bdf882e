// reduce.hip — CDNA4 (gfx950) element-wise chunk reduction for Gloo.
//
// Replaces the reference's per-chunk reduction (gloo/math.h:15-73 on the host,
// the grid-stride CUDA kernels gloo/cuda.cu:274-401 on the device).  The op is
// one instruction per element against 2 loads + 1 store, i.e. purely
// HBM-bound, so the kernel is built around the memory system, not arithmetic:
//
//  * every lane moves 16 B per access (global_load_dwordx4 / store_dwordx4),
//    64 lanes -> 1 KiB contiguous per wave-instruction, fully coalesced;
//  * UNROLL independent 16-B packets per operand per lane are in flight
//    before the first use (memory-level parallelism instead of occupancy);
//  * raw buffer loads/stores with the `nt` cache policy (data is streamed
//    exactly once) through per-tile buffer descriptors;
//  * the aligned body is a flat tile grid (one tile = 512 lanes x UNROLL
//    packets), tiles dealt round-robin over the 8 XCDs by the dispatcher;
//  * a chunk may start at any element offset (Gloo chunk offsets are
//    arbitrary element counts, gloo/allreduce_ring_chunked.h:128): the first
//    `head` elements up to the 16-B boundary of the destination and the
//    ragged tail are done element-wise by block 0 inside the same launch;
//  * operands whose misalignment differs from the destination's (relative
//    offset not a multiple of 16 B) still move in 16-B accesses: their
//    misalignment rides in the buffer instruction's scalar offset;
//  * 64-bit indices throughout (the reference uses `int`, Appendix A.4).
//
// Arithmetic is bit-exact with gloo/math.h evaluated in the same order: see
// include/gloo_amd.h for the contract and the NaN / signed-zero rules.

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "gloo_amd.h"
#include "gloo_amd/errors.h"
#include "gloo_amd/signal.h"

namespace gloo_amd {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// Element traits.  S = storage type.  Integers compute in the unsigned type of
// the same width so overflow wraps (gloo/math.h relies on the platform's
// modular conversion: c[i] = a[i] + b[i] for int8 promotes to int and
// truncates, which is the same low bits).
// ---------------------------------------------------------------------------
template <typename S, typename U>
struct IntTraits {
  using Storage = S;
  __device__ static __forceinline__ S sum(S a, S b) { return (S)(U)((U)a + (U)b); }
  __device__ static __forceinline__ S product(S a, S b) {
    return (S)(U)((U)a * (U)b);
  }
  __device__ static __forceinline__ S max(S a, S b) { return (a < b) ? b : a; }
  __device__ static __forceinline__ S min(S a, S b) { return (b < a) ? b : a; }
};

// uint8 * uint8 promotes to int in C++; 255*255 fits, truncation gives the
// same low byte.  For the 32/64-bit unsigned types the product is already
// unsigned and wraps.
using TrI8 = IntTraits<int8_t, uint32_t>;
using TrU8 = IntTraits<uint8_t, uint32_t>;
using TrI32 = IntTraits<int32_t, uint32_t>;
using TrU32 = IntTraits<uint32_t, uint32_t>;
using TrI64 = IntTraits<int64_t, uint64_t>;
using TrU64 = IntTraits<uint64_t, uint64_t>;

template <typename S>
struct FloatTraits {
  using Storage = S;
  __device__ static __forceinline__ S sum(S a, S b) { return a + b; }
  __device__ static __forceinline__ S product(S a, S b) { return a * b; }
  // std::max(a, b) == (a < b) ? b : a ; std::min(a, b) == (b < a) ? b : a.
  // Written as compare + select so NaN and -0/+0 follow the reference (the
  // IEEE v_max_f32 would return the non-NaN operand instead).
  __device__ static __forceinline__ S max(S a, S b) { return (a < b) ? b : a; }
  __device__ static __forceinline__ S min(S a, S b) { return (b < a) ? b : a; }
};
using TrF32 = FloatTraits<float>;
using TrF64 = FloatTraits<double>;

// IEEE binary16 held as raw bits.  Op in f32, round-to-nearest-even back
// (v_cvt_f16_f32 honours the default RNE mode).  A single f32 rounding
// followed by the f16 rounding equals one correctly rounded f16 result for
// + and * because 24 >= 2*11+2, so this matches F16C (gloo/math.cc:17-97)
// and CUDA __float2half(__half2float(a) op __half2float(b)) (cuda.cu:301-318).
//
// NaN results carry the reference's bits, not the convert's: the F16C body as
// the reference builds it (g++, -mf16c) returns the second operand's NaN
// quietened, else the first's, else x86's default NaN 0xFE00 for an invalid
// operation (inf - inf, 0 * inf).  Probed on oracle/_ref, pinned by
// tests/golden/math_golden.npz "f16_nan/*".  One compare + two selects on the
// rare path's condition; they hide under the memory stream.
struct TrF16 {
  using Storage = uint16_t;
  __device__ static __forceinline__ float widen(uint16_t x) {
    return (float)__builtin_bit_cast(_Float16, x);
  }
  __device__ static __forceinline__ uint16_t narrow(float f) {
    return __builtin_bit_cast(uint16_t, (_Float16)f);
  }
  __device__ static __forceinline__ bool is_nan(uint16_t x) { return (x & 0x7FFFu) > 0x7C00u; }
  __device__ static __forceinline__ uint16_t nan_of(uint16_t a, uint16_t b) {
    return is_nan(b) ? (uint16_t)(b | 0x0200u) : is_nan(a) ? (uint16_t)(a | 0x0200u) : (uint16_t)0xFE00u;
  }
  __device__ static __forceinline__ uint16_t sum(uint16_t a, uint16_t b) {
    const float r = widen(a) + widen(b);
    return r != r ? nan_of(a, b) : narrow(r);
  }
  __device__ static __forceinline__ uint16_t product(uint16_t a, uint16_t b) {
    const float r = widen(a) * widen(b);
    return r != r ? nan_of(a, b) : narrow(r);
  }
  __device__ static __forceinline__ uint16_t max(uint16_t a, uint16_t b) {
    return (widen(a) < widen(b)) ? b : a;
  }
  __device__ static __forceinline__ uint16_t min(uint16_t a, uint16_t b) {
    return (widen(b) < widen(a)) ? b : a;
  }
};

// bfloat16 held as raw bits (c10::BFloat16 semantics: widen by <<16, op in
// f32, round-to-nearest-even back; v_cvt_pk_bf16_f32 on gfx950).  c10's
// round_to_nearest_even returns the canonical 0x7FC0 for every NaN
// (torch/headeronly/util/BFloat16.h:100-108), where the convert keeps sign
// and payload: one compare + select restores the reference's bits.
struct TrBF16 {
  using Storage = uint16_t;
  __device__ static __forceinline__ float widen(uint16_t x) {
    return __builtin_bit_cast(float, (uint32_t)x << 16);
  }
  __device__ static __forceinline__ uint16_t narrow(float f) {
    return f != f ? (uint16_t)0x7FC0u : __builtin_bit_cast(uint16_t, (__bf16)f);
  }
  __device__ static __forceinline__ uint16_t sum(uint16_t a, uint16_t b) {
    return narrow(widen(a) + widen(b));
  }
  __device__ static __forceinline__ uint16_t product(uint16_t a, uint16_t b) {
    return narrow(widen(a) * widen(b));
  }
  __device__ static __forceinline__ uint16_t max(uint16_t a, uint16_t b) {
    return (widen(a) < widen(b)) ? b : a;
  }
  __device__ static __forceinline__ uint16_t min(uint16_t a, uint16_t b) {
    return (widen(b) < widen(a)) ? b : a;
  }
};

template <class Tr, int OP>
__device__ __forceinline__ typename Tr::Storage apply(typename Tr::Storage a,
                                                      typename Tr::Storage b) {
  if constexpr (OP == GLOO_HIP_SUM) return Tr::sum(a, b);
  else if constexpr (OP == GLOO_HIP_PRODUCT) return Tr::product(a, b);
  else if constexpr (OP == GLOO_HIP_MAX) return Tr::max(a, b);
  else return Tr::min(a, b);
}

// Apply the op lane-wise to one 16-byte packet.
template <class Tr, int OP>
__device__ __forceinline__ u32x4 generic_packet(u32x4 a, u32x4 b) {
  using S = typename Tr::Storage;
  constexpr int kV = 16 / sizeof(S);
  union P {
    u32x4 v;
    S e[kV];
  };
  P pa, pb, pc;
  pa.v = a;
  pb.v = b;
#pragma unroll
  for (int i = 0; i < kV; i++) pc.e[i] = apply<Tr, OP>(pa.e[i], pb.e[i]);
  return pc.v;
}
template <class Tr, int OP>
__device__ __forceinline__ u32x4 apply_packet(u32x4 a, u32x4 b) {
  return generic_packet<Tr, OP>(a, b);
}

// Byte-lane SWAR specialisations: 16 int8/uint8 adds in 4 dword ops each
// instead of 16 extract/insert sequences.  Wrap semantics are identical.
__device__ __forceinline__ uint32_t swar_add8(uint32_t a, uint32_t b) {
  return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
}
template <>
__device__ __forceinline__ u32x4 apply_packet<TrI8, GLOO_HIP_SUM>(u32x4 a, u32x4 b) {
  return u32x4{swar_add8(a.x, b.x), swar_add8(a.y, b.y), swar_add8(a.z, b.z),
               swar_add8(a.w, b.w)};
}
template <>
__device__ __forceinline__ u32x4 apply_packet<TrU8, GLOO_HIP_SUM>(u32x4 a, u32x4 b) {
  return u32x4{swar_add8(a.x, b.x), swar_add8(a.y, b.y), swar_add8(a.z, b.z),
               swar_add8(a.w, b.w)};
}

// fp16 SUM / PRODUCT two elements per instruction (v_pk_add_f16 /
// v_pk_mul_f16): one correctly rounded f16 op equals TrF16's f32 op + RNE
// narrowing (24 >= 2*11 + 2), denormals included (gfx9 keeps f16 denormals).
// Only the NaN bits need TrF16's rule: a half is NaN iff
// ((h & 0x7FFF) + 0x03FF) sets bit 15 (no carry leaves the half), so one
// and + add + or per dword finds any NaN of the packet, and such a packet
// (rare in real buckets) gets the rule by bit operations on both halves.
// Measured at 64 MiB (profiles/round4/r4n_*, r4m_*): finite data 31.84 us,
// as bf16 and f32 on the same box; the per-element form it replaces cost
// 3 % (32.6 us) whatever the data.
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
template <int OP>
__device__ __forceinline__ uint32_t f16_pk_dword(uint32_t a, uint32_t b) {
  const h2 x = __builtin_bit_cast(h2, a), y = __builtin_bit_cast(h2, b);
  const h2 z = OP == GLOO_HIP_SUM ? x + y : x * y;
  return __builtin_bit_cast(uint32_t, z);
}
__device__ __forceinline__ uint32_t f16_nan_bits(uint32_t r) { return (r & 0x7FFF7FFFu) + 0x03FF03FFu; }
// 0xFFFF in each half of x that is a NaN
__device__ __forceinline__ uint32_t f16_nan_mask(uint32_t x) { return ((f16_nan_bits(x) >> 15) & 0x00010001u) * 0xFFFFu; }
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t x, uint32_t y) { return (m & x) | (~m & y); }
// TrF16's NaN rule on both halves at once: where the result r is NaN, b's
// NaN quietened, else a's, else 0xFE00
__device__ __forceinline__ uint32_t f16_fix_nans(uint32_t a, uint32_t b, uint32_t r) {
  const uint32_t fix = bsel(f16_nan_mask(b), b | 0x02000200u, bsel(f16_nan_mask(a), a | 0x02000200u, 0xFE00FE00u));
  return bsel(f16_nan_mask(r), fix, r);
}
template <int OP>
__device__ __forceinline__ u32x4 f16_pk_packet(u32x4 a, u32x4 b) {
  u32x4 r = u32x4{f16_pk_dword<OP>(a.x, b.x), f16_pk_dword<OP>(a.y, b.y), f16_pk_dword<OP>(a.z, b.z),
                  f16_pk_dword<OP>(a.w, b.w)};
  const uint32_t nan = f16_nan_bits(r.x) | f16_nan_bits(r.y) | f16_nan_bits(r.z) | f16_nan_bits(r.w);
  if (__builtin_expect((nan & 0x80008000u) != 0, 0))
    r = u32x4{f16_fix_nans(a.x, b.x, r.x), f16_fix_nans(a.y, b.y, r.y), f16_fix_nans(a.z, b.z, r.z),
              f16_fix_nans(a.w, b.w, r.w)};
  return r;
}
template <>
__device__ __forceinline__ u32x4 apply_packet<TrF16, GLOO_HIP_SUM>(u32x4 a, u32x4 b) {
  return f16_pk_packet<GLOO_HIP_SUM>(a, b);
}
template <>
__device__ __forceinline__ u32x4 apply_packet<TrF16, GLOO_HIP_PRODUCT>(u32x4 a, u32x4 b) {
  return f16_pk_packet<GLOO_HIP_PRODUCT>(a, b);
}

// Buffer resources.  Each workgroup builds descriptors whose base is its own
// tile (wave-uniform, SGPRs) and whose range is the bytes left in the body, so
// 32-bit lane offsets suffice for any chunk size and the hardware range check
// drops the out-of-range packets of a ragged last tile (loads return 0, stores
// are discarded) without per-lane branches.
constexpr int kRsrcFlags = 0x00020000;  // gfx950 raw-buffer word 3
constexpr int kAuxNT = 2;               // cache policy `nt`: streamed once
constexpr int kAuxWT = 1 | 2 | 16;      // `sc0 nt sc1`: streamed once, written through (not held in L2)

// Completion protocol of the kernels that signal a peer after writing into
// its inbox (copy_signal_kernel, fold_send_kernel, the interpreter): the
// signalled bytes are stored write-through (sc0 nt sc1) and every wave waits
// for them (vmcnt 0) before its workgroup takes a relaxed ticket; no L2
// write-back is needed except by a workgroup that also made plain stores (the
// edge elements), and the ticket holder publishes the flag with a relaxed
// store.  The interpreter's sends work the same way, and its credits (NOTIFY)
// publish no data, so neither releases.  (Rounds 1-2 released at system scope
// in every workgroup: 4x slower at 16 MiB; that protocol and its
// switch are gone.)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, kRsrcFlags);
}
template <int AUX>
__device__ __forceinline__ u32x4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff = 0) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, AUX);
}

// A source operand of the vector body: its first body byte sits `mis` bytes
// past a 16-B boundary (0 when it is congruent with the destination).  The
// descriptor is based at the aligned-down address and `mis` rides in the
// instruction's scalar offset, so a relatively misaligned operand still
// moves in 16-B accesses (gfx950 runs global/buffer accesses in unaligned
// mode; the compiler itself emits dwordx4 for byte-aligned data).
struct Src {
  const char* base;  // 16-B aligned
  uint32_t mis;      // 0..15
};
__device__ __forceinline__ Src src_of(const void* body) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(body);
  return Src{reinterpret_cast<const char*>(p & ~uintptr_t(15)), (uint32_t)(p & 15)};
}
template <int AUX>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v, uint32_t soff = 0) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, soff, AUX);
}

// Element-wise head / tail: elements [0, head) and [tail0, n) of the chunk,
// done by the first block's lanes.  Disjoint from the vector body, so safe
// under c == a aliasing.
template <class Tr, int OP>
__device__ __forceinline__ void edges(typename Tr::Storage* c,
                                      const typename Tr::Storage* a,
                                      const typename Tr::Storage* b,
                                      size_t head, size_t tail0, size_t n) {
  const size_t t = threadIdx.x;
  if (t < head) c[t] = apply<Tr, OP>(a[t], b[t]);
  const size_t j = tail0 + t;
  if (j < n) c[j] = apply<Tr, OP>(a[j], b[j]);
}

// Device-side kernel timing (the executor's stamp mode, executor.h).  A
// stamp slot is kStampShards begin words and kStampShards end words, each on
// its own 128-B line (signal.h).  Workgroups 0..kStampHead-1 fold their start
// time into begin shard blockIdx % kStampShards (atomic min); the last
// kStampTail workgroups of the grid, once all their waves' stores have
// completed, fold their end time into an end shard (atomic max); the 100 MHz
// constant clock.  Dispatch is in blockIdx order, so the first workgroup to
// start is among the first kStampHead and the last to finish among the last
// kStampTail.  Sharding matters: one device-scope atomic word retires about
// 88 updates per microsecond, so one stamp per workgroup on a single word
// stretched a 16,384-workgroup fold by ~100 us (profiles/round2/
// r2k_stamp_check.jsonl).  stamp == nullptr (every other launch): one uniform
// branch each.  Unlike host events, stamps survive hipGraph capture and
// replay and exclude the dispatch gap between launches.
constexpr unsigned kStampHead = 1024, kStampTail = 4096;
__device__ __forceinline__ void stamp_begin(uint64_t* stamp) {
  if (stamp && threadIdx.x == 0 && blockIdx.x < kStampHead)
    __hip_atomic_fetch_min(stamp + (blockIdx.x % kStampShards) * kStampLineWords, __builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stamp_end(uint64_t* stamp) {
  if (!stamp || blockIdx.x + kStampTail < gridDim.x) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_max(stamp + (kStampShards + blockIdx.x % kStampShards) * kStampLineWords,
                           __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void stamp_init_kernel(uint64_t* stamps, size_t words) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < words) stamps[i] = (i % kStampSlotWords) < kStampShards * kStampLineWords ? ~0ull : 0ull;
}

thread_local uint64_t* t_stamp = nullptr;  // stamp slot of the next reduce launch on this thread
thread_local bool t_plainStores = false;   // setReducePlainStores

// Vector body.  `head` elements bring the destination c to a 16-B boundary;
// a and b may sit at any element offset relative to it (Src).  One workgroup = one tile of BLOCK lanes x UNROLL
// 16-B packets per operand; packet u of lane t sits at (t + u*BLOCK)*16 bytes
// into the tile, so every wave-instruction covers 1 KiB contiguous.  All loads
// of the tile are issued before the first use.  Measured on MI355X (profiles/
// round1): `nt` on both loads and stores, UNROLL 2, BLOCK 512, one tile per
// workgroup is the fastest of 126 variants for the 64 MiB fp32 chunk.
//
// IL: the two operands' loads issued interleaved, packet by packet (a0 b0 a1
// b1), instead of stream by stream (a0 a1 b0 b1, the default).  Round 3 made
// IL the default on stripped-harness readings within the run-to-run spread
// (profiles/round3/r3ab_*, r3ac_*); round 6 timed the product kernel both ways
// in two sessions, interleaved over 3 and 10 repetitions of 500 launches at
// 64 MiB (profiles/round6/r6ad/, r6ae/): stream by stream 0.8023 / 0.8000 of
// 8 TB/s against 0.7986 / 0.7971 interleaved, equal at 16 MiB (0.6743 against
// 0.6745), so the default went back to stream by stream (variant 15 keeps IL).
template <class Tr, int OP, int UNROLL, int BLOCK, int LAUX, int SAUX, int IL = 0>
__global__ __launch_bounds__(BLOCK) void reduce_vec_kernel(
    typename Tr::Storage* c, const typename Tr::Storage* a,
    const typename Tr::Storage* b, size_t n, size_t head, uint64_t* stamp) {
  using S = typename Tr::Storage;
  constexpr int kV = 16 / sizeof(S);
  constexpr uint32_t kTileBytes = (uint32_t)BLOCK * UNROLL * 16;
  stamp_begin(stamp);
  const size_t nvec = (n - head) / kV;
  if (blockIdx.x == 0) edges<Tr, OP>(c, a, b, head, head + nvec * kV, n);

  const size_t body = nvec * 16;
  const size_t base = (size_t)blockIdx.x * kTileBytes;
  if (base >= body) return;
  const uint32_t bytes = (uint32_t)((body - base) < kTileBytes ? (body - base) : kTileBytes);
  const Src sa = src_of(a + head), sb = src_of(b + head);
  const auto ra = make_rsrc(sa.base + base, bytes + sa.mis);
  const auto rb = make_rsrc(sb.base + base, bytes + sb.mis);
  const auto rc = make_rsrc(reinterpret_cast<const char*>(c + head) + base, bytes);
  const uint32_t lane_off = threadIdx.x * 16u;
  u32x4 x[UNROLL], y[UNROLL];
  if constexpr (IL) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      x[u] = bload<LAUX>(ra, lane_off + u * BLOCK * 16, sa.mis);
      y[u] = bload<LAUX>(rb, lane_off + u * BLOCK * 16, sb.mis);
    }
  } else {
#pragma unroll
    for (int u = 0; u < UNROLL; u++) x[u] = bload<LAUX>(ra, lane_off + u * BLOCK * 16, sa.mis);
#pragma unroll
    for (int u = 0; u < UNROLL; u++) y[u] = bload<LAUX>(rb, lane_off + u * BLOCK * 16, sb.mis);
  }
#pragma unroll
  for (int u = 0; u < UNROLL; u++)
    bstore<SAUX>(rc, lane_off + u * BLOCK * 16, apply_packet<Tr, OP>(x[u], y[u]));
  stamp_end(stamp);
}

// Software-pipelined persistent form (measurement variants 9-12): a grid of
// G workgroups walks tiles g, g + G, ...; the loads of the next tile are in
// flight while the current one is combined and stored, so a workgroup keeps
// two tiles outstanding and the grid pays one dispatch ramp for many tiles.
template <class Tr, int OP, int UNROLL, int BLOCK, int LAUX, int SAUX>
__global__ __launch_bounds__(BLOCK) void reduce_vec_pipe_kernel(
    typename Tr::Storage* c, const typename Tr::Storage* a,
    const typename Tr::Storage* b, size_t n, size_t head) {
  using S = typename Tr::Storage;
  constexpr int kV = 16 / sizeof(S);
  constexpr uint32_t kTileBytes = (uint32_t)BLOCK * UNROLL * 16;
  const size_t nvec = (n - head) / kV;
  if (blockIdx.x == 0) edges<Tr, OP>(c, a, b, head, head + nvec * kV, n);
  const size_t body = nvec * 16;
  const Src sa = src_of(a + head), sb = src_of(b + head);
  const char* cbase = reinterpret_cast<const char*>(c + head);
  const uint32_t lane_off = threadIdx.x * 16u;
  const size_t stride = (size_t)gridDim.x * kTileBytes;
  size_t base = (size_t)blockIdx.x * kTileBytes;
  if (base >= body) return;
  u32x4 x[UNROLL], y[UNROLL], nx[UNROLL], ny[UNROLL];
  {
    const uint32_t bytes = (uint32_t)((body - base) < kTileBytes ? (body - base) : kTileBytes);
    const auto ra = make_rsrc(sa.base + base, bytes + sa.mis);
    const auto rb = make_rsrc(sb.base + base, bytes + sb.mis);
#pragma unroll
    for (int u = 0; u < UNROLL; u++) x[u] = bload<LAUX>(ra, lane_off + u * BLOCK * 16, sa.mis);
#pragma unroll
    for (int u = 0; u < UNROLL; u++) y[u] = bload<LAUX>(rb, lane_off + u * BLOCK * 16, sb.mis);
  }
  for (;;) {
    const size_t next = base + stride;
    const bool more = next < body;
    if (more) {
      const uint32_t nbytes = (uint32_t)((body - next) < kTileBytes ? (body - next) : kTileBytes);
      const auto ra = make_rsrc(sa.base + next, nbytes + sa.mis);
      const auto rb = make_rsrc(sb.base + next, nbytes + sb.mis);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) nx[u] = bload<LAUX>(ra, lane_off + u * BLOCK * 16, sa.mis);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) ny[u] = bload<LAUX>(rb, lane_off + u * BLOCK * 16, sb.mis);
    }
    const uint32_t bytes = (uint32_t)((body - base) < kTileBytes ? (body - base) : kTileBytes);
    const auto rc = make_rsrc(cbase + base, bytes);
#pragma unroll
    for (int u = 0; u < UNROLL; u++) bstore<SAUX>(rc, lane_off + u * BLOCK * 16, apply_packet<Tr, OP>(x[u], y[u]));
    if (!more) break;
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      x[u] = nx[u];
      y[u] = ny[u];
    }
    base = next;
  }
}

// Multi-source left fold dst = ((s0 op s1) op s2) ... in one pass.
struct SrcList {
  const void* p[GLOO_HIP_MAX_SRCS];
};

// MODE 0: left fold acc = acc op s_j.  MODE 1 (reverse): acc = s_j op acc,
// the fold a ring schedule performs when every hop computes `local op
// incoming`.  MODE 2 (tree): balanced pairwise tree over the sources in order
// (k a power of two), the fold of recursive halving.
template <class Tr, int OP>
__device__ __forceinline__ typename Tr::Storage tree_fold(typename Tr::Storage* v, int k) {
#pragma unroll
  for (int w = GLOO_HIP_MAX_SRCS; w > 1; w >>= 1)
    if (w <= k) {
#pragma unroll
      for (int j = 0; j < w / 2; j++) v[j] = apply<Tr, OP>(v[2 * j], v[2 * j + 1]);
    }
  return v[0];
}

// One element of a k-source fold (block 0's head / tail), in MODE's order.
template <class Tr, int OP, int MODE>
__device__ __forceinline__ typename Tr::Storage fold_elem(const SrcList& srcs, int k, size_t i) {
  using S = typename Tr::Storage;
  if (MODE == 2) {
    S v[GLOO_HIP_MAX_SRCS];
#pragma unroll
    for (int j = 0; j < GLOO_HIP_MAX_SRCS; j++)
      if (j < k) v[j] = static_cast<const S*>(srcs.p[j])[i];
    return tree_fold<Tr, OP>(v, k);
  }
  S acc = static_cast<const S*>(srcs.p[0])[i];
  for (int j = 1; j < k; j++) {
    const S v = static_cast<const S*>(srcs.p[j])[i];
    acc = MODE == 1 ? apply<Tr, OP>(v, acc) : apply<Tr, OP>(acc, v);
  }
  return acc;
}

// One vector tile of a k-source fold: `bytes` (<= BLOCK * UNROLL * 16) of
// the body starting `base` bytes past element `head`, into acc.
// FOLD_PRELOAD=1: the chain folds (MODE 0 / 1) issue every source's loads
// before the first op, as the tree does.  Measured slower (round 4, 64 MiB
// fp32 per source, profiles/round4/r4t_multi_*: k = 4..8 at 54.3-98.7 us
// against 53.1-97.8 us loading source by source): the extra VGPRs cost
// more waves than the extra loads in flight gain.  So the default (0) keeps
// two tiles per source step and relies on occupancy.
#ifndef FOLD_PRELOAD
#define FOLD_PRELOAD 0
#endif
template <class Tr, int OP, int UNROLL, int BLOCK, int MODE>
__device__ __forceinline__ void fold_tile(const SrcList& srcs, int k, size_t head, size_t base, uint32_t bytes,
                                          u32x4 (&acc)[UNROLL]) {
  using S = typename Tr::Storage;
  const uint32_t lane_off = threadIdx.x * 16u;
  if (MODE == 2) {
    // all sources resident, then the tree level by level (k <= 8, uniform)
    u32x4 v[GLOO_HIP_MAX_SRCS][UNROLL];
#pragma unroll
    for (int j = 0; j < GLOO_HIP_MAX_SRCS; j++)
      if (j < k) {
        const Src sj = src_of(static_cast<const S*>(srcs.p[j]) + head);
        const auto rj = make_rsrc(sj.base + base, bytes + sj.mis);
#pragma unroll
        for (int u = 0; u < UNROLL; u++) v[j][u] = bload<kAuxNT>(rj, lane_off + u * BLOCK * 16, sj.mis);
      }
#pragma unroll
    for (int w = GLOO_HIP_MAX_SRCS; w > 1; w >>= 1)
      if (w <= k) {
#pragma unroll
        for (int j = 0; j < w / 2; j++)
#pragma unroll
          for (int u = 0; u < UNROLL; u++) v[j][u] = apply_packet<Tr, OP>(v[2 * j][u], v[2 * j + 1][u]);
      }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) acc[u] = v[0][u];
  } else if (FOLD_PRELOAD) {
    // every source's loads in flight before the first op (k <= 8, uniform),
    // then the chain in order: a k-source fold keeps k tiles in flight per
    // wave instead of two
    u32x4 v[GLOO_HIP_MAX_SRCS][UNROLL];
#pragma unroll
    for (int j = 0; j < GLOO_HIP_MAX_SRCS; j++)
      if (j < k) {
        const Src sj = src_of(static_cast<const S*>(srcs.p[j]) + head);
        const auto rj = make_rsrc(sj.base + base, bytes + sj.mis);
#pragma unroll
        for (int u = 0; u < UNROLL; u++) v[j][u] = bload<kAuxNT>(rj, lane_off + u * BLOCK * 16, sj.mis);
      }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) acc[u] = v[0][u];
#pragma unroll
    for (int j = 1; j < GLOO_HIP_MAX_SRCS; j++)
      if (j < k) {
#pragma unroll
        for (int u = 0; u < UNROLL; u++)
          acc[u] = MODE == 1 ? apply_packet<Tr, OP>(v[j][u], acc[u]) : apply_packet<Tr, OP>(acc[u], v[j][u]);
      }
  } else {
    {
      const Src s0 = src_of(static_cast<const S*>(srcs.p[0]) + head);
      const auto r0 = make_rsrc(s0.base + base, bytes + s0.mis);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) acc[u] = bload<kAuxNT>(r0, lane_off + u * BLOCK * 16, s0.mis);
    }
    for (int j = 1; j < k; j++) {
      const Src sj = src_of(static_cast<const S*>(srcs.p[j]) + head);
      const auto rj = make_rsrc(sj.base + base, bytes + sj.mis);
      u32x4 r[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) r[u] = bload<kAuxNT>(rj, lane_off + u * BLOCK * 16, sj.mis);
#pragma unroll
      for (int u = 0; u < UNROLL; u++)
        acc[u] = MODE == 1 ? apply_packet<Tr, OP>(r[u], acc[u]) : apply_packet<Tr, OP>(acc[u], r[u]);
    }
  }
}

template <class Tr, int OP, int UNROLL, int BLOCK, int MODE>
__global__ __launch_bounds__(BLOCK) void reduce_multi_vec_kernel(
    typename Tr::Storage* dst, SrcList srcs, int k, size_t n, size_t head, uint64_t* stamp, int plain) {
  using S = typename Tr::Storage;
  constexpr int kV = 16 / sizeof(S);
  constexpr uint32_t kTileBytes = (uint32_t)BLOCK * UNROLL * 16;
  stamp_begin(stamp);
  const size_t nvec = (n - head) / kV;
  const size_t tail0 = head + nvec * kV;
  if (blockIdx.x == 0) {
    const size_t t = threadIdx.x;
    for (int pass = 0; pass < 2; pass++) {
      const size_t i = pass == 0 ? t : tail0 + t;
      if ((pass == 0 && t < head) || (pass == 1 && i < n)) dst[i] = fold_elem<Tr, OP, MODE>(srcs, k, i);
    }
  }
  const size_t body = nvec * 16;
  const size_t base = (size_t)blockIdx.x * kTileBytes;
  if (base >= body) return;
  const uint32_t bytes = (uint32_t)((body - base) < kTileBytes ? (body - base) : kTileBytes);
  const uint32_t lane_off = threadIdx.x * 16u;
  u32x4 acc[UNROLL];
  fold_tile<Tr, OP, UNROLL, BLOCK, MODE>(srcs, k, head, base, bytes, acc);
  const auto rd = make_rsrc(reinterpret_cast<const char*>(dst + head) + base, bytes);
  if (plain) {  // the executor's folds: the result's next reader is a send or the caller (setReducePlainStores)
#pragma unroll
    for (int u = 0; u < UNROLL; u++) bstore<0>(rd, lane_off + u * BLOCK * 16, acc[u]);
  } else {
#pragma unroll
    for (int u = 0; u < UNROLL; u++) bstore<kAuxNT>(rd, lane_off + u * BLOCK * 16, acc[u]);
  }
  stamp_end(stamp);
}

// ---------------------------------------------------------------------------
// Fused small-message step: [wait for a flag] -> dst (op)= src over n
// elements (OP 0: plain copy) -> [signal a flag].  One workgroup: for chunks
// of a few KiB a schedule hop is dispatch-bound, so the executor folds the
// wait / reduce-or-copy / notify chain of a plan into this one launch.
// Protocol (MI355X_MICROARCH.md, inter-workgroup visibility): ONE lane polls
// relaxed, ONE system-scope acquire, barrier, then plain loads; every wave
// drains its memory ops (vmcnt(0)) before the barrier that precedes the
// single system-scope release + flag store.
// ---------------------------------------------------------------------------
constexpr int kFusedBlock = 512;

template <class Tr, int OP>
__global__ __launch_bounds__(kFusedBlock) void fused_small_kernel(
    typename Tr::Storage* dst, const typename Tr::Storage* src, size_t n, const uint64_t* waitFlag,
    Seq wait, uint64_t timeoutTicks, uint32_t* err, uint64_t* sigFlag, Seq sig, const uint64_t* epoch) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    int good = 1;
    if (waitFlag) {
      const uint64_t waitTarget = epoch ? wait.base + *epoch * wait.perRun : wait.base;
      // counters compare by signed difference: a target "below" the counter
      // (a previous-run credit in the first run) is satisfied
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while ((int64_t)(__hip_atomic_load(waitFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - waitTarget) < 0) {
        __builtin_amdgcn_s_sleep(4);
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeoutTicks) {
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          good = 0;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    ok = good;
  }
  __syncthreads();
  if (!ok) return;  // timed out: no work, no signal (the host raises)
  for (size_t i = threadIdx.x; i < n; i += kFusedBlock) {
    if constexpr (OP == 0) dst[i] = src[i];
    else dst[i] = apply<Tr, OP>(dst[i], src[i]);
  }
  if (sigFlag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t sigValue = epoch ? sig.base + *epoch * sig.perRun : sig.base;
      // one release, then a relaxed flag store: a release store would write
      // the L2 back a second time (MI355X_MICROARCH.md: fence, wait, relaxed flag)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(sigFlag, sigValue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <class Tr>
int launch_fused(int op, void* dst, const void* src, size_t n, const uint64_t* wf, Seq wt, uint64_t tt,
                 uint32_t* err, uint64_t* sf, Seq sv, const uint64_t* ep, hipStream_t s) {
  using S = typename Tr::Storage;
  S* d = static_cast<S*>(dst);
  const S* x = static_cast<const S*>(src);
  switch (op) {
    case 0: fused_small_kernel<Tr, 0><<<1, kFusedBlock, 0, s>>>(d, x, n, wf, wt, tt, err, sf, sv, ep); break;
    case GLOO_HIP_SUM: fused_small_kernel<Tr, GLOO_HIP_SUM><<<1, kFusedBlock, 0, s>>>(d, x, n, wf, wt, tt, err, sf, sv, ep); break;
    case GLOO_HIP_PRODUCT: fused_small_kernel<Tr, GLOO_HIP_PRODUCT><<<1, kFusedBlock, 0, s>>>(d, x, n, wf, wt, tt, err, sf, sv, ep); break;
    case GLOO_HIP_MAX: fused_small_kernel<Tr, GLOO_HIP_MAX><<<1, kFusedBlock, 0, s>>>(d, x, n, wf, wt, tt, err, sf, sv, ep); break;
    case GLOO_HIP_MIN: fused_small_kernel<Tr, GLOO_HIP_MIN><<<1, kFusedBlock, 0, s>>>(d, x, n, wf, wt, tt, err, sf, sv, ep); break;
    default: return GLOO_HIP_EINVAL_OP;
  }
  return GLOO_HIP_OK;
}

// ---------------------------------------------------------------------------
// One-launch plan interpreter (signal.h InterpStep): one workgroup walks the
// whole step list of a small plan.  Visibility follows the fused step's
// protocol: every data step ends with each wave draining its memory
// operations (vmcnt 0) and a workgroup barrier, so a following send / signal
// can publish them with ONE lane's system-scope release + flag store; a wait
// has ONE lane poll relaxed, then ONE system-scope acquire, then a barrier
// before any lane reads the inbox.
// ---------------------------------------------------------------------------
#ifndef GLOO_AMD_INTERP_BLOCK
#define GLOO_AMD_INTERP_BLOCK 512
#endif
#ifndef GLOO_AMD_INTERP_COPY_UNROLL
#define GLOO_AMD_INTERP_COPY_UNROLL 8
#endif
#ifndef GLOO_AMD_INTERP_FOLD_UNROLL
#define GLOO_AMD_INTERP_FOLD_UNROLL 4
#endif
constexpr int kInterpBlock = GLOO_AMD_INTERP_BLOCK;
// Packets per lane in flight per pass: a pass costs ONE memory latency (all
// of its loads issue before the first use), so a 64 KiB copy is one pass and
// a fold moves 32 KiB per source per pass (210-223 VGPRs, no spills: still
// one 512-lane workgroup per CU, as with 4 / 2 packets; 4 MiB HD per rank
// 32.8 us against 34.2 us, profiles/round3/r3y_latency_interp_variants.jsonl).
constexpr int kInterpCopyUnroll = GLOO_AMD_INTERP_COPY_UNROLL;
constexpr int kInterpFoldUnroll = GLOO_AMD_INTERP_FOLD_UNROLL;

// Bytes [0, n) of src to dst.  The destination is brought to a 16-byte
// boundary element-wise (head); the body then moves in 16-byte packets
// whatever the source's misalignment (Src: aligned-down descriptor base, the
// byte offset in the buffer instruction's soffset, as reduce_vec_kernel);
// the ragged tail goes byte-wise.  Per pass the descriptors are rebuilt at
// the pass base, so 32-bit lane offsets suffice, and the range check drops
// the packets past the body.
// A byte stored write-through (`sc0 nt sc1`), for the edges of a WT copy.
__device__ __forceinline__ void wt_byte(char* p, char v) {
  __builtin_amdgcn_raw_buffer_store_b8((unsigned char)v, make_rsrc(p, 1), 0, 0, kAuxWT);
}

// WT: every byte of dst is stored write-through (an interpreter SEND under
// the once-per-launch protocol, fwdLean: its flag then needs no release).
template <bool WT = false>
__device__ __forceinline__ void interp_copy(char* dst, const char* src, uint64_t n) {
  const uint64_t t = threadIdx.x;
  uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
  if (head > n) head = n;
  if (t < head) {
    if (WT) wt_byte(dst + t, src[t]);
    else dst[t] = src[t];
  }
  const uint64_t body = (n - head) / 16 * 16;
  char* d = dst + head;
  const Src ss = src_of(src + head);
  constexpr uint64_t kPass = (uint64_t)kInterpBlock * kInterpCopyUnroll * 16;
  const uint32_t lane_off = (uint32_t)t * 16u;
  for (uint64_t b = 0; b < body; b += kPass) {
    const uint32_t bytes = (uint32_t)(body - b < kPass ? body - b : kPass);
    const auto rs = make_rsrc(ss.base + b, bytes + ss.mis);
    const auto rd = make_rsrc(d + b, bytes);
    u32x4 v[kInterpCopyUnroll];
#pragma unroll
    for (int u = 0; u < kInterpCopyUnroll; u++) v[u] = bload<0>(rs, lane_off + u * kInterpBlock * 16, ss.mis);
#pragma unroll
    for (int u = 0; u < kInterpCopyUnroll; u++) bstore<WT ? kAuxWT : 0>(rd, lane_off + u * kInterpBlock * 16, v[u]);
  }
  for (uint64_t i = head + body + t; i < n; i += kInterpBlock) {
    if (WT) wt_byte(dst + i, src[i]);
    else dst[i] = src[i];
  }
}

// dst[i] = fold over the step's sources (mode as launchFold) for n elements:
// the destination's head element-wise up to a 16-byte boundary, then
// 16-byte packets with every source at its own misalignment (soffset, as
// interp_copy), then the ragged tail element-wise.
template <class Tr, int OP>
__device__ __forceinline__ void interp_fold(const InterpStep& st, uint64_t lo, uint64_t hi) {
  using S = typename Tr::Storage;
  constexpr int kV = 16 / sizeof(S);
  // byte lanes unpack 16 per packet: one packet per lane keeps them in VGPRs
  constexpr int kU = sizeof(S) == 1 ? 1 : kInterpFoldUnroll;
  const int ns = st.nsrc, mode = st.mode;
  const uint64_t n = hi - lo;
  const uint64_t t = threadIdx.x;
  const char* src[GLOO_HIP_MAX_SRCS];
  char* dstp = st.dst + lo * sizeof(S);
#pragma unroll
  for (int j = 0; j < GLOO_HIP_MAX_SRCS; j++) src[j] = j < ns ? st.src[j] + lo * sizeof(S) : nullptr;
  auto one = [&](uint64_t i) {
    S e[GLOO_HIP_MAX_SRCS];
#pragma unroll
    for (int j = 0; j < GLOO_HIP_MAX_SRCS; j++)
      if (j < ns) e[j] = reinterpret_cast<const S*>(src[j])[i];
    if (mode == 2) {
      reinterpret_cast<S*>(dstp)[i] = tree_fold<Tr, OP>(e, ns);
    } else {
      S acc = e[0];
#pragma unroll
      for (int j = 1; j < GLOO_HIP_MAX_SRCS; j++)
        if (j < ns) acc = mode == 1 ? apply<Tr, OP>(e[j], acc) : apply<Tr, OP>(acc, e[j]);
      reinterpret_cast<S*>(dstp)[i] = acc;
    }
  };
  uint64_t head = ((16 - ((uintptr_t)dstp & 15)) & 15) / sizeof(S);
  if (head > n) head = n;
  const uint64_t nv = (n - head) / kV;
  const uint64_t body = nv * 16;
  char* dbody = dstp + head * sizeof(S);
  constexpr uint64_t kPass = (uint64_t)kInterpBlock * kU * 16;
  const uint32_t lane_off = (uint32_t)t * 16u;
  for (uint64_t b = 0; b < body; b += kPass) {
    const uint32_t bytes = (uint32_t)(body - b < kPass ? body - b : kPass);
    u32x4 v[GLOO_HIP_MAX_SRCS][kU];
#pragma unroll
    for (int j = 0; j < GLOO_HIP_MAX_SRCS; j++)
      if (j < ns) {
        const Src sj = src_of(src[j] + head * sizeof(S));
        const auto rj = make_rsrc(sj.base + b, bytes + sj.mis);
#pragma unroll
        for (int u = 0; u < kU; u++) v[j][u] = bload<0>(rj, lane_off + u * kInterpBlock * 16, sj.mis);
      }
    if (mode == 2) {
#pragma unroll
      for (int w = GLOO_HIP_MAX_SRCS; w > 1; w >>= 1)
        if (w <= ns) {
#pragma unroll
          for (int j = 0; j < w / 2; j++)
#pragma unroll
            for (int u = 0; u < kU; u++) v[j][u] = apply_packet<Tr, OP>(v[2 * j][u], v[2 * j + 1][u]);
        }
    } else {
#pragma unroll
      for (int j = 1; j < GLOO_HIP_MAX_SRCS; j++)
        if (j < ns) {
#pragma unroll
          for (int u = 0; u < kU; u++)
            v[0][u] = mode == 1 ? apply_packet<Tr, OP>(v[j][u], v[0][u]) : apply_packet<Tr, OP>(v[0][u], v[j][u]);
        }
    }
    const auto rd = make_rsrc(dbody + b, bytes);
#pragma unroll
    for (int u = 0; u < kU; u++) bstore<0>(rd, lane_off + u * kInterpBlock * 16, v[0][u]);
  }
  // the head [0, head) and the ragged tail [head + nv * kV, n), one loop
  const uint64_t tail0 = head + nv * kV, edge = head + (n - tail0);
  for (uint64_t k = t; k < edge; k += kInterpBlock) one(k < head ? k : tail0 + (k - head));
}

template <class Tr, int OP>
__global__ __launch_bounds__(kInterpBlock) void plan_interp_kernel(const InterpStep* steps, int nsteps, uint64_t run,
                                                                   uint64_t timeoutTicks, uint32_t* err,
                                                                   uint64_t* done, unsigned* doneTicket) {
  using S = typename Tr::Storage;
  constexpr uint64_t kV = 16 / sizeof(S);
  __shared__ int ok;
  const uint64_t g = blockIdx.x, G = gridDim.x;
  int good = 1;   // lane 0: no wait of this launch has timed out
  int batch = 0;  // first step of the current batch (kInterpDefer)
  for (int k = 0; k < nsteps; k++) {
    const InterpStep& st = steps[k];
    const int kind = st.kind;
    const bool defer = st.flags & kInterpDefer;
    if (kind == kInterpWait) {
      if (threadIdx.x == 0) {
        const uint64_t value = st.base + run * st.perRun;
        const uint64_t* flag = st.flag + g;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        // signed difference: a target below the counter is already met
        while (good && (int64_t)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - value) < 0) {
          __builtin_amdgcn_s_sleep(2);
          if (__builtin_amdgcn_s_memrealtime() - t0 > timeoutTicks) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            good = 0;
          }
        }
        // a batch of waits: every flag polled first, then ONE acquire (it
        // orders every relaxed load above before the inbox reads below)
        if (!defer) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          ok = good;
        }
      }
      batch = k + 1;
      if (defer) continue;
      __syncthreads();
      if (!ok) return;  // timed out: no further work, no further signal
      continue;
    }
    // this workgroup's slice of the step (signal.h): 16-byte granular
    const uint64_t n = st.n;
    const uint64_t q = ((n + G - 1) / G + kV - 1) / kV * kV;
    const uint64_t lo = g * q < n ? g * q : n;
    const uint64_t hi = lo + q < n ? lo + q : n;
    if (kind == kInterpSend) {
      interp_copy<true>(st.dst + lo * sizeof(S), st.src[0] + lo * sizeof(S), (hi - lo) * sizeof(S));
    } else if (kind == kInterpCopy || kind == kInterpSend) {
      interp_copy(st.dst + lo * sizeof(S), st.src[0] + lo * sizeof(S), (hi - lo) * sizeof(S));
    } else if (kind == kInterpFold) {
      interp_fold<Tr, OP>(st, lo, hi);
    }
    // the next step neither reads nor writes what this one touches: keep
    // this step's memory operations in flight, publish its flag with the batch's
    if (defer) continue;
    // every wave's reads and writes of the batch are performed before the barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      // a SEND's bytes went out write-through and a SIGNAL is a credit that
      // publishes no data (its reads are complete), so neither needs the L2
      // write-back of a release
      for (int j = batch; j <= k; j++) {
        const InterpStep& sj = steps[j];
        if (sj.kind != kInterpSend && sj.kind != kInterpSignal) continue;
        __hip_atomic_store(sj.flag + g, sj.base + run * sj.perRun, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    batch = k + 1;
  }
  if (!done) return;
  // The run's completion for a host that spins on `done` instead of
  // synchronising the stream (signal.h): every workgroup's stores are
  // performed and released before it takes its ticket; the workgroup taking
  // the last ticket resets the counter and publishes the run.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const unsigned t = __hip_atomic_fetch_add(doneTicket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t == G - 1) {
      __hip_atomic_store(doneTicket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(done, run, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <class Tr>
int launch_interp(int op, const InterpStep* steps, int nsteps, uint64_t run, uint64_t tt, uint32_t* err,
                  int G, hipStream_t s, uint64_t* done, unsigned* dt) {
  switch (op) {
    case GLOO_HIP_SUM: plan_interp_kernel<Tr, GLOO_HIP_SUM><<<G, kInterpBlock, 0, s>>>(steps, nsteps, run, tt, err, done, dt); break;
    case GLOO_HIP_PRODUCT: plan_interp_kernel<Tr, GLOO_HIP_PRODUCT><<<G, kInterpBlock, 0, s>>>(steps, nsteps, run, tt, err, done, dt); break;
    case GLOO_HIP_MAX: plan_interp_kernel<Tr, GLOO_HIP_MAX><<<G, kInterpBlock, 0, s>>>(steps, nsteps, run, tt, err, done, dt); break;
    case GLOO_HIP_MIN: plan_interp_kernel<Tr, GLOO_HIP_MIN><<<G, kInterpBlock, 0, s>>>(steps, nsteps, run, tt, err, done, dt); break;
    default: return GLOO_HIP_EINVAL_OP;
  }
  return GLOO_HIP_OK;
}

// ---------------------------------------------------------------------------
// Peer copy with the arrival signal fused in: the SEND of a plan as one
// launch.  A capped grid walks 16 KiB tiles (512 lanes x 2 x 16 B): loads
// from local HBM (`nt`, any misalignment via soffset), 16-B stores into the
// peer's inbox (over xGMI when it is another GPU).  Completion: every wave
// drains (vmcnt 0), the workgroup syncs, one lane releases at system scope
// and takes a ticket; the workgroup holding the last ticket of this launch
// resets the counter and publishes `*flag = seq` (MI355X_MICROARCH.md:
// counter fan-in + flag).
// ---------------------------------------------------------------------------
constexpr int kCopyBlock = 512;
constexpr int kCopyUnroll = 2;
constexpr int kMaxCopies = kMaxCopyEntries;

// Several copies in one launch (the mesh schedules send to every peer at
// once, one xGMI link each): entry j owns blocks [first[j], first[j+1]),
// grid-strides over its bytes and, through its own ticket counter, the
// workgroup finishing last publishes its flag.
struct CopyList {
  int n;
  unsigned first[kMaxCopies + 1];
  char* dst[kMaxCopies];
  const char* src[kMaxCopies];
  uint64_t bytes[kMaxCopies];
  uint64_t* flag[kMaxCopies];
  Seq seq[kMaxCopies];
  unsigned* ticket[kMaxCopies];
  int plainStore;  // stores of a flag-less copy (CopyStore, signal.h)
};

__global__ __launch_bounds__(kCopyBlock) void copy_signal_kernel(CopyList L, const uint64_t* epoch) {
  int j = 0;
  while (j + 1 < L.n && blockIdx.x >= L.first[j + 1]) j++;
  const unsigned lb = blockIdx.x - L.first[j], nb = L.first[j + 1] - L.first[j];
  char* dst = L.dst[j];
  const char* src = L.src[j];
  const size_t bytes = L.bytes[j];
  // dst head up to a 16-B boundary and the ragged tail: the entry's block 0, bytewise
  const size_t head = ((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15) < bytes
                          ? ((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15) : bytes;
  const size_t nvec = (bytes - head) / 16;
  const size_t tail0 = head + nvec * 16;
  if (lb == 0) {
    for (size_t i = threadIdx.x; i < head; i += kCopyBlock) dst[i] = src[i];
    for (size_t i = tail0 + threadIdx.x; i < bytes; i += kCopyBlock) dst[i] = src[i];
  }
  constexpr uint32_t kTileBytes = kCopyBlock * kCopyUnroll * 16;
  const size_t body = nvec * 16;
  const Src ss = src_of(src + head);
  for (size_t base = (size_t)lb * kTileBytes; base < body; base += (size_t)nb * kTileBytes) {
    const uint32_t n = (uint32_t)((body - base) < kTileBytes ? (body - base) : kTileBytes);
    const auto rs = make_rsrc(ss.base + base, n + ss.mis);
    const auto rd = make_rsrc(dst + head + base, n);
    const uint32_t lane_off = threadIdx.x * 16u;
    u32x4 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; u++) v[u] = bload<kAuxNT>(rs, lane_off + u * kCopyBlock * 16, ss.mis);
    if (L.flag[j] || L.plainStore == kCopyStoreWT) {
#pragma unroll
      for (int u = 0; u < kCopyUnroll; u++) bstore<kAuxWT>(rd, lane_off + u * kCopyBlock * 16, v[u]);
    } else if (L.plainStore == kCopyStorePlain) {
#pragma unroll
      for (int u = 0; u < kCopyUnroll; u++) bstore<0>(rd, lane_off + u * kCopyBlock * 16, v[u]);
    } else {
#pragma unroll
      for (int u = 0; u < kCopyUnroll; u++) bstore<kAuxNT>(rd, lane_off + u * kCopyBlock * 16, v[u]);
    }
  }
  if (!L.flag[j]) return;  // a plain (local) copy: nobody to tell
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    // the body went out write-through and every wave has waited for it;
    // only the entry's block 0, whose head / tail bytes are plain stores,
    // releases before its ticket
    if (lb == 0 && (head || tail0 < bytes)) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint64_t ep = epoch ? *epoch : 0;
    const unsigned t = __hip_atomic_fetch_add(L.ticket[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == nb - 1) {
      // last workgroup of this entry: reset the counter for the next launch
      // (launches on one channel's counter are stream-ordered), publish
      __hip_atomic_store(L.ticket[j], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(L.flag[j], L.seq[j].base + ep * L.seq[j].perRun, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------
// Host-side dispatch.
// ---------------------------------------------------------------------------
int g_variant = 0;  // fp32 SUM kernel variant (measurement knob)



int set_error(int code, const char* what) { return setError(code, what); }

int check_launch(const char* name) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return setError((int)e, std::string(name) + ": " + hipGetErrorString(e));
  return GLOO_HIP_OK;
}

constexpr int kUnroll = 2;      // 16-B packets per operand per lane
constexpr int kVecBlock = 512;  // lanes per workgroup on the vector body
constexpr int kMultiUnroll = 2;

inline size_t ceil_div(size_t a, size_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------
// Fold + forward (signal.h launchFoldSend): a FOLD whose finished range the
// plan then SENDs unchanged to up to kMaxCopyEntries peers (a mesh owner
// returning its range to every rank).  Each result tile is stored to dst AND
// to every forward destination in the same pass — the result is never read
// back, and the fold, the copies and their signal kernels become one launch.
// Completion as copy_signal_kernel: every wave drains, one lane releases at
// system scope and takes a ticket; the workgroup holding the launch's last
// ticket resets the counter and publishes every forward's flag.  The mode is
// a uniform runtime argument (0 left, 1 reverse, 2 tree) selecting the same
// fold_elem / fold_tile as reduce_multi_vec_kernel, so the bits are the same.
// ---------------------------------------------------------------------------
struct FwdList {
  int n;
  char* dst[kMaxCopyEntries];       // any element-aligned address; nullptr: a credit (flag only)
  uint64_t* flag[kMaxCopyEntries];  // nullptr: no arrival flag for this entry
  Seq seq[kMaxCopyEntries];
  unsigned* ticket;                 // zero between launches; nullptr: no signals
};

template <class Tr, int OP>
__global__ __launch_bounds__(kVecBlock) void fold_send_kernel(typename Tr::Storage* dst, SrcList srcs, int k,
                                                              int mode, size_t n, size_t head, FwdList F,
                                                              const uint64_t* epoch, uint64_t* stamp) {
  using S = typename Tr::Storage;
  constexpr int kV = 16 / sizeof(S);
  constexpr int UNROLL = kMultiUnroll, BLOCK = kVecBlock;
  constexpr uint32_t kTileBytes = (uint32_t)BLOCK * UNROLL * 16;
  stamp_begin(stamp);
  const size_t nvec = (n - head) / kV;
  const size_t tail0 = head + nvec * kV;
  if (blockIdx.x == 0) {
    const size_t t = threadIdx.x;
    for (int pass = 0; pass < 2; pass++) {
      const size_t i = pass == 0 ? t : tail0 + t;
      if ((pass == 0 && t < head) || (pass == 1 && i < n)) {
        const S acc = mode == 2   ? fold_elem<Tr, OP, 2>(srcs, k, i)
                      : mode == 1 ? fold_elem<Tr, OP, 1>(srcs, k, i)
                                  : fold_elem<Tr, OP, 0>(srcs, k, i);
        dst[i] = acc;
        for (int r = 0; r < F.n; r++)
          if (F.dst[r]) reinterpret_cast<S*>(F.dst[r])[i] = acc;
      }
    }
  }
  const size_t body = nvec * 16;
  const size_t base = (size_t)blockIdx.x * kTileBytes;
  if (base < body) {
    const uint32_t bytes = (uint32_t)((body - base) < kTileBytes ? (body - base) : kTileBytes);
    const uint32_t lane_off = threadIdx.x * 16u;
    u32x4 acc[UNROLL];
    if (mode == 2) fold_tile<Tr, OP, UNROLL, BLOCK, 2>(srcs, k, head, base, bytes, acc);
    else if (mode == 1) fold_tile<Tr, OP, UNROLL, BLOCK, 1>(srcs, k, head, base, bytes, acc);
    else fold_tile<Tr, OP, UNROLL, BLOCK, 0>(srcs, k, head, base, bytes, acc);
    const auto rd = make_rsrc(reinterpret_cast<const char*>(dst + head) + base, bytes);
    // plain local stores: the result stays in the Infinity Cache for its
    // next reader (`nt` measured slower per call)
#pragma unroll
    for (int u = 0; u < UNROLL; u++) bstore<0>(rd, lane_off + u * BLOCK * 16, acc[u]);
    for (int r = 0; r < F.n; r++) {
      if (!F.dst[r]) continue;  // a credit: no data
      // a forward destination may sit at another residue mod 16 B than dst
      // (ragged inbox regions): its misalignment rides in soffset, as a
      // relatively misaligned source's does
      const Src fr = src_of(F.dst[r] + head * sizeof(S));
      const auto rf = make_rsrc(fr.base + base, bytes + fr.mis);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) bstore<kAuxWT>(rf, lane_off + u * BLOCK * 16, acc[u], fr.mis);
    }
  }
  stamp_end(stamp);
  if (!F.ticket) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    // the forwarded bytes were stored write-through (sc0 sc1) and this
    // workgroup's waves have all seen them acknowledged, so no workgroup
    // writes its L2 back except block 0 for its plain edge stores, and the
    // ticket holder publishes with a relaxed store
    if (blockIdx.x == 0 && (head || tail0 < n)) {  // block 0's edge elements are plain stores
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint64_t ep = epoch ? *epoch : 0;
    const unsigned t = __hip_atomic_fetch_add(F.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(F.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      for (int r = 0; r < F.n; r++)
        if (F.flag[r])
          __hip_atomic_store(F.flag[r], F.seq[r].base + ep * F.seq[r].perRun, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <class Tr, int OP>
int launch_fold_send(void* dst, const SrcList& list, int k, int mode, size_t n, const FwdList& F,
                     const uint64_t* epoch, hipStream_t s) {
  using S = typename Tr::Storage;
  size_t head = ((16 - ((uintptr_t)dst & 15)) & 15) / sizeof(S);
  if (head > n) head = n;
  constexpr int kV = 16 / sizeof(S);
  const size_t nvec = (n - head) / kV;
  size_t grid = ceil_div(nvec, (size_t)kVecBlock * kMultiUnroll);
  if (grid == 0) grid = 1;
  fold_send_kernel<Tr, OP><<<dim3((unsigned)grid), dim3(kVecBlock), 0, s>>>(static_cast<S*>(dst), list, k, mode, n,
                                                                          head, F, epoch, t_stamp);
  return check_launch("fold_send_kernel");
}

template <class Tr>
int by_op_fold_send(int op, void* dst, const SrcList& list, int k, int mode, size_t n, const FwdList& F,
                    const uint64_t* epoch, hipStream_t s) {
  switch (op) {
    case GLOO_HIP_SUM: return launch_fold_send<Tr, GLOO_HIP_SUM>(dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_PRODUCT: return launch_fold_send<Tr, GLOO_HIP_PRODUCT>(dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_MAX: return launch_fold_send<Tr, GLOO_HIP_MAX>(dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_MIN: return launch_fold_send<Tr, GLOO_HIP_MIN>(dst, list, k, mode, n, F, epoch, s);
    default: return set_error(GLOO_HIP_EINVAL_OP, "fold+forward needs a built-in op");
  }
}

// lds: a dynamic LDS allocation the kernel never touches; it only caps the
// workgroups a CU holds (160 KiB / lds), a measurement knob (variants 16, 17).
template <class Tr, int OP, int UNROLL, int BLOCK, int LAUX, int SAUX, int IL = 0>
int launch_vec(void* c, const void* a, const void* b, size_t n, size_t head, hipStream_t s, unsigned lds = 0) {
  using S = typename Tr::Storage;
  constexpr int kV = 16 / sizeof(S);
  const size_t nvec = (n - head) / kV;
  size_t grid = ceil_div(nvec, (size_t)BLOCK * UNROLL);
  if (grid == 0) grid = 1;
  reduce_vec_kernel<Tr, OP, UNROLL, BLOCK, LAUX, SAUX, IL><<<dim3((unsigned)grid), dim3(BLOCK), lds, s>>>(
      static_cast<S*>(c), static_cast<const S*>(a), static_cast<const S*>(b), n, head, t_stamp);
  return check_launch("reduce_vec_kernel");
}

template <class Tr, int OP, int UNROLL, int BLOCK, int LAUX, int SAUX>
int launch_vec_pipe(void* c, const void* a, const void* b, size_t n, size_t head, size_t maxGrid, hipStream_t s) {
  using S = typename Tr::Storage;
  constexpr int kV = 16 / sizeof(S);
  const size_t nvec = (n - head) / kV;
  size_t grid = ceil_div(nvec, (size_t)BLOCK * UNROLL);
  if (grid > maxGrid) grid = maxGrid;
  if (grid == 0) grid = 1;
  reduce_vec_pipe_kernel<Tr, OP, UNROLL, BLOCK, LAUX, SAUX><<<dim3((unsigned)grid), dim3(BLOCK), 0, s>>>(
      static_cast<S*>(c), static_cast<const S*>(a), static_cast<const S*>(b), n, head);
  return check_launch("reduce_vec_pipe_kernel");
}

template <class Tr, int OP>
int launch3(void* c, const void* a, const void* b, size_t n, hipStream_t s) {
  using S = typename Tr::Storage;
  constexpr size_t kV = 16 / sizeof(S);
  if (n == 0) return GLOO_HIP_OK;
  const uintptr_t pc = (uintptr_t)c, pa = (uintptr_t)a, pb = (uintptr_t)b;
  if ((pc % sizeof(S)) || (pa % sizeof(S)) || (pb % sizeof(S)))
    return set_error(GLOO_HIP_EINVAL_PTR, "pointer not aligned to the element size");
  size_t head = ((16 - (pc & 15)) & 15) / sizeof(S);
  if (head > n) head = n;
  (void)kV;
  if constexpr (std::is_same<Tr, TrF32>::value && OP == GLOO_HIP_SUM) {
    // A/B knob for the measurement harness (tools/sweep_variants.py).
    switch (g_variant) {
      case 1: return launch_vec<Tr, OP, 2, 256, kAuxNT, kAuxNT>(c, a, b, n, head, s);
      case 2: return launch_vec<Tr, OP, 4, 256, kAuxNT, kAuxNT>(c, a, b, n, head, s);
      case 3: return launch_vec<Tr, OP, 1, 512, kAuxNT, kAuxNT>(c, a, b, n, head, s);
      case 4: return launch_vec<Tr, OP, 2, 512, kAuxNT, 0>(c, a, b, n, head, s);
      case 5: return launch_vec<Tr, OP, 2, 1024, kAuxNT, kAuxNT>(c, a, b, n, head, s);
      case 9: return launch_vec_pipe<Tr, OP, 2, 512, kAuxNT, kAuxNT>(c, a, b, n, head, 256, s);
      case 10: return launch_vec_pipe<Tr, OP, 2, 512, kAuxNT, kAuxNT>(c, a, b, n, head, 512, s);
      case 11: return launch_vec_pipe<Tr, OP, 2, 512, kAuxNT, kAuxNT>(c, a, b, n, head, 1024, s);
      case 12: return launch_vec_pipe<Tr, OP, 2, 512, kAuxNT, kAuxNT>(c, a, b, n, head, 2048, s);
      case 13: return launch_vec_pipe<Tr, OP, 1, 512, kAuxNT, kAuxNT>(c, a, b, n, head, 1024, s);
      case 14: return launch_vec_pipe<Tr, OP, 2, 256, kAuxNT, kAuxNT>(c, a, b, n, head, 2048, s);
      case 15: return launch_vec<Tr, OP, 2, 512, kAuxNT, kAuxNT, 1>(c, a, b, n, head, s);  // round 3-5 load order (IL)
      // round 6: three workgroups per CU instead of four (48 KiB of unused LDS
      // each): 64 MiB +0.1-0.2 %, 16 MiB -1.3-2 % (profiles/round6/r6ae/)
      case 16: return launch_vec<Tr, OP, 2, 512, kAuxNT, kAuxNT, 1>(c, a, b, n, head, s, 48u << 10);
      case 17: return launch_vec<Tr, OP, 2, 512, kAuxNT, kAuxNT, 0>(c, a, b, n, head, s, 48u << 10);
      default: break;
    }
  }
  if (t_plainStores) return launch_vec<Tr, OP, kUnroll, kVecBlock, kAuxNT, 0>(c, a, b, n, head, s);
  return launch_vec<Tr, OP, kUnroll, kVecBlock, kAuxNT, kAuxNT>(c, a, b, n, head, s);
}

template <class Tr, int OP, int MODE = 0>
int launch_multi(void* dst, const void* const* srcs, int k, size_t n, hipStream_t s) {
  using S = typename Tr::Storage;
  if (n == 0) return GLOO_HIP_OK;
  SrcList list;
  memset(&list, 0, sizeof(list));
  const uintptr_t pd = (uintptr_t)dst;
  if (pd % sizeof(S)) return set_error(GLOO_HIP_EINVAL_PTR, "dst not aligned to the element size");
  for (int j = 0; j < k; j++) {
    if (srcs[j] == nullptr) return set_error(GLOO_HIP_EINVAL_PTR, "null source pointer");
    const uintptr_t p = (uintptr_t)srcs[j];
    if (p % sizeof(S)) return set_error(GLOO_HIP_EINVAL_PTR, "source not aligned to the element size");
    list.p[j] = srcs[j];
  }
  size_t head = ((16 - (pd & 15)) & 15) / sizeof(S);
  if (head > n) head = n;
  constexpr int kV = 16 / sizeof(S);
  const size_t nvec = (n - head) / kV;
  size_t grid = ceil_div(nvec, (size_t)kVecBlock * kMultiUnroll);
  if (grid == 0) grid = 1;
  reduce_multi_vec_kernel<Tr, OP, kMultiUnroll, kVecBlock, MODE><<<dim3((unsigned)grid), dim3(kVecBlock), 0, s>>>(
      static_cast<S*>(dst), list, k, n, head, t_stamp, t_plainStores ? 1 : 0);
  return check_launch("reduce_multi_vec_kernel");
}

template <class Tr>
int by_op3(int op, void* c, const void* a, const void* b, size_t n, hipStream_t s) {
  switch (op) {
    case GLOO_HIP_SUM: return launch3<Tr, GLOO_HIP_SUM>(c, a, b, n, s);
    case GLOO_HIP_PRODUCT: return launch3<Tr, GLOO_HIP_PRODUCT>(c, a, b, n, s);
    case GLOO_HIP_MAX: return launch3<Tr, GLOO_HIP_MAX>(c, a, b, n, s);
    case GLOO_HIP_MIN: return launch3<Tr, GLOO_HIP_MIN>(c, a, b, n, s);
    default: return set_error(GLOO_HIP_EINVAL_OP, "unknown reduction op");
  }
}

template <class Tr, int MODE = 0>
int by_op_multi(int op, void* d, const void* const* srcs, int k, size_t n, hipStream_t s) {
  switch (op) {
    case GLOO_HIP_SUM: return launch_multi<Tr, GLOO_HIP_SUM, MODE>(d, srcs, k, n, s);
    case GLOO_HIP_PRODUCT: return launch_multi<Tr, GLOO_HIP_PRODUCT, MODE>(d, srcs, k, n, s);
    case GLOO_HIP_MAX: return launch_multi<Tr, GLOO_HIP_MAX, MODE>(d, srcs, k, n, s);
    case GLOO_HIP_MIN: return launch_multi<Tr, GLOO_HIP_MIN, MODE>(d, srcs, k, n, s);
    default: return set_error(GLOO_HIP_EINVAL_OP, "unknown reduction op");
  }
}

int dispatch3(int op, int dtype, void* c, const void* a, const void* b, size_t n,
              hipStream_t s) {
  switch (dtype) {
    case GLOO_HIP_I8: return by_op3<TrI8>(op, c, a, b, n, s);
    case GLOO_HIP_U8: return by_op3<TrU8>(op, c, a, b, n, s);
    case GLOO_HIP_I32: return by_op3<TrI32>(op, c, a, b, n, s);
    case GLOO_HIP_U32: return by_op3<TrU32>(op, c, a, b, n, s);
    case GLOO_HIP_I64: return by_op3<TrI64>(op, c, a, b, n, s);
    case GLOO_HIP_U64: return by_op3<TrU64>(op, c, a, b, n, s);
    case GLOO_HIP_F16: return by_op3<TrF16>(op, c, a, b, n, s);
    case GLOO_HIP_BF16: return by_op3<TrBF16>(op, c, a, b, n, s);
    case GLOO_HIP_F32: return by_op3<TrF32>(op, c, a, b, n, s);
    case GLOO_HIP_F64: return by_op3<TrF64>(op, c, a, b, n, s);
    default: return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
  }
}

template <int MODE = 0>
int dispatch_multi(int op, int dtype, void* d, const void* const* srcs, int k, size_t n,
                   hipStream_t s) {
  switch (dtype) {
    case GLOO_HIP_I8: return by_op_multi<TrI8, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_U8: return by_op_multi<TrU8, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_I32: return by_op_multi<TrI32, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_U32: return by_op_multi<TrU32, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_I64: return by_op_multi<TrI64, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_U64: return by_op_multi<TrU64, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_F16: return by_op_multi<TrF16, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_BF16: return by_op_multi<TrBF16, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_F32: return by_op_multi<TrF32, MODE>(op, d, srcs, k, n, s);
    case GLOO_HIP_F64: return by_op_multi<TrF64, MODE>(op, d, srcs, k, n, s);
    default: return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
  }
}

}  // namespace

unsigned copySignalGrid(size_t bytes, unsigned maxBlocks) {
  const size_t tiles = (bytes + (size_t)kCopyBlock * kCopyUnroll * 16 - 1) / ((size_t)kCopyBlock * kCopyUnroll * 16);
  size_t g = tiles < maxBlocks ? tiles : maxBlocks;
  return (unsigned)(g == 0 ? 1 : g);
}

int launchCopySignalMulti(const CopyDesc* d, int n, const uint64_t* epoch, hipStream_t s, CopyStore localStore) {
  if (n < 1 || n > kMaxCopies) return set_error(GLOO_HIP_EINVAL_ARG, "copy list size out of range");
  CopyList L;
  memset(&L, 0, sizeof(L));
  L.n = n;
  unsigned total = 0;
  for (int j = 0; j < n; j++) {
    if ((d[j].flag && !d[j].ticket) || d[j].blocks == 0) return set_error(GLOO_HIP_EINVAL_ARG, "bad copy entry");
    L.first[j] = total;
    total += d[j].blocks;
    L.dst[j] = static_cast<char*>(d[j].dst);
    L.src[j] = static_cast<const char*>(d[j].src);
    L.bytes[j] = d[j].bytes;
    L.flag[j] = d[j].flag;
    L.seq[j] = d[j].seq;
    L.ticket[j] = d[j].ticket;
  }
  L.first[n] = total;
  L.plainStore = localStore;
  copy_signal_kernel<<<total, kCopyBlock, 0, s>>>(L, epoch);
  return check_launch("copy_signal_kernel");
}

int launchCopySignal(void* dst, const void* src, size_t bytes, uint64_t* flag, Seq seq, unsigned* ticket,
                     const uint64_t* epoch, unsigned grid, hipStream_t s) {
  CopyDesc d{dst, src, bytes, flag, seq, ticket, grid};
  return launchCopySignalMulti(&d, 1, epoch, s);
}

struct CustomEntry {
  gloo_hip_custom_fn fn;
  void* user;
};
std::mutex& customMutex() {
  static std::mutex m;
  return m;
}
std::vector<CustomEntry>& customOps() {
  static std::vector<CustomEntry> v;
  return v;
}

bool isBuiltinOp(int op) { return op >= GLOO_HIP_SUM && op <= GLOO_HIP_MIN; }

bool customOp(int op, gloo_hip_custom_fn* fn, void** user) {
  if (op < GLOO_HIP_CUSTOM) return false;
  std::lock_guard<std::mutex> lk(customMutex());
  const size_t i = (size_t)(op - GLOO_HIP_CUSTOM);
  if (i >= customOps().size()) return false;
  *fn = customOps()[i].fn;
  *user = customOps()[i].user;
  return true;
}

// A k-source fold with a custom op: k - 1 calls of the 3-operand function,
// left to right (the association of the reference's sequential calls).  The
// destination may alias the first source only.
int customFold(gloo_hip_custom_fn fn, void* user, int dtype, void* dst, const void* const* srcs, int k, size_t n,
               int mode, hipStream_t s) {
  if (mode != 0) return set_error(GLOO_HIP_EINVAL_ARG, "custom ops fold left to right only");
  const size_t bytes = n * gloo_hip_dtype_size(dtype);
  for (int j = 1; j < k; j++) {
    const char* p = static_cast<const char*>(srcs[j]);
    const char* d = static_cast<const char*>(dst);
    if (d < p + bytes && p < d + bytes) return set_error(GLOO_HIP_EINVAL_ARG, "custom fold: dst overlaps a source");
  }
  if (k == 1) {
    if (dst != srcs[0]) {
      hipError_t e = hipMemcpyAsync(dst, srcs[0], bytes, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return set_error((int)e, hipGetErrorString(e));
    }
    return GLOO_HIP_OK;
  }
  fn(user, dst, srcs[0], srcs[1], n, s);
  for (int j = 2; j < k; j++) fn(user, dst, dst, srcs[j], n, s);
  return check_launch("custom reduction");
}

int launchFold(int op, int dtype, void* dst, const void* const* srcs, int k, size_t n, int mode,
               hipStream_t s) {
  if (k < 1 || k > GLOO_HIP_MAX_SRCS) return set_error(GLOO_HIP_EINVAL_ARG, "source count out of range");
  gloo_hip_custom_fn cfn;
  void* cuser;
  if (customOp(op, &cfn, &cuser)) {
    if (n == 0) return GLOO_HIP_OK;
    return customFold(cfn, cuser, dtype, dst, srcs, k, n, mode, s);
  }
  if (mode == 2 && (k & (k - 1))) return set_error(GLOO_HIP_EINVAL_ARG, "tree fold needs a power-of-two count");
  if (n == 0) return GLOO_HIP_OK;
  switch (mode) {
    case 0: return dispatch_multi<0>(op, dtype, dst, srcs, k, n, s);
    case 1: return dispatch_multi<1>(op, dtype, dst, srcs, k, n, s);
    case 2: return dispatch_multi<2>(op, dtype, dst, srcs, k, n, s);
    default: return set_error(GLOO_HIP_EINVAL_ARG, "unknown fold mode");
  }
}

int launchFoldSend(int op, int dtype, void* dst, const void* const* srcs, int k, size_t n, int mode,
                   const FwdDesc* fwd, int nf, unsigned* ticket, const uint64_t* epoch, hipStream_t s) {
  if (k < 1 || k > GLOO_HIP_MAX_SRCS) return set_error(GLOO_HIP_EINVAL_ARG, "source count out of range");
  if (nf < 1 || nf > kMaxCopyEntries) return set_error(GLOO_HIP_EINVAL_ARG, "forward count out of range");
  if (mode < 0 || mode > 2 || (mode == 2 && (k & (k - 1))))
    return set_error(GLOO_HIP_EINVAL_ARG, "bad fold mode for fold+forward");
  const size_t es = gloo_hip_dtype_size(dtype);
  if (es == 0) return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
  if (!dst || (uintptr_t)dst % es) return set_error(GLOO_HIP_EINVAL_PTR, "dst not aligned to the element size");
  SrcList list;
  memset(&list, 0, sizeof(list));
  for (int j = 0; j < k; j++) {
    if (!srcs[j] || (uintptr_t)srcs[j] % es) return set_error(GLOO_HIP_EINVAL_PTR, "bad source pointer");
    list.p[j] = srcs[j];
  }
  FwdList F;
  memset(&F, 0, sizeof(F));
  F.n = nf;
  F.ticket = ticket;
  // (the local result is stored plain: the range stays in the Infinity Cache
  // for its next reader — the copy-out's peers, the caller, the next call —
  // 1-5 % faster per HD / ring call than `nt` from 16 to 64 MiB per rank,
  // equal at 256 MiB: DESIGN.md §4, profiles/round5/r5p_*)
  for (int r = 0; r < nf; r++) {
    if (!fwd[r].dst && !fwd[r].flag) return set_error(GLOO_HIP_EINVAL_ARG, "forward entry with neither data nor flag");
    if ((uintptr_t)fwd[r].dst % es)
      return set_error(GLOO_HIP_EINVAL_PTR, "forward destination not aligned to the element size");
    if (fwd[r].flag && !ticket) return set_error(GLOO_HIP_EINVAL_ARG, "forward flag without a ticket counter");
    F.dst[r] = static_cast<char*>(fwd[r].dst);
    F.flag[r] = fwd[r].flag;
    F.seq[r] = fwd[r].seq;
  }
  switch (dtype) {
    case GLOO_HIP_I8: return by_op_fold_send<TrI8>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_U8: return by_op_fold_send<TrU8>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_I32: return by_op_fold_send<TrI32>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_U32: return by_op_fold_send<TrU32>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_I64: return by_op_fold_send<TrI64>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_U64: return by_op_fold_send<TrU64>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_F16: return by_op_fold_send<TrF16>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_BF16: return by_op_fold_send<TrBF16>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_F32: return by_op_fold_send<TrF32>(op, dst, list, k, mode, n, F, epoch, s);
    case GLOO_HIP_F64: return by_op_fold_send<TrF64>(op, dst, list, k, mode, n, F, epoch, s);
    default: return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
  }
}

bool setReducePlainStores(bool plain) {
  const bool prev = t_plainStores;
  t_plainStores = plain;
  return prev;
}

uint64_t* setLaunchStamp(uint64_t* stamp) {
  uint64_t* prev = t_stamp;
  t_stamp = stamp;
  return prev;
}

int launchStampInit(uint64_t* stamps, int k, hipStream_t s) {
  if (k <= 0) return GLOO_HIP_OK;
  const size_t words = (size_t)k * kStampSlotWords;
  stamp_init_kernel<<<(unsigned)((words + 255) / 256), 256, 0, s>>>(stamps, words);
  return check_launch("stamp_init_kernel");
}

// Internal entry for the plan executor (see gloo_amd/signal.h).
int launchFusedSmall(int op, int dtype, void* dst, const void* src, size_t n, const uint64_t* waitFlag,
                     Seq waitTarget, uint64_t timeoutTicks, uint32_t* err, uint64_t* sigFlag, Seq sigValue,
                     const uint64_t* epoch, hipStream_t s) {
  int rc;
  switch (dtype) {
    case GLOO_HIP_I8: rc = launch_fused<TrI8>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_U8: rc = launch_fused<TrU8>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_I32: rc = launch_fused<TrI32>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_U32: rc = launch_fused<TrU32>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_I64: rc = launch_fused<TrI64>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_U64: rc = launch_fused<TrU64>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_F16: rc = launch_fused<TrF16>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_BF16: rc = launch_fused<TrBF16>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_F32: rc = launch_fused<TrF32>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    case GLOO_HIP_F64: rc = launch_fused<TrF64>(op, dst, src, n, waitFlag, waitTarget, timeoutTicks, err, sigFlag, sigValue, epoch, s); break;
    default: return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
  }
  if (rc != GLOO_HIP_OK) return set_error(rc, "fused step: bad op");
  return check_launch("fused_small_kernel");
}

int launchPlanInterp(int op, int dtype, const InterpStep* steps, int nsteps, uint64_t run, uint64_t tt,
                     uint32_t* err, int G, hipStream_t s, uint64_t* done, unsigned* doneTicket) {
  if ((done == nullptr) != (doneTicket == nullptr)) return set_error(GLOO_HIP_EINVAL_ARG, "interpreter: half a done signal");
  static_assert(GLOO_HIP_MAX_SRCS <= 8, "InterpStep holds 8 sources");
  if (nsteps < 0 || nsteps > kInterpMaxSteps) return set_error(GLOO_HIP_EINVAL_ARG, "interpreter: bad step count");
  if (G < 1 || G > kMaxSlices) return set_error(GLOO_HIP_EINVAL_ARG, "interpreter: bad slice count");
  int rc;
  switch (dtype) {
    case GLOO_HIP_I8: rc = launch_interp<TrI8>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_U8: rc = launch_interp<TrU8>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_I32: rc = launch_interp<TrI32>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_U32: rc = launch_interp<TrU32>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_I64: rc = launch_interp<TrI64>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_U64: rc = launch_interp<TrU64>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_F16: rc = launch_interp<TrF16>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_BF16: rc = launch_interp<TrBF16>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_F32: rc = launch_interp<TrF32>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    case GLOO_HIP_F64: rc = launch_interp<TrF64>(op, steps, nsteps, run, tt, err, G, s, done, doneTicket); break;
    default: return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
  }
  if (rc != GLOO_HIP_OK) return set_error(rc, "interpreter: bad op");
  return check_launch("plan_interp_kernel");
}

}  // namespace gloo_amd

using namespace gloo_amd;

extern "C" {

int gloo_hip_reduce3(int op, int dtype, void* c, const void* a, const void* b, size_t n,
                     gloo_hip_stream_t stream) {
  gloo_hip_custom_fn cfn = nullptr;
  void* cuser = nullptr;
  const bool custom = customOp(op, &cfn, &cuser);
  if (n == 0) {
    if (!custom && (op < GLOO_HIP_SUM || op > GLOO_HIP_MIN)) return set_error(GLOO_HIP_EINVAL_OP, "unknown reduction op");
    if (dtype < 0 || dtype >= GLOO_HIP_NUM_DTYPES) return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
    return GLOO_HIP_OK;
  }
  if (!c || !a || !b) return set_error(GLOO_HIP_EINVAL_PTR, "null buffer pointer");
  if (custom) {
    if (dtype < 0 || dtype >= GLOO_HIP_NUM_DTYPES) return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
    cfn(cuser, c, a, b, n, stream);
    return check_launch("custom reduction");
  }
  return dispatch3(op, dtype, c, a, b, n, static_cast<hipStream_t>(stream));
}

int gloo_hip_copy_kernel(void* dst, const void* src, size_t bytes, unsigned blocks, gloo_hip_stream_t stream) {
  if (bytes == 0) return GLOO_HIP_OK;
  if (!dst || !src) return set_error(GLOO_HIP_EINVAL_PTR, "null buffer pointer");
  CopyDesc d{dst, src, bytes, nullptr, Seq{}, nullptr, copySignalGrid(bytes, blocks ? blocks : 1024u)};
  return launchCopySignalMulti(&d, 1, nullptr, static_cast<hipStream_t>(stream));
}

int gloo_hip_copy_kernel_multi(void* const* dsts, const void* const* srcs, const size_t* bytes, int n, unsigned blocks,
                               gloo_hip_stream_t stream) {
  if (n < 1 || n > kMaxCopies) return set_error(GLOO_HIP_EINVAL_ARG, "copy list size out of range");
  if (!dsts || !srcs || !bytes) return set_error(GLOO_HIP_EINVAL_PTR, "null argument");
  CopyDesc d[kMaxCopies];
  int m = 0;
  for (int j = 0; j < n; j++) {
    if (bytes[j] == 0) continue;
    if (!dsts[j] || !srcs[j]) return set_error(GLOO_HIP_EINVAL_PTR, "null buffer pointer");
    d[m++] = CopyDesc{dsts[j], srcs[j], bytes[j], nullptr, Seq{}, nullptr, copySignalGrid(bytes[j], blocks ? blocks : 64u)};
  }
  if (m == 0) return GLOO_HIP_OK;
  return launchCopySignalMulti(d, m, nullptr, static_cast<hipStream_t>(stream));
}

int gloo_hip_register_op(gloo_hip_custom_fn fn, void* user, int* op_out) {
  if (!fn || !op_out) return set_error(GLOO_HIP_EINVAL_ARG, "null argument");
  std::lock_guard<std::mutex> lk(customMutex());
  customOps().push_back(CustomEntry{fn, user});
  *op_out = GLOO_HIP_CUSTOM + (int)customOps().size() - 1;
  return GLOO_HIP_OK;
}

int gloo_hip_reduce(int op, int dtype, void* dst, const void* src, size_t n,
                    gloo_hip_stream_t stream) {
  return gloo_hip_reduce3(op, dtype, dst, dst, src, n, stream);
}

int gloo_hip_reduce_multi(int op, int dtype, void* dst, const void* const* srcs, int k,
                          size_t n, gloo_hip_stream_t stream) {
  if (k < 1 || k > GLOO_HIP_MAX_SRCS) return set_error(GLOO_HIP_EINVAL_ARG, "source count out of range");
  gloo_hip_custom_fn cfn = nullptr;
  void* cuser = nullptr;
  const bool custom = customOp(op, &cfn, &cuser);
  if (!custom && (op < GLOO_HIP_SUM || op > GLOO_HIP_MIN)) return set_error(GLOO_HIP_EINVAL_OP, "unknown reduction op");
  if (dtype < 0 || dtype >= GLOO_HIP_NUM_DTYPES) return set_error(GLOO_HIP_EINVAL_DTYPE, "unknown dtype");
  if (n == 0) return GLOO_HIP_OK;
  if (!dst || !srcs) return set_error(GLOO_HIP_EINVAL_PTR, "null buffer pointer");
  if (custom) return customFold(cfn, cuser, dtype, dst, srcs, k, n, 0, static_cast<hipStream_t>(stream));
  return dispatch_multi(op, dtype, dst, srcs, k, n, static_cast<hipStream_t>(stream));
}

size_t gloo_hip_dtype_size(int dtype) {
  static const size_t kSizes[GLOO_HIP_NUM_DTYPES] = {1, 1, 4, 4, 8, 8, 2, 2, 4, 8};
  if (dtype < 0 || dtype >= GLOO_HIP_NUM_DTYPES) return 0;
  return kSizes[dtype];
}



int gloo_hip_set_variant(int variant) {
  const int prev = g_variant;
  g_variant = variant;
  return prev;
}

}  // extern "C"

// hbm_ceiling.hip — MEASUREMENT ONLY (not the product): streaming kernels
// with the access shape of reduce_vec_kernel (raw buffer loads/stores of
// 16 B per lane, `nt`, BLOCK lanes x U packets per stream per workgroup, one
// tile per workgroup) and R read streams / W write streams, so the config-2
// kernel (2 reads + 1 write in place) can be set against the best rate this
// chip sustains for the same mix and for its neighbours:
//   R1W0 read, R0W1 write, R1W1 copy, R2W0, R2W1 (c distinct), R2W1 in place.
// Read-only kernels keep their loads live with a data-dependent vector store
// that never fires.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kNT = 2;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

template <int R, int W, int U, int B>
__global__ __launch_bounds__(B) void stream_k(float* c, const float* a, const float* b, uint32_t* sink) {
  constexpr uint32_t kTile = (uint32_t)B * U * 16;
  const size_t base = (size_t)blockIdx.x * kTile;
  const auto ra = rsrc(reinterpret_cast<const char*>(a) + base, kTile);
  const auto rb = rsrc(reinterpret_cast<const char*>(b) + base, kTile);
  const auto rc = rsrc(reinterpret_cast<const char*>(c) + base, kTile);
  const uint32_t lane = threadIdx.x * 16u;
  u32x4 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; u++) x[u] = R >= 1 ? __builtin_amdgcn_raw_buffer_load_b128(ra, lane + u * B * 16, 0, kNT)
                                            : u32x4{blockIdx.x, threadIdx.x, (uint32_t)u, 0u};
#pragma unroll
  for (int u = 0; u < U; u++) y[u] = R >= 2 ? __builtin_amdgcn_raw_buffer_load_b128(rb, lane + u * B * 16, 0, kNT)
                                            : u32x4{0u, 0u, 0u, 0u};
  if (W) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const f32x4 s = __builtin_bit_cast(f32x4, x[u]) + __builtin_bit_cast(f32x4, y[u]);
      __builtin_amdgcn_raw_buffer_store_b128(R == 2 ? __builtin_bit_cast(u32x4, s) : x[u], rc, lane + u * B * 16, 0,
                                             kNT);
    }
  } else {
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; u++) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w ^ y[u].x ^ y[u].y ^ y[u].z ^ y[u].w;
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // never in practice; keeps the loads
  }
}

// The same 2-read + 1-write mix with both reads by LDS-DMA (`buffer_load
// ... lds`, 16 B per lane on gfx950, nt): each wave's packets land in LDS at
// M0 + lane * 16, are read back with ds_read_b128 after vmcnt(0), added and
// stored with raw nt buffer stores.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
template <int U, int B>
__global__ __launch_bounds__(B) void stream_lds_k(float* c, const float* a, const float* b, uint32_t*) {
  __shared__ u32x4 lds[2][U][B];
  constexpr uint32_t kTile = (uint32_t)B * U * 16;
  const size_t base = (size_t)blockIdx.x * kTile;
  const auto ra = rsrc(reinterpret_cast<const char*>(a) + base, kTile);
  const auto rb = rsrc(reinterpret_cast<const char*>(b) + base, kTile);
  const auto rc = rsrc(reinterpret_cast<const char*>(c) + base, kTile);
  const uint32_t lane = threadIdx.x * 16u;
  const int w0 = (threadIdx.x / 64) * 64;
#pragma unroll
  for (int u = 0; u < U; u++)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)&lds[0][u][w0], 16, lane + u * B * 16, 0, 0, kNT);
#pragma unroll
  for (int u = 0; u < U; u++)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)&lds[1][u][w0], 16, lane + u * B * 16, 0, 0, kNT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < U; u++) {
    const f32x4 s = __builtin_bit_cast(f32x4, lds[0][u][threadIdx.x]) + __builtin_bit_cast(f32x4, lds[1][u][threadIdx.x]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, s), rc, lane + u * B * 16, 0, kNT);
  }
}

// 2-read + 1-write with explicit cache policies for the loads (LP) and the
// store (SP), and optionally the two read streams interleaved packet by packet
// (IL): round-3 variants of the config-2 mix (policy bits on gfx950: sc0 = 1,
// nt = 2, sc1 = 16).
template <int U, int B, int LP, int SP, int IL>
__global__ __launch_bounds__(B) void stream_pol_k(float* c, const float* a, const float* b, uint32_t*) {
  constexpr uint32_t kTile = (uint32_t)B * U * 16;
  const size_t base = (size_t)blockIdx.x * kTile;
  const auto ra = rsrc(reinterpret_cast<const char*>(a) + base, kTile);
  const auto rb = rsrc(reinterpret_cast<const char*>(b) + base, kTile);
  const auto rc = rsrc(reinterpret_cast<const char*>(c) + base, kTile);
  const uint32_t lane = threadIdx.x * 16u;
  u32x4 x[U], y[U];
  if (IL) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, lane + u * B * 16, 0, LP);
      y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, lane + u * B * 16, 0, LP);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, lane + u * B * 16, 0, LP);
#pragma unroll
    for (int u = 0; u < U; u++) y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, lane + u * B * 16, 0, LP);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const f32x4 s = __builtin_bit_cast(f32x4, x[u]) + __builtin_bit_cast(f32x4, y[u]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, s), rc, lane + u * B * 16, 0, SP);
  }
}

// Round 6, the product's shape (u2 x 512 lanes, nt loads interleaved, nt
// stores) with three levers not measured before: MODE 0 with a dynamic LDS
// allocation the kernel never touches, which only caps the workgroups a CU
// holds (160 KiB / LDS); MODE 1 tiles dealt XCD-contiguously (workgroup i
// runs on XCD i % 8, so XCD x streams one contiguous eighth of the buffer);
// MODE 2 each wave's two packets per stream adjacent (2 KiB contiguous per
// wave and stream instead of 2 x 1 KiB, 8 KiB apart).
template <int MODE>
__global__ __launch_bounds__(512) void stream_x_k(float* c, const float* a, const float* b, uint32_t*) {
  constexpr int U = 2, B = 512;
  constexpr uint32_t kTile = (uint32_t)B * U * 16;
  uint32_t tile = blockIdx.x;
  if (MODE == 1) tile = (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u;
  const size_t base = (size_t)tile * kTile;
  const auto ra = rsrc(reinterpret_cast<const char*>(a) + base, kTile);
  const auto rb = rsrc(reinterpret_cast<const char*>(b) + base, kTile);
  const auto rc = rsrc(reinterpret_cast<const char*>(c) + base, kTile);
  uint32_t off[U];
#pragma unroll
  for (int u = 0; u < U; u++)
    off[u] = MODE == 2 ? ((threadIdx.x / 64u) * (64u * U) + u * 64u + threadIdx.x % 64u) * 16u
                       : threadIdx.x * 16u + u * B * 16u;
  u32x4 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, off[u], 0, kNT);
    y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, off[u], 0, kNT);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const f32x4 s = __builtin_bit_cast(f32x4, x[u]) + __builtin_bit_cast(f32x4, y[u]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, s), rc, off[u], 0, kNT);
  }
}

struct P {
  int r, w, u, b;
  void (*launch)(float*, const float*, const float*, uint32_t*, size_t, hipStream_t);
};

#define X(R, W, U, B)                                                                                      \
  {R, W, U, B, [](float* c, const float* a, const float* b, uint32_t* sink, size_t bytes, hipStream_t s) { \
     stream_k<R, W, U, B><<<(unsigned)(bytes / ((size_t)B * U * 16)), B, 0, s>>>(c, a, b, sink);           \
   }},
#define XL(U, B)                                                                                        \
  {2, 1 + 10 * U, U, B, [](float* c, const float* a, const float* b, uint32_t* sink, size_t bytes, hipStream_t s) { \
     stream_lds_k<U, B><<<(unsigned)(bytes / ((size_t)B * U * 16)), B, 0, s>>>(c, a, b, sink);          \
   }},
#define XX(MODE, LDSKIB)                                                                                \
  {2, 1 + 1000000 * (1 + MODE) + 1000 * LDSKIB, 2, 512,                                                \
   [](float* c, const float* a, const float* b, uint32_t* sink, size_t bytes, hipStream_t s) {          \
     stream_x_k<MODE><<<(unsigned)(bytes / (512 * 2 * 16)), 512, LDSKIB * 1024, s>>>(c, a, b, sink);    \
   }},
#define XP(U, B, LP, SP, IL)                                                                            \
  {2, 1 + 100 * (1 + LP + 32 * SP + 1024 * IL), U, B,                                                   \
   [](float* c, const float* a, const float* b, uint32_t* sink, size_t bytes, hipStream_t s) {          \
     stream_pol_k<U, B, LP, SP, IL><<<(unsigned)(bytes / ((size_t)B * U * 16)), B, 0, s>>>(c, a, b, sink); \
   }},
// pattern 8 (R2W1 u2 b512) is the product kernel's shape: bench.py times it
// beside the product in the same run; 10-12 read through LDS-DMA (w = 1 + 10 u)
static const P kP[] = {X(1, 0, 2, 512) X(1, 0, 4, 512) X(0, 1, 2, 512) X(0, 1, 4, 512) X(1, 1, 2, 512)
                           X(1, 1, 4, 512) X(2, 0, 2, 512) X(2, 0, 4, 512) X(2, 1, 2, 512) X(2, 1, 4, 256)
                               XL(1, 512) XL(2, 512) XL(2, 256)
                                   // 13..: cache policies, interleaved reads, wider tiles (w = 1 + 100 * code)
                                   XP(2, 512, 2, 2, 1) XP(2, 512, 2, 18, 0) XP(2, 512, 2, 19, 0)
                                       XP(2, 512, 2, 0, 0) XP(2, 512, 0, 2, 0) XP(2, 512, 3, 2, 0)
                                           XP(2, 512, 18, 2, 0) XP(2, 1024, 2, 2, 0) XP(1, 1024, 2, 2, 0)
                                               XP(4, 256, 2, 2, 1) XP(1, 512, 2, 2, 0)
                                                   // 25..: round 6 (w = 1 + 1e6 (1 + mode) + 1e3 LDS KiB)
                                                   XX(0, 0) XX(0, 48) XX(0, 64) XX(0, 96) XX(1, 0) XX(2, 0)};
#undef X
#undef XL
#undef XP
#undef XX

extern "C" {
int ceil_count() { return (int)(sizeof(kP) / sizeof(kP[0])); }
int ceil_desc(int i, int* out4) {
  if (i < 0 || i >= ceil_count()) return -1;
  out4[0] = kP[i].r; out4[1] = kP[i].w; out4[2] = kP[i].u; out4[3] = kP[i].b;
  return 0;
}
// bytes per stream must be a multiple of B * U * 16 (the harness uses 64 MiB)
int ceil_run(int i, float* c, const float* a, const float* b, uint32_t* sink, size_t bytes, void* stream) {
  if (i < 0 || i >= ceil_count()) return -1;
  kP[i].launch(c, a, b, sink, bytes, (hipStream_t)stream);
  return (int)hipGetLastError();
}
}

// tune_reduce.hip — TUNING ONLY (not the product): fp32 in-place sum kernel
// variants for the 64 MiB chunk, differing in unroll, cache-policy bits on
// loads/stores (aux: 2 = nt, 16 = sc1, 1 = sc0), workgroup size, grid shape
// (0 = one tile per block, else persistent grid of that many blocks) and an
// XCD-contiguous tile mapping.  Aligned body only: the harness passes n as a
// multiple of the tile.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U, int LAUX, int SAUX, int B, int G, int XCD>
__global__ __launch_bounds__(B) void tk(float* c, const float* a, const float* b, uint32_t nvec) {
  const uint32_t nbytes = nvec * 16u;
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)a, 0, nbytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)b, 0, nbytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)c, 0, nbytes, 0x00020000);
  const uint32_t tiles = nvec / (B * U);
  uint32_t t = blockIdx.x;
  if (XCD) {
    const uint32_t g = gridDim.x;
    t = (blockIdx.x % 8) * (g / 8) + blockIdx.x / 8;
  }
  const uint32_t step = G ? gridDim.x : tiles;
  for (; t < tiles; t += step) {
    const uint32_t off = (t * (B * U) + threadIdx.x) * 16u;
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, off + u * B * 16, 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; u++) y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, off + u * B * 16, 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 s = __builtin_bit_cast(f32x4, x[u]) + __builtin_bit_cast(f32x4, y[u]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, s), rc, off + u * B * 16, 0, SAUX);
    }
  }
}

#define VARIANTS \
  X(2,0,0,256,0,0) \
  X(2,0,0,256,2048,0) \
  X(2,0,0,512,0,0) \
  X(2,0,0,512,2048,0) \
  X(2,2,0,256,0,0) \
  X(2,2,0,256,2048,0) \
  X(2,2,0,512,0,0) \
  X(2,2,0,512,2048,0) \
  X(2,2,2,256,0,0) \
  X(2,2,2,256,2048,0) \
  X(2,2,2,512,0,0) \
  X(2,2,2,512,2048,0) \
  X(2,0,2,256,0,0) \
  X(2,0,2,256,2048,0) \
  X(2,0,2,512,0,0) \
  X(2,0,2,512,2048,0) \
  X(2,2,16,256,0,0) \
  X(2,2,16,256,2048,0) \
  X(2,2,16,512,0,0) \
  X(2,2,16,512,2048,0) \
  X(2,16,16,256,0,0) \
  X(2,16,16,256,2048,0) \
  X(2,16,16,512,0,0) \
  X(2,16,16,512,2048,0) \
  X(2,0,16,256,0,0) \
  X(2,0,16,256,2048,0) \
  X(2,0,16,512,0,0) \
  X(2,0,16,512,2048,0) \
  X(2,16,0,256,0,0) \
  X(2,16,0,256,2048,0) \
  X(2,16,0,512,0,0) \
  X(2,16,0,512,2048,0) \
  X(4,0,0,256,0,0) \
  X(4,0,0,256,2048,0) \
  X(4,0,0,512,0,0) \
  X(4,0,0,512,2048,0) \
  X(4,2,0,256,0,0) \
  X(4,2,0,256,2048,0) \
  X(4,2,0,512,0,0) \
  X(4,2,0,512,2048,0) \
  X(4,2,2,256,0,0) \
  X(4,2,2,256,2048,0) \
  X(4,2,2,512,0,0) \
  X(4,2,2,512,2048,0) \
  X(4,0,2,256,0,0) \
  X(4,0,2,256,2048,0) \
  X(4,0,2,512,0,0) \
  X(4,0,2,512,2048,0) \
  X(4,2,16,256,0,0) \
  X(4,2,16,256,2048,0) \
  X(4,2,16,512,0,0) \
  X(4,2,16,512,2048,0) \
  X(4,16,16,256,0,0) \
  X(4,16,16,256,2048,0) \
  X(4,16,16,512,0,0) \
  X(4,16,16,512,2048,0) \
  X(4,0,16,256,0,0) \
  X(4,0,16,256,2048,0) \
  X(4,0,16,512,0,0) \
  X(4,0,16,512,2048,0) \
  X(4,16,0,256,0,0) \
  X(4,16,0,256,2048,0) \
  X(4,16,0,512,0,0) \
  X(4,16,0,512,2048,0) \
  X(8,0,0,256,0,0) \
  X(8,0,0,256,2048,0) \
  X(8,0,0,512,0,0) \
  X(8,0,0,512,2048,0) \
  X(8,2,0,256,0,0) \
  X(8,2,0,256,2048,0) \
  X(8,2,0,512,0,0) \
  X(8,2,0,512,2048,0) \
  X(8,2,2,256,0,0) \
  X(8,2,2,256,2048,0) \
  X(8,2,2,512,0,0) \
  X(8,2,2,512,2048,0) \
  X(8,0,2,256,0,0) \
  X(8,0,2,256,2048,0) \
  X(8,0,2,512,0,0) \
  X(8,0,2,512,2048,0) \
  X(8,2,16,256,0,0) \
  X(8,2,16,256,2048,0) \
  X(8,2,16,512,0,0) \
  X(8,2,16,512,2048,0) \
  X(8,16,16,256,0,0) \
  X(8,16,16,256,2048,0) \
  X(8,16,16,512,0,0) \
  X(8,16,16,512,2048,0) \
  X(8,0,16,256,0,0) \
  X(8,0,16,256,2048,0) \
  X(8,0,16,512,0,0) \
  X(8,0,16,512,2048,0) \
  X(8,16,0,256,0,0) \
  X(8,16,0,256,2048,0) \
  X(8,16,0,512,0,0) \
  X(8,16,0,512,2048,0) \
  X(4,2,0,256,1024,1) \
  X(4,2,0,256,2048,1) \
  X(4,2,0,256,4096,1) \
  X(4,2,2,256,1024,1) \
  X(4,2,2,256,2048,1) \
  X(4,2,2,256,4096,1) \
  X(8,2,0,256,1024,1) \
  X(8,2,0,256,2048,1) \
  X(8,2,0,256,4096,1) \
  X(8,2,2,256,1024,1) \
  X(8,2,2,256,2048,1) \
  X(8,2,2,256,4096,1) \
  X(4,2,0,256,1024,0) \
  X(4,2,0,1024,256,0) \
  X(4,2,0,1024,512,0) \
  X(4,2,2,256,1024,0) \
  X(4,2,2,1024,256,0) \
  X(4,2,2,1024,512,0) \
  X(8,2,0,256,1024,0) \
  X(8,2,0,1024,256,0) \
  X(8,2,0,1024,512,0) \
  X(8,2,2,256,1024,0) \
  X(8,2,2,1024,256,0) \
  X(8,2,2,1024,512,0) \
  X(16,2,0,256,1024,0) \
  X(16,2,0,1024,256,0) \
  X(16,2,0,1024,512,0) \
  X(16,2,2,256,1024,0) \
  X(16,2,2,1024,256,0) \
  X(16,2,2,1024,512,0)

struct V { int u, la, sa, b, g, x; void (*launch)(float*, const float*, const float*, uint32_t, hipStream_t); };

#define X(U, LA, SA, B, G, XC) \
  {U, LA, SA, B, G, XC, [](float* c, const float* a, const float* b, uint32_t nvec, hipStream_t s) { \
     uint32_t tiles = nvec / (B * U); uint32_t grid = G ? (G < tiles ? G : tiles) : tiles; \
     tk<U, LA, SA, B, G, XC><<<grid, B, 0, s>>>(c, a, b, nvec); }},
static const V kV[] = { VARIANTS };
#undef X

extern "C" {
int tune_count() { return (int)(sizeof(kV) / sizeof(kV[0])); }
int tune_desc(int i, int* out6) {
  if (i < 0 || i >= tune_count()) return -1;
  out6[0] = kV[i].u; out6[1] = kV[i].la; out6[2] = kV[i].sa; out6[3] = kV[i].b; out6[4] = kV[i].g; out6[5] = kV[i].x;
  return 0;
}
int tune_run(int i, float* c, const float* a, const float* b, size_t n, void* stream) {
  if (i < 0 || i >= tune_count()) return -1;
  kV[i].launch(c, a, b, (uint32_t)(n / 4), (hipStream_t)stream);
  return (int)hipGetLastError();
}
}

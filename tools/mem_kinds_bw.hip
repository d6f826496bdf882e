// mem_kinds_bw.hip — streaming read+write rate of the kinds of device memory
// an inbox arena could be (VMM route): hipMalloc (coarse),
// hipExtMallocWithFlags(hipDeviceMallocFinegrained) (the executor's
// cross-written inboxes today), and VMM blocks (hipMemCreate) of type Pinned
// (coarse) and Uncached.  The kernel is the config-2 access mix: c = a + b
// over fp32, 16-byte loads and stores; a and c in plain hipMalloc memory, b
// (the "inbox") in the kind under test.  Buffers rotate over 768 MiB (beyond
// the 256 MiB Infinity Cache).  One JSON line per kind.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
#include <vector>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                        \
    }                                                                                      \
  } while (0)

__global__ __launch_bounds__(256) void add_kernel(float4* c, const float4* a, const float4* b, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 x = a[i], y = b[i];
    c[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
}

static void* vmmBlock(size_t bytes, bool uncached) {
  hipMemAllocationProp p{};
  p.type = uncached ? hipMemAllocationTypeUncached : hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  size_t g = 0;
  CHECK(hipMemGetAllocationGranularity(&g, &p, hipMemAllocationGranularityRecommended));
  bytes = (bytes + g - 1) / g * g;
  hipMemGenericAllocationHandle_t h;
  CHECK(hipMemCreate(&h, bytes, &p, 0));
  void* va;
  CHECK(hipMemAddressReserve(&va, bytes, g, nullptr, 0));
  CHECK(hipMemMap(va, bytes, 0, h, 0));
  hipMemAccessDesc d{};
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  CHECK(hipMemSetAccess(va, bytes, &d, 1));
  return va;
}

int main() {
  CHECK(hipSetDevice(0));
  const size_t chunk = 64u << 20, slots = 4, foot = chunk * slots;  // 3 x 256 MiB rotating footprint
  const size_t n4 = chunk / 16;
  float *a, *c;
  CHECK(hipMalloc(&a, foot));
  CHECK(hipMalloc(&c, foot));
  CHECK(hipMemset(a, 0, foot));
  for (std::string kind : {"hipMalloc", "fine", "vmm_pinned", "vmm_uncached"}) {
    void* b = nullptr;
    if (kind == "hipMalloc") CHECK(hipMalloc(&b, foot));
    if (kind == "fine") CHECK(hipExtMallocWithFlags(&b, foot, hipDeviceMallocFinegrained));
    if (kind == "vmm_pinned") b = vmmBlock(foot, false);
    if (kind == "vmm_uncached") b = vmmBlock(foot, true);
    CHECK(hipMemset(b, 0, foot));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 200;
    for (int w = 0; w < 20; w++)
      add_kernel<<<4096, 256>>>((float4*)((char*)c + (w % slots) * chunk), (const float4*)((char*)a + ((w + 1) % slots) * chunk),
                                (const float4*)((char*)b + ((w + 2) % slots) * chunk), n4);
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++)
      add_kernel<<<4096, 256>>>((float4*)((char*)c + (r % slots) * chunk), (const float4*)((char*)a + ((r + 1) % slots) * chunk),
                                (const float4*)((char*)b + ((r + 2) % slots) * chunk), n4);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    std::printf("{\"inbox_kind\": \"%s\", \"chunk_bytes\": %zu, \"us_per_launch\": %.2f, \"GBs_2r1w\": %.1f}\n",
                kind.c_str(), chunk, us, 3.0 * chunk / us / 1e3);
    std::fflush(stdout);
  }
  return 0;
}

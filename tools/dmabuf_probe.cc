// dmabuf_probe.cc — MEASUREMENT / DIAGNOSIS ONLY: can a
// caller's hipMalloc block be shared without hipIpc?  Exports the block with
// hsa_amd_portable_export_dmabuf (the HSA runtime the HIP runtime loaded,
// found with dlopen RTLD_NOLOAD) and imports the fd back two ways:
//   vmem     hipMemImportFromShareableHandle + hipMemMap into a fresh range
//   interop  hsa_amd_interop_map_buffer (the dma-buf interop path)
// For each: the bytes written through the import must be what the owner
// reads, and the owner's writes what the import reads.  Then the block is
// freed, a new one of the same size is allocated (often at the same
// address) and exported again: the new import must show the NEW block.
// One JSON line per (way, size).  Same process: the API's acceptance of the
// fd is what is probed (a peer process receives the same fd by SCM_RIGHTS).
//   dmabuf_probe [bytes...]
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::printf("{\"fatal\": \"%s:%d %s: %s\"}\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

using ExportFn = hsa_status_t (*)(const void*, size_t, int*, uint64_t*);
using CloseFn = hsa_status_t (*)(int);
using IterFn = hsa_status_t (*)(hsa_status_t (*)(hsa_agent_t, void*), void*);
using InfoFn = hsa_status_t (*)(hsa_agent_t, hsa_agent_info_t, void*);
using MapFn = hsa_status_t (*)(uint32_t, hsa_agent_t*, int, uint32_t, size_t*, void**, size_t*, const void**);
using UnmapFn = hsa_status_t (*)(void*);

static void* hsaSym(const char* name) {
  static void* h = [] {
    void* x = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!x) x = dlopen("libhsa-runtime64.so", RTLD_NOW | RTLD_NOLOAD);
    return x;
  }();
  return h ? dlsym(h, name) : nullptr;
}

__global__ void fill(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v + (uint32_t)i;
}
__global__ void sum(const uint32_t* p, size_t n, uint32_t v, unsigned long long* bad) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != v + (uint32_t)i) atomicAdd(bad, 1ull);
}

static unsigned long long check(const void* p, size_t bytes, uint32_t v) {
  unsigned long long* bad;
  CHECK(hipMallocManaged(&bad, sizeof(*bad)));
  *bad = 0;
  sum<<<256, 256>>>(static_cast<const uint32_t*>(p), bytes / 4, v, bad);
  CHECK(hipDeviceSynchronize());
  unsigned long long r = *bad;
  CHECK(hipFree(bad));
  return r;
}

static hsa_agent_t g_agent{0};
static hsa_status_t pickGpu(hsa_agent_t a, void* info) {
  hsa_device_type_t t;
  reinterpret_cast<InfoFn>(info)(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && g_agent.handle == 0) g_agent = a;
  return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
  std::vector<size_t> sizes;
  for (int i = 1; i < argc; i++) sizes.push_back(std::strtoull(argv[i], nullptr, 10));
  if (sizes.empty()) sizes = {4096, 1 << 20, 64 << 20};
  CHECK(hipSetDevice(0));
  CHECK(hipFree(nullptr));
  auto exportFn = reinterpret_cast<ExportFn>(hsaSym("hsa_amd_portable_export_dmabuf"));
  auto closeFn = reinterpret_cast<CloseFn>(hsaSym("hsa_amd_portable_close_dmabuf"));
  auto iterFn = reinterpret_cast<IterFn>(hsaSym("hsa_iterate_agents"));
  auto infoFn = reinterpret_cast<InfoFn>(hsaSym("hsa_agent_get_info"));
  auto mapFn = reinterpret_cast<MapFn>(hsaSym("hsa_amd_interop_map_buffer"));
  auto unmapFn = reinterpret_cast<UnmapFn>(hsaSym("hsa_amd_interop_unmap_buffer"));
  std::printf("{\"hsa_symbols\": {\"export\": %d, \"close\": %d, \"iterate\": %d, \"interop_map\": %d}}\n",
              exportFn != nullptr, closeFn != nullptr, iterFn != nullptr, mapFn != nullptr);
  if (!exportFn) return 1;
  if (iterFn && infoFn) iterFn(pickGpu, reinterpret_cast<void*>(infoFn));
  std::fflush(stdout);
  for (const char* way : {"vmem", "interop"}) {
    for (size_t bytes : sizes) {
      std::string err;
      unsigned long long badA = 0, badB = 0, badNew = 0;
      void* first = nullptr;
      void* second = nullptr;
      for (int round = 0; round < 2; round++) {
        void* p = nullptr;
        CHECK(hipMalloc(&p, bytes));
        (round == 0 ? first : second) = p;
        const uint32_t v = 1000u * (round + 1);
        fill<<<256, 256>>>(static_cast<uint32_t*>(p), bytes / 4, v);
        CHECK(hipDeviceSynchronize());
        int fd = -1;
        uint64_t off = 0;
        hsa_status_t hs = exportFn(p, bytes, &fd, &off);
        if (hs != HSA_STATUS_SUCCESS) {
          err = "export rc " + std::to_string((int)hs);
          CHECK(hipFree(p));
          break;
        }
        void* mapped = nullptr;
        size_t mappedBytes = 0;
        hipMemGenericAllocationHandle_t h = nullptr;
        void* va = nullptr;
        size_t vaBytes = 0;
        if (std::string(way) == "vmem") {
          hipError_t e = hipMemImportFromShareableHandle(&h, reinterpret_cast<void*>((intptr_t)fd),
                                                         hipMemHandleTypePosixFileDescriptor);
          if (e != hipSuccess) {
            int fdv = fd;  // HIP 7.0 takes the fd's address
            e = hipMemImportFromShareableHandle(&h, &fdv, hipMemHandleTypePosixFileDescriptor);
          }
          if (e != hipSuccess) {
            err = std::string("import: ") + hipGetErrorString(e);
            (void)hipGetLastError();
          } else {
            size_t gran = 0;
            hipMemAllocationProp prop;
            std::memset(&prop, 0, sizeof(prop));
            prop.type = hipMemAllocationTypePinned;
            prop.location.type = hipMemLocationTypeDevice;
            prop.location.id = 0;
            (void)hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
            if (gran == 0) gran = 4096;
            vaBytes = (off + bytes + gran - 1) / gran * gran;
            e = hipMemAddressReserve(&va, vaBytes, 0, nullptr, 0);
            if (e == hipSuccess) e = hipMemMap(va, vaBytes, 0, h, 0);
            if (e == hipSuccess) {
              hipMemAccessDesc d;
              std::memset(&d, 0, sizeof(d));
              d.location.type = hipMemLocationTypeDevice;
              d.location.id = 0;
              d.flags = hipMemAccessFlagsProtReadWrite;
              e = hipMemSetAccess(va, vaBytes, &d, 1);
            }
            if (e != hipSuccess) {
              err = std::string("map: ") + hipGetErrorString(e);
              (void)hipGetLastError();
            } else {
              mapped = static_cast<char*>(va) + off;
            }
          }
        } else {
          if (!mapFn || g_agent.handle == 0) {
            err = "no interop map / agent";
          } else {
            void* ptr = nullptr;
            size_t sz = 0;
            hsa_status_t ms = mapFn(1, &g_agent, fd, 0, &sz, &ptr, nullptr, nullptr);
            if (ms != HSA_STATUS_SUCCESS) {
              err = "interop map rc " + std::to_string((int)ms);
            } else {
              mapped = static_cast<char*>(ptr) + off;
              mappedBytes = sz;
            }
          }
        }
        if (mapped) {
          // the import shows the owner's bytes ...
          unsigned long long b1 = check(mapped, bytes, v);
          // ... and the owner sees the import's writes
          fill<<<256, 256>>>(static_cast<uint32_t*>(mapped), bytes / 4, v + 7);
          CHECK(hipDeviceSynchronize());
          unsigned long long b2 = check(p, bytes, v + 7);
          if (round == 0) {
            badA = b1;
            badB = b2;
          } else {
            badNew = b1 + b2;
          }
          if (std::string(way) == "vmem") {
            (void)hipMemUnmap(va, vaBytes);
            (void)hipMemRelease(h);
            // the range stays reserved (ipc.h: never mapped twice)
          } else {
            (void)unmapFn(static_cast<char*>(mapped) - off);
          }
        }
        if (closeFn) (void)closeFn(fd);
        else ::close(fd);
        CHECK(hipFree(p));
        if (!err.empty()) break;
        (void)mappedBytes;
      }
      std::printf("{\"way\": \"%s\", \"bytes\": %zu, \"ok\": %s, \"err\": \"%s\", \"bad_import_reads\": %llu, "
                  "\"bad_owner_reads\": %llu, \"bad_after_realloc\": %llu, \"same_address_realloc\": %s}\n",
                  way, bytes, err.empty() && badA == 0 && badB == 0 && badNew == 0 ? "true" : "false",
                  err.c_str(), badA, badB, badNew, first == second ? "true" : "false");
      std::fflush(stdout);
    }
  }
  return 0;
}

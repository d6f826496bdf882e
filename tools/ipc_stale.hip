// ipc_stale.hip — MEASUREMENT / DIAGNOSIS ONLY: the minimal reproduction of
// the stale HIP IPC import (DESIGN.md §4 "IPC imports").
//
// Two processes on one GPU, records through files in DIR:
//   ipc_stale 1 DIR WRITER ITERS   exporter
//   ipc_stale 0 DIR WRITER ITERS   importer (one JSON line per iteration)
// Every iteration the exporter hipMalloc's a BYTES block (hipFree'd at the
// end of the iteration, so the next one comes back at the same address and
// the same size: a byte-identical IPC handle), writes a fresh nonce at its
// start, exports it and waits for the importer.  The importer opens the
// handle, reads the first word through the mapping twice (hipMemcpy = the
// runtime's record of the pointer; a kernel load = the GPU page tables),
// then WRITES into the mapping with WRITER:
//   none     nothing
//   memcpy   hipMemcpyAsync device-to-device into the mapping (an executor SEND
//            on the memcpy engine, or the transport's Buffer::send)
//   kernel   a copy kernel into the mapping (the copy_signal_kernel engine)
//   graph-memcpy / graph-kernel   the memcpy / kernel write captured into a
//            hipGraph, replayed twice, graph destroyed before the close
// and closes the mapping (hipIpcCloseMemHandle) before acking.
// Importer exit 1 = some iteration read a stale nonce.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

struct Rec {
  uint64_t ptr, nonce;
  hipIpcMemHandle_t handle;
};

__global__ void probe(const uint64_t* p, uint64_t* out) {
  if (threadIdx.x == 0) *out = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void fill(uint32_t* dst, const uint32_t* src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

static void waitFile(const std::string& f) {
  for (int i = 0; i < 200000; i++) {
    if (access(f.c_str(), F_OK) == 0) return;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  std::fprintf(stderr, "timeout waiting for %s\n", f.c_str());
  std::exit(3);
}

static void writeFile(const std::string& f, const void* p, size_t n) {
  const std::string tmp = f + ".tmp";
  std::ofstream o(tmp, std::ios::binary);
  o.write(static_cast<const char*>(p), n);
  o.close();
  std::rename(tmp.c_str(), f.c_str());
}

int main(int argc, char** argv) {
  if (argc < 5) return 1;
  const int rank = std::atoi(argv[1]);
  const std::string dir = argv[2], writer = argv[3];
  const int iters = std::atoi(argv[4]);
  const size_t bytes = std::getenv("IPC_MIB") ? (size_t)std::atoi(std::getenv("IPC_MIB")) << 20 : (size_t)128 << 20;
  CHECK(hipSetDevice(0));
  if (rank == 1) {
    for (int it = 0; it < iters; it++) {
      void* p = nullptr;
      CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
      Rec r;
      std::memset(&r, 0, sizeof(r));
      r.ptr = reinterpret_cast<uint64_t>(p);
      r.nonce = 0x1234567800000000ull + (uint64_t)it * 7919 + (uint64_t)getpid();
      CHECK(hipMemcpy(p, &r.nonce, 8, hipMemcpyHostToDevice));
      CHECK(hipDeviceSynchronize());
      CHECK(hipIpcGetMemHandle(&r.handle, p));
      writeFile(dir + "/exp_" + std::to_string(it), &r, sizeof(r));
      waitFile(dir + "/ack_" + std::to_string(it));
      CHECK(hipFree(p));
    }
    return 0;
  }
  // IPC_WRITE_MIB per write (default 1), IPC_WRITES writes at consecutive offsets (default 1)
  const size_t wbytes = (std::getenv("IPC_WRITE_MIB") ? (size_t)std::atoi(std::getenv("IPC_WRITE_MIB")) : 1) << 20;
  const int writes = std::getenv("IPC_WRITES") ? std::atoi(std::getenv("IPC_WRITES")) : 1;
  void* local = nullptr;
  uint64_t* out = nullptr;
  hipStream_t s;
  CHECK(hipMalloc(&local, wbytes));
  CHECK(hipMemset(local, 0x33, wbytes));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&out), 8, 0));
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int bad = 0;
  uint64_t prevPtr = 0;
  void* prevMap = nullptr;
  for (int it = 0; it < iters; it++) {
    const std::string f = dir + "/exp_" + std::to_string(it);
    waitFile(f);
    Rec r;
    std::ifstream i(f, std::ios::binary);
    i.read(reinterpret_cast<char*>(&r), sizeof(r));
    void* m = nullptr;
    CHECK(hipIpcOpenMemHandle(&m, r.handle, hipIpcMemLazyEnablePeerAccess));
    uint64_t viaCopy = 0;
    CHECK(hipMemcpy(&viaCopy, m, 8, hipMemcpyDeviceToHost));
    *out = 0;
    probe<<<1, 64, 0, s>>>(static_cast<const uint64_t*>(m), out);
    CHECK(hipStreamSynchronize(s));
    const uint64_t viaKernel = *out;
    const bool ok = viaCopy == r.nonce && viaKernel == r.nonce;
    if (writer == "memcpy") {
      for (int w = 0; w < writes; w++)
        CHECK(hipMemcpyAsync(static_cast<char*>(m) + 4096 + (size_t)w * wbytes, local, wbytes,
                             hipMemcpyDeviceToDevice, s));
    } else if (writer == "kernel") {
      fill<<<64, 256, 0, s>>>(reinterpret_cast<uint32_t*>(static_cast<char*>(m) + 4096),
                              static_cast<const uint32_t*>(local), wbytes / 4);
    } else if (writer == "graph-memcpy" || writer == "graph-kernel") {
      // the same write captured into a hipGraph, replayed twice, then the
      // graph destroyed before the close (an executor's graph replay)
      hipGraph_t g = nullptr;
      hipGraphExec_t ge = nullptr;
      CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      if (writer == "graph-memcpy")
        CHECK(hipMemcpyAsync(static_cast<char*>(m) + 4096, local, wbytes, hipMemcpyDeviceToDevice, s));
      else
        fill<<<64, 256, 0, s>>>(reinterpret_cast<uint32_t*>(static_cast<char*>(m) + 4096),
                                static_cast<const uint32_t*>(local), wbytes / 4);
      CHECK(hipStreamEndCapture(s, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CHECK(hipGraphDestroy(g));
      CHECK(hipGraphLaunch(ge, s));
      CHECK(hipGraphLaunch(ge, s));
      CHECK(hipStreamSynchronize(s));
      CHECK(hipGraphExecDestroy(ge));
    }
    CHECK(hipStreamSynchronize(s));
    bad += !ok;
    std::printf("{\"writer\": \"%s\", \"mib\": %zu, \"iter\": %d, \"exporter_ptr\": \"%p\", \"same_exporter_ptr\": %s, "
                "\"mapped\": \"%p\", \"same_mapping\": %s, \"ok\": %s, \"via_memcpy\": \"%llx\", "
                "\"via_kernel\": \"%llx\", \"want\": \"%llx\"}\n",
                writer.c_str(), bytes >> 20, it, (void*)r.ptr, r.ptr == prevPtr ? "true" : "false", m,
                m == prevMap ? "true" : "false", ok ? "true" : "false", (unsigned long long)viaCopy,
                (unsigned long long)viaKernel, (unsigned long long)r.nonce);
    std::fflush(stdout);
    prevPtr = r.ptr;
    prevMap = m;
    CHECK(hipIpcCloseMemHandle(m));
    writeFile(dir + "/ack_" + std::to_string(it), "k", 1);
  }
  return bad ? 1 : 0;
}

// ipc_reuse.cc — does a HIP IPC import reach the exporter's CURRENT block
// when blocks are freed / reused / re-exported between imports?
//
// Two processes on one GPU, exchanging records through files in DIR:
//   ipc_reuse 1 DIR MODE    exporter
//   ipc_reuse 0 DIR MODE    importer (prints one JSON line per iteration)
// MODE (exporter, importer):
//   free-close   new block per iteration, freed after use; importer closes
//   pool-close   one block reused every iteration;          importer closes
//   pool-keep    one block reused;                          importer keeps its first mapping
//   free-keep    new block per iteration, freed;            importer keeps (never closes)
//   twobuf-close two blocks of one size alternately reused; importer closes
//   ...-w        (suffix) the importer also writes IPC_WRITE_MIB (default 1) MiB
//                into the mapping with hipMemcpyAsync device-to-device before
//                closing it
// Each iteration the exporter writes a fresh nonce at the block's start
// (hipMemcpy H2D, synchronised), exports the handle and waits for the
// importer's verdict before the next iteration.
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                      \
    }                                                                                    \
  } while (0)

struct Rec {
  uint64_t ptr, nonce;
  hipIpcMemHandle_t handle;
};

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
  if (argc < 4) return 1;
  const int rank = std::atoi(argv[1]);
  const std::string dir = argv[2], mode = argv[3];
  const int iters = argc > 4 ? std::atoi(argv[4]) : 6;
  const size_t bytes = 128u << 20;
  CHECK(hipSetDevice(0));
  const bool pool = mode.rfind("pool", 0) == 0, twobuf = mode.rfind("twobuf", 0) == 0;
  const bool keep = mode.find("keep") != std::string::npos;
  if (rank == 1) {
    void* blocks[2] = {nullptr, nullptr};
    for (int it = 0; it < iters; it++) {
      void* p = nullptr;
      if (pool) {
        if (!blocks[0]) CHECK(hipMalloc(&blocks[0], bytes));
        p = blocks[0];
      } else if (twobuf) {
        if (!blocks[it & 1]) CHECK(hipMalloc(&blocks[it & 1], bytes));
        p = blocks[it & 1];
      } else {
        CHECK(hipMalloc(&p, bytes));
      }
      // something else allocated and freed in between, as a framework would
      void* junk = nullptr;
      CHECK(hipMalloc(&junk, bytes));
      CHECK(hipMemset(junk, 0x5a, bytes));
      CHECK(hipDeviceSynchronize());
      Rec r;
      std::memset(&r, 0, sizeof(r));
      r.ptr = reinterpret_cast<uint64_t>(p);
      r.nonce = 0x1234567800000000ull + it * 7919 + getpid();
      CHECK(hipMemcpy(p, &r.nonce, 8, hipMemcpyHostToDevice));
      CHECK(hipDeviceSynchronize());
      CHECK(hipIpcGetMemHandle(&r.handle, p));
      writeFile(dir + "/exp_" + std::to_string(it), &r, sizeof(r));
      waitFile(dir + "/ack_" + std::to_string(it));
      CHECK(hipFree(junk));
      if (!pool && !twobuf) CHECK(hipFree(p));
    }
    return 0;
  }
  void* kept = nullptr;
  uint64_t keptPtr = 0;
  const bool write = mode.find("-w") != std::string::npos;
  void* local = nullptr;
  hipStream_t s;
  const size_t wbytes = std::getenv("IPC_WRITE_MIB") ? (size_t)std::atoi(std::getenv("IPC_WRITE_MIB")) << 20 : 1u << 20;
  CHECK(hipMalloc(&local, wbytes));
  CHECK(hipMemset(local, 0x33, wbytes));
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int bad = 0;
  for (int it = 0; it < iters; it++) {
    const std::string f = dir + "/exp_" + std::to_string(it);
    waitFile(f);
    Rec r;
    std::ifstream i(f, std::ios::binary);
    i.read(reinterpret_cast<char*>(&r), sizeof(r));
    void* m = nullptr;
    bool reused = false;
    if (keep && kept && keptPtr == r.ptr) {
      m = kept;
      reused = true;
    } else {
      CHECK(hipIpcOpenMemHandle(&m, r.handle, hipIpcMemLazyEnablePeerAccess));
    }
    uint64_t seen = 0;
    CHECK(hipMemcpy(&seen, m, 8, hipMemcpyDeviceToHost));
    CHECK(hipDeviceSynchronize());
    const bool ok = seen == r.nonce;
    if (write) {
      // as an executor's SEND does: device-to-device copies into the mapping
      CHECK(hipMemcpyAsync(static_cast<char*>(m) + 4096, local, wbytes, hipMemcpyDeviceToDevice, s));
      CHECK(hipStreamSynchronize(s));
    }
    bad += !ok;
    std::printf("{\"mode\": \"%s\", \"iter\": %d, \"exporter_ptr\": \"%p\", \"mapped\": \"%p\", \"reused_mapping\": %s, "
                "\"ok\": %s, \"seen\": \"%llx\", \"want\": \"%llx\"}\n",
                mode.c_str(), it, (void*)r.ptr, m, reused ? "true" : "false", ok ? "true" : "false",
                (unsigned long long)seen, (unsigned long long)r.nonce);
    std::fflush(stdout);
    if (keep) {
      if (!kept) {
        kept = m;
        keptPtr = r.ptr;
      }
    } else {
      CHECK(hipIpcCloseMemHandle(m));
    }
    writeFile(dir + "/ack_" + std::to_string(it), "k", 1);
  }
  return bad ? 1 : 0;
}

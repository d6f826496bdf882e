// transport_big.cc — diagnosis: a device receive buffer in a 2.5 GiB
// allocation, written by a peer process through gloo_hip_buffer_* (the
// landing-slab route of transport.cc), with a SIGSEGV handler that prints the
// native backtrace (library offsets, for addr2line against the same build).
//   transport_big RANK STORE_DIR
#include <execinfo.h>
#include <hip/hip_runtime_api.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gloo_amd.h"

#define OK(x)                                                                                       \
  do {                                                                                              \
    int rc_ = (x);                                                                                  \
    if (rc_ != 0) {                                                                                 \
      std::fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, rc_, gloo_hip_last_error()); \
      std::exit(2);                                                                                 \
    }                                                                                               \
  } while (0)

static void onSegv(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "SIGSEGV backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  signal(SIGSEGV, onSegv);
  const int rank = std::atoi(argv[1]);
  (void)hipSetDevice(0);
  gloo_hip_context_t ctx;
  OK(gloo_hip_context_create(rank, 2, (std::string("file:") + argv[2]).c_str(), 0, 30000, &ctx));
  gloo_hip_transport_t t;
  OK(gloo_hip_transport_create(ctx, nullptr, &t));
  const size_t n = size_t(5) << 29, msg = 16u << 20, far = n - msg - 5;
  if (rank == 1) {
    void* big = nullptr;
    if (hipMalloc(&big, n) != hipSuccess) return 3;
    (void)hipMemset(big, 0, n);
    gloo_hip_buffer_t rb;
    OK(gloo_hip_buffer_create(t, 0, 1, big, n, 0, &rb));
    std::fprintf(stderr, "[r1] receive buffer created\n");
    OK(gloo_hip_buffer_wait_recv(rb));
    std::vector<unsigned char> h(msg);
    (void)hipMemcpy(h.data(), static_cast<char*>(big) + far, msg, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < msg; i++) bad += h[i] != (unsigned char)(i % 253);
    std::printf("bad %zu\n", bad);
    OK(gloo_hip_buffer_destroy(rb));
    (void)hipFree(big);
  } else {
    std::vector<unsigned char> h(msg);
    for (size_t i = 0; i < msg; i++) h[i] = (unsigned char)(i % 253);
    void* src = nullptr;
    if (hipMalloc(&src, msg) != hipSuccess) return 3;
    (void)hipMemcpy(src, h.data(), msg, hipMemcpyHostToDevice);
    gloo_hip_buffer_t sb;
    OK(gloo_hip_buffer_create(t, 1, 1, src, msg, 1, &sb));
    std::fprintf(stderr, "[r0] sending\n");
    OK(gloo_hip_buffer_send(sb, 0, msg, far));
    std::fprintf(stderr, "[r0] sent\n");
    OK(gloo_hip_buffer_wait_send(sb));
    OK(gloo_hip_buffer_destroy(sb));
    (void)hipFree(src);
  }
  OK(gloo_hip_transport_destroy(t));
  OK(gloo_hip_context_destroy(ctx));
  std::fprintf(stderr, "[r%d] done\n", rank);
  return 0;
}

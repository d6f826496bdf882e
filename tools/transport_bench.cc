// transport_bench.cc — latency and bandwidth of gloo::transport::hip's bound
// buffers (gloo_amd/csrc/transport.cc) between two processes, with the
// reference benchmark runner's method (gloo/benchmark/runner.cc:311-363,
// printDistribution :481-520):
//   * 5 warm-up iterations;
//   * an iteration count from the warm-up median: max(1, min_time / median),
//     decided on rank 0 and sent to rank 1 (the runner broadcasts it), then
//     grown by 2x until the samples span min_time (GLOO_BENCH_MIN_MS, default
//     500 ms; the runner's default is 2 s);
//   * per size: min / p50 / p99 / max one-way latency and GiB/s = bytes x
//     samples / summed one-way time, as printDistribution computes it.
// One sample is a ping-pong: rank 0 sends `bytes` into rank 1's receive
// buffer, rank 1 waits for it and sends `bytes` back, rank 0 waits; the
// one-way time is half the round trip.  Kinds: "device" (both buffers device
// memory: the copy kernel with its fused arrival signal) and "host" (both
// host memory: the receiver's landing segment).  One JSON line per size.
//
// Usage: transport_bench RANK STORE_DIR KIND [MIN_BYTES MAX_BYTES]
//        (two processes, RANK 0 and 1; tools/transport_bench.sh runs both)
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gloo_amd.h"

#define OK(x)                                                                                   \
  do {                                                                                          \
    int rc_ = (x);                                                                              \
    if (rc_ != 0) {                                                                             \
      std::fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, rc_, gloo_hip_last_error()); \
      std::exit(2);                                                                             \
    }                                                                                           \
  } while (0)
#define HIPOK(x)                                                                               \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      std::exit(2);                                                                            \
    }                                                                                          \
  } while (0)

using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s RANK STORE_DIR device|host [MIN_BYTES MAX_BYTES]\n", argv[0]);
    return 2;
  }
  const int rank = std::atoi(argv[1]);
  const std::string dir = argv[2];
  const std::string kind = argv[3];
  const size_t minBytes = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 1024;
  const size_t maxBytes = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 256u << 20;
  const char* mt = std::getenv("GLOO_BENCH_MIN_MS");
  const double minSeconds = (mt ? std::atof(mt) : 500.0) / 1e3;
  const bool device = kind == "device";
  const int peer = 1 - rank;
  HIPOK(hipSetDevice(0));
  gloo_hip_context_t ctx;
  OK(gloo_hip_context_create(rank, 2, ("file:" + dir).c_str(), 0, 60000, &ctx));
  gloo_hip_transport_t t;
  OK(gloo_hip_transport_create(ctx, nullptr, &t));
  // control channel: rank 0 tells rank 1 how many iterations to run (host words)
  int ctrlOut = 0, ctrlIn = 0;
  gloo_hip_buffer_t ctrlSend, ctrlRecv;
  OK(gloo_hip_buffer_create(t, peer, 1, &ctrlOut, sizeof(int), 1, &ctrlSend));
  OK(gloo_hip_buffer_create(t, peer, 1, &ctrlIn, sizeof(int), 0, &ctrlRecv));
  int slot = 2;
  for (size_t bytes = minBytes; bytes <= maxBytes; bytes *= 4, slot++) {
    void *sp = nullptr, *rp = nullptr;
    if (device) {
      HIPOK(hipMalloc(&sp, bytes));
      HIPOK(hipMalloc(&rp, bytes));
      HIPOK(hipMemset(sp, rank + 1, bytes));
      HIPOK(hipMemset(rp, 0, bytes));
    } else {
      sp = std::malloc(bytes);
      rp = std::malloc(bytes);
      std::memset(sp, rank + 1, bytes);
      std::memset(rp, 0, bytes);
    }
    gloo_hip_buffer_t sb, rb;
    OK(gloo_hip_buffer_create(t, peer, slot, sp, bytes, 1, &sb));
    OK(gloo_hip_buffer_create(t, peer, slot, rp, bytes, 0, &rb));
    // one ping-pong; rank 0 returns its round-trip seconds
    auto once = [&]() -> double {
      const auto t0 = Clock::now();
      if (rank == 0) {
        OK(gloo_hip_buffer_send(sb, 0, bytes, 0));
        OK(gloo_hip_buffer_wait_recv(rb));
      } else {
        OK(gloo_hip_buffer_wait_recv(rb));
        OK(gloo_hip_buffer_send(sb, 0, bytes, 0));
      }
      return std::chrono::duration<double>(Clock::now() - t0).count();
    };
    auto run = [&](int n, std::vector<double>* out) {
      for (int i = 0; i < n; i++) {
        const double s = once();
        if (out) out->push_back(s / 2);
      }
      OK(gloo_hip_buffer_wait_send(sb));
    };
    auto agree = [&](int n) {  // rank 0's count, as the runner's broadcast()
      if (rank == 0) {
        ctrlOut = n;
        OK(gloo_hip_buffer_send(ctrlSend, 0, sizeof(int), 0));
      } else {
        OK(gloo_hip_buffer_wait_recv(ctrlRecv));
        n = ctrlIn;
      }
      return n;
    };
    std::vector<double> warm;
    run(5, &warm);
    std::sort(warm.begin(), warm.end());
    int iters = agree(std::max(1, (int)(minSeconds / std::max(1e-9, 2 * warm[warm.size() / 2]))));
    std::vector<double> lat;
    for (;;) {
      lat.clear();
      run(iters, &lat);
      double sum = 0;
      for (double x : lat) sum += x;
      const int next = (rank == 0 && 2 * sum < minSeconds && iters < (1 << 20)) ? iters * 2 : 0;
      const int n = agree(next);
      if (n == 0) break;
      iters = n;
    }
    // bytes landed intact (the last message rank 1 sent back to rank 0)
    std::vector<unsigned char> check(std::min<size_t>(bytes, 4096));
    if (device) {
      HIPOK(hipMemcpy(check.data(), static_cast<char*>(rp) + bytes - check.size(), check.size(), hipMemcpyDeviceToHost));
    } else {
      std::memcpy(check.data(), static_cast<char*>(rp) + bytes - check.size(), check.size());
    }
    const bool intact = std::all_of(check.begin(), check.end(), [&](unsigned char c) { return c == (unsigned char)(peer + 1); });
    if (rank == 0) {
      std::vector<double> s = lat;
      std::sort(s.begin(), s.end());
      double sum = 0;
      for (double x : s) sum += x;
      auto pct = [&](double p) { return s[std::min(s.size() - 1, (size_t)(p * (double)s.size()))]; };
      std::printf("{\"kind\": \"%s\", \"publish\": \"%s\", \"bytes\": %zu, \"samples\": %zu, \"min_us\": %.2f, "
                  "\"p50_us\": %.2f, \"p99_us\": %.2f, \"max_us\": %.2f, \"GiB_s\": %.3f, \"intact\": %s}\n",
                  kind.c_str(), "device", bytes,
                  s.size(), s.front() * 1e6, pct(0.5) * 1e6, pct(0.99) * 1e6, s.back() * 1e6,
                  (double)bytes * (double)s.size() / sum / (1024.0 * 1024 * 1024), intact ? "true" : "false");
      std::fflush(stdout);
    }
    if (!intact) {
      std::fprintf(stderr, "rank %d: %zu-byte message corrupted\n", rank, bytes);
      return 1;
    }
    OK(gloo_hip_buffer_destroy(sb));
    OK(gloo_hip_buffer_destroy(rb));
    if (device) {
      HIPOK(hipFree(sp));
      HIPOK(hipFree(rp));
    } else {
      std::free(sp);
      std::free(rp);
    }
  }
  OK(gloo_hip_buffer_destroy(ctrlSend));
  OK(gloo_hip_buffer_destroy(ctrlRecv));
  OK(gloo_hip_transport_destroy(t));
  OK(gloo_hip_context_destroy(ctx));
  return 0;
}

// tools/latency.cc — measurement tool (not part of the product): where the
// time of a small allreduce goes on the host.  Two (or more) rank processes
// run HipAllreduceHalvingDoubling<float> over `count` elements `iters` times
// on a caller stream and time, per call:
//   enqueue  run() returning (the plan's launches or one graph launch)
//   total    run() + hipStreamSynchronize (the call as a user sees it)
// and, as the floor, one empty kernel launch + hipStreamSynchronize.
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -Igloo_amd/include tools/latency.cc \
//        -o tools/latency -Lgloo_amd -lgloo_amd -Wl,-rpath,'$ORIGIN/../gloo_amd'
// Prints one JSON line per rank with p50 / p90 of both, in microseconds.
// LATENCY_ALGO=ring_chunked runs HipAllreduceRingChunked<float> instead.
// LATENCY_OWN_STREAM=1 passes no stream: run() returns with the outputs
// complete (the synchronous form) and `total` is run() alone.
//
//   latency <rank> <size> <store-url> [count=256] [iters=2000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "gloo_amd/hip_allreduce.h"
#include "gloo_amd/store.h"

__global__ void nop_kernel() {}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: latency rank size store [count] [iters]\n");
    return 2;
  }
  const int rank = std::atoi(argv[1]), size = std::atoi(argv[2]);
  const std::string url = argv[3];
  const int count = argc > 4 ? std::atoi(argv[4]) : 256;
  const int iters = argc > 5 ? std::atoi(argv[5]) : 2000;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return 2;
  const int dev = rank % ndev;
  (void)hipSetDevice(dev);
  auto ctx = std::make_shared<gloo_amd::Context>(rank, size);
  ctx->connect(gloo_amd::openStore(url), dev);
  float* d = nullptr;
  (void)hipMalloc(&d, count * sizeof(float));
  (void)hipMemset(d, 0, count * sizeof(float));
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const char* la = std::getenv("LATENCY_ALGO");
  const std::string algoName = la ? la : "halving_doubling";
  // LATENCY_OWN_STREAM=1: no stream passed, so run() returns with the outputs
  // valid (the reference's synchronous form) and the tool synchronises nothing
  const char* os = std::getenv("LATENCY_OWN_STREAM");
  std::vector<hipStream_t> streams;
  if (!(os && os[0] == '1')) streams.push_back(s);
  std::unique_ptr<gloo_amd::Algorithm> algop;
  if (algoName == "ring_chunked") {
    algop.reset(new gloo_amd::HipAllreduceRingChunked<float>(ctx, {d}, count, streams));
  } else if (algoName == "bcube") {  // LATENCY_BASE: gloo::Context::base (default 2)
    const char* lb = std::getenv("LATENCY_BASE");
    ctx->base = lb ? std::atoi(lb) : 2;
    algop.reset(new gloo_amd::HipAllreduceBcube<float>(ctx, {d}, count, streams));
  } else
    algop.reset(new gloo_amd::HipAllreduceHalvingDoubling<float>(ctx, {d}, count, streams));
  gloo_amd::Algorithm& algo = *algop;
  for (int i = 0; i < 50; i++) {
    algo.run();
    (void)hipStreamSynchronize(s);
  }
  // floor: one empty launch + synchronize on the same stream
  std::vector<double> nop;
  for (int i = 0; i < iters; i++) {
    const auto t0 = std::chrono::steady_clock::now();
    nop_kernel<<<1, 64, 0, s>>>();
    (void)hipStreamSynchronize(s);
    nop.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6);
  }
  std::vector<double> enq, tot;
  for (int i = 0; i < iters; i++) {
    const auto t0 = std::chrono::steady_clock::now();
    algo.run();
    const auto t1 = std::chrono::steady_clock::now();
    if (!streams.empty()) (void)hipStreamSynchronize(s);  // own stream: run() returned complete
    const auto t2 = std::chrono::steady_clock::now();
    enq.push_back(std::chrono::duration<double>(t1 - t0).count() * 1e6);
    tot.push_back(std::chrono::duration<double>(t2 - t0).count() * 1e6);
  }
  auto pct = [](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (v.size() - 1))];
  };
  const char* g = std::getenv("LATENCY_LABEL");
  std::printf("{\"rank\": %d, \"size\": %d, \"algo\": \"%s\", \"count\": %d, \"mode\": \"%s\", \"enqueue_us_p50\": %.2f, "
              "\"enqueue_us_p90\": %.2f, \"total_us_p50\": %.2f, \"total_us_p90\": %.2f, \"nop_launch_sync_us_p50\": %.2f}\n",
              rank, size, algoName.c_str(), count, g ? g : "auto", pct(enq, 0.5), pct(enq, 0.9), pct(tot, 0.5), pct(tot, 0.9),
              pct(nop, 0.5));
  (void)hipFree(d);
  return 0;
}

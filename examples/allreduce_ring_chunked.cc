// examples/allreduce_ring_chunked.cc — the reference's usage pattern
// (gloo/examples/example_allreduce.cc, gloo/benchmark/cuda_main.cc:173-214)
// on the MI355X-native surface: N ranks as threads, one GPU each (wrapping
// around the visible GPUs), fp32 sum over device buffers, checked against the
// closed form of gloo/test/base_test.h:184-236.
//
// With "host" as the third argument the inboxes live in pinned host memory
// (HipHostWorkspace, the reference's CudaHostWorkspace placement).
//
//   ./examples/allreduce_ring_chunked [ranks=4] [count=1048576] [device|host]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "gloo_amd/hip_allreduce.h"
#include "gloo_amd/store.h"

int main(int argc, char** argv) {
  const int P = argc > 1 ? std::atoi(argv[1]) : 4;
  const int count = argc > 2 ? std::atoi(argv[2]) : (1 << 20);
  const bool hostWs = argc > 3 && std::string(argv[3]) == "host";
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    std::fprintf(stderr, "no GPU\n");
    return 2;
  }
  auto store = gloo_amd::openStore("mem:example");
  std::vector<int> bad(P, 0);
  std::vector<std::thread> ts;
  for (int r = 0; r < P; r++) {
    ts.emplace_back([&, r] {
      const int dev = r % ndev;
      (void)hipSetDevice(dev);
      auto ctx = std::make_shared<gloo_amd::Context>(r, P);
      ctx->connect(store, dev);
      std::vector<float> host(count);
      for (int j = 0; j < count; j++) host[j] = float(j % 1000) * P + r;
      float* d = nullptr;
      (void)hipMalloc(&d, count * sizeof(float));
      (void)hipMemcpy(d, host.data(), count * sizeof(float), hipMemcpyHostToDevice);
      if (hostWs) {
        gloo_amd::HipAllreduceRingChunked<float, gloo_amd::HipHostWorkspace<float>> algo(ctx, {d}, count);
        algo.run();
      } else {
        gloo_amd::HipAllreduceRingChunked<float> algo(ctx, {d}, count);
        algo.run();
      }
      (void)hipMemcpy(host.data(), d, count * sizeof(float), hipMemcpyDeviceToHost);
      for (int j = 0; j < count; j++) {
        const float want = float(j % 1000) * P * P + P * (P - 1) / 2.0f;
        if (host[j] != want) bad[r]++;
      }
      (void)hipFree(d);
    });
  }
  for (auto& t : ts) t.join();
  int total = 0;
  for (int r = 0; r < P; r++) total += bad[r];
  std::printf("allreduce_ring_chunked: %d ranks x %d floats (%s workspace): %s\n", P, count,
              hostWs ? "host" : "device", total ? "MISMATCH" : "ok");
  return total ? 1 : 0;
}

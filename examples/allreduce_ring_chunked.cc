// examples/allreduce_ring_chunked.cc — the reference's usage pattern
// (gloo/examples/example_allreduce.cc, gloo/benchmark/cuda_main.cc:173-214)
// on the MI355X-native surface: N ranks as threads, one GPU each (wrapping
// around the visible GPUs), fp32 sum over device buffers, checked against the
// closed form of gloo/test/base_test.h:184-236.  After the ring-chunked
// allreduce the same check runs for halving-doubling (the reference's
// constructor signature) and the new-style BCUBE allreduce and reduce.
//
// With "host" as the third argument the inboxes live in pinned host memory
// (HipHostWorkspace, the reference's CudaHostWorkspace placement).
//
//   ./examples/allreduce_ring_chunked [ranks=4] [count=1048576] [device|host]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>
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
  // the framework's allocation mutex (gloo::CudaShared::setMutex, gloo/cuda.h:40-54)
  static std::mutex frameworkAllocMutex;
  gloo_amd::HipShared::setMutex(&frameworkAllocMutex);
  auto store = gloo_amd::openStore("mem:example");
  std::vector<int> bad(P, 0);
  std::vector<std::thread> ts;
  for (int r = 0; r < P; r++) {
    ts.emplace_back([&, r] {
      const int dev = r % ndev;
      (void)hipSetDevice(dev);
      auto ctx = std::make_shared<gloo_amd::Context>(r, P);
      ctx->connect(store, dev);
      std::vector<float> init(count), host(count);
      for (int j = 0; j < count; j++) init[j] = float(j % 1000) * P + r;
      float* d = nullptr;
      float* o = nullptr;
      (void)hipMalloc(&d, count * sizeof(float));
      (void)hipMalloc(&o, count * sizeof(float));
      auto load = [&] { (void)hipMemcpy(d, init.data(), count * sizeof(float), hipMemcpyHostToDevice); };
      auto verify = [&](const float* p) {
        (void)hipMemcpy(host.data(), p, count * sizeof(float), hipMemcpyDeviceToHost);
        for (int j = 0; j < count; j++) {
          const float want = float(j % 1000) * P * P + P * (P - 1) / 2.0f;
          if (host[j] != want) bad[r]++;
        }
      };
      load();
      if (hostWs) {
        gloo_amd::HipAllreduceRingChunked<float, gloo_amd::HipHostWorkspace<float>> algo(ctx, {d}, count);
        algo.run();
      } else {
        gloo_amd::HipAllreduceRingChunked<float> algo(ctx, {d}, count);
        algo.run();
      }
      verify(d);
      // the reference's HD signature (streams, pipelineBroadcastAndReduce)
      load();
      {
        gloo_amd::HipAllreduceHalvingDoubling<float> hd(ctx, {d}, count, {}, true);
        hd.run();
      }
      verify(d);
      // new-style gloo::allreduce(opts) with BCUBE, separate input and output
      load();
      {
        gloo_amd::AllreduceOptions opts(ctx);
        opts.setInput(d, count);
        opts.setOutput(o, count);
        opts.setAlgorithm(gloo_amd::AllreduceOptions::Algorithm::BCUBE);
        opts.setReduceFunction(gloo_amd::SUM);
        gloo_amd::allreduce(opts);
      }
      verify(o);
      // new-style gloo::reduce(opts) to rank P-1
      {
        gloo_amd::ReduceOptions opts(ctx);
        opts.setInput(d, count);
        opts.setOutput(o, count);
        opts.setRoot(P - 1);
        opts.setReduceFunction(gloo_amd::SUM);
        gloo_amd::reduce(opts);
      }
      if (r == P - 1) verify(o);
      (void)hipFree(o);
      (void)hipFree(d);
    });
  }
  for (auto& t : ts) t.join();
  int total = 0;
  for (int r = 0; r < P; r++) total += bad[r];
  std::printf("ring_chunked, halving_doubling, bcube, reduce: %d ranks x %d floats (%s workspace): %s\n", P, count,
              hostWs ? "host" : "device", total ? "MISMATCH" : "ok");
  return total ? 1 : 0;
}

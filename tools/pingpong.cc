// tools/pingpong.cc — measurement tool (not part of the product): the cost of
// one cross-rank hop of the executor's device-side signalling, by placement
// of the flag word.  Two rank processes on the visible GPU(s) bounce a
// sequence number K times inside one captured hipGraph (replayed R times):
//   host    the flag lives in the node's shared control block (pinned host
//           memory, hipHostRegister) — where the executor keeps it today;
//   device  the flag lives in the RECEIVER's fine-grained device memory,
//           shared by HIP IPC: the sender writes it remotely, the receiver
//           polls its own HBM.
// and by kernel shape:
//   split   signal kernel + wait kernel per hop and rank (the executor's
//           WAIT / NOTIFY steps);
//   fused   one kernel that waits, then signals (the fused small step).
// Prints one JSON line per rank: microseconds per round trip (two hops).
//
//   pingpong <rank> <store-url> <host|device> <split|fused> [K=2000] [R=5]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gloo_amd.h"
#include "gloo_amd/common.h"
#include "gloo_amd/context.h"
#include "gloo_amd/signal.h"
#include "gloo_amd/store.h"

using namespace gloo_amd;

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: pingpong rank store host|device split|fused [K] [R]\n");
    return 2;
  }
  const int rank = std::atoi(argv[1]);
  const std::string url = argv[2], place = argv[3], shape = argv[4];
  const int K = argc > 5 ? std::atoi(argv[5]) : 2000;
  const int R = argc > 6 ? std::atoi(argv[6]) : 5;
  int ndev = 0;
  GLOO_AMD_HIP_CHECK(hipGetDeviceCount(&ndev));
  const int dev = rank % ndev;
  GLOO_AMD_HIP_CHECK(hipSetDevice(dev));
  auto ctx = std::make_shared<Context>(rank, 2, std::chrono::seconds(60));
  ctx->connect(openStore(url), dev);
  const int peer = 1 - rank;

  // inbox[r] = the flag rank r waits on
  uint64_t* inbox[2] = {nullptr, nullptr};
  uint64_t* mine = nullptr;
  void* peerMapped = nullptr;
  if (place == "host") {
    inbox[0] = ctx->counterDevicePtr(Context::kMaxLiveInstances - 1, 1, 0, 0);
    inbox[1] = ctx->counterDevicePtr(Context::kMaxLiveInstances - 1, 0, 1, 0);
  } else {
    GLOO_AMD_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&mine), 4096, hipDeviceMallocFinegrained));
    GLOO_AMD_HIP_CHECK(hipMemset(mine, 0, 4096));
    GLOO_AMD_HIP_CHECK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    GLOO_AMD_HIP_CHECK(hipIpcGetMemHandle(&h, mine));
    std::vector<char> blob(sizeof(h));
    std::memcpy(blob.data(), &h, sizeof(h));
    ctx->store().set("pingpong/" + std::to_string(rank), blob);
    auto v = ctx->store().get("pingpong/" + std::to_string(peer), std::chrono::seconds(60));
    std::memcpy(&h, v.data(), sizeof(h));
    GLOO_AMD_HIP_CHECK(hipIpcOpenMemHandle(&peerMapped, h, hipIpcMemLazyEnablePeerAccess));
    inbox[rank] = mine;
    inbox[peer] = static_cast<uint64_t*>(peerMapped);
  }
  uint64_t* epoch = nullptr;
  GLOO_AMD_HIP_CHECK(hipMalloc(&epoch, sizeof(uint64_t)));
  GLOO_AMD_HIP_CHECK(hipMemset(epoch, 0, sizeof(uint64_t)));
  uint32_t* err = ctx->errorWordDevicePtr(rank);
  const uint64_t ticks = 2ull * 100000000ull;  // 2 s of the 100 MHz clock
  hipStream_t s;
  GLOO_AMD_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  GLOO_AMD_HIP_CHECK(hipDeviceSynchronize());
  ctx->barrier("ready");

  // Round i (1..K) of replay e has value i + e*K: rank 0 signals it to
  // rank 1 and waits for rank 1's echo of it.
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  GLOO_AMD_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  GLOO_AMD_HIP_CHECK(launchEpochBump(epoch, s));
  for (int i = 1; i <= K; i++) {
    const Seq v{(uint64_t)i, (uint64_t)K};
    if (shape == "split") {
      if (rank == 0) {
        GLOO_AMD_HIP_CHECK(launchSignal(inbox[1], v, epoch, s));
        GLOO_AMD_HIP_CHECK(launchWait(inbox[0], v, epoch, ticks, err, s));
      } else {
        GLOO_AMD_HIP_CHECK(launchWait(inbox[1], v, epoch, ticks, err, s));
        GLOO_AMD_HIP_CHECK(launchSignal(inbox[0], v, epoch, s));
      }
    } else {
      if (rank == 0) {
        // signal round i; the wait for round i is fused with the signal of i+1
        if (i == 1) GLOO_AMD_HIP_CHECK(launchSignal(inbox[1], v, epoch, s));
        const Seq next{(uint64_t)i + 1, (uint64_t)K};
        if (i < K) {
          if (launchFusedSmall(0, GLOO_HIP_F32, nullptr, nullptr, 0, inbox[0], v, ticks, err, inbox[1], next, epoch,
                               s) != GLOO_HIP_OK)
            throw EnforceNotMet("fused launch");
        } else {
          GLOO_AMD_HIP_CHECK(launchWait(inbox[0], v, epoch, ticks, err, s));
        }
      } else {
        if (launchFusedSmall(0, GLOO_HIP_F32, nullptr, nullptr, 0, inbox[1], v, ticks, err, inbox[0], v, epoch, s) !=
            GLOO_HIP_OK)
          throw EnforceNotMet("fused launch");
      }
    }
  }
  GLOO_AMD_HIP_CHECK(hipStreamEndCapture(s, &g));
  GLOO_AMD_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  std::vector<double> us;
  for (int r = 0; r < R; r++) {
    ctx->barrier("rep" + std::to_string(r));
    const auto t0 = std::chrono::steady_clock::now();
    GLOO_AMD_HIP_CHECK(hipGraphLaunch(ge, s));
    GLOO_AMD_HIP_CHECK(hipStreamSynchronize(s));
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    us.push_back(dt * 1e6 / K);
  }
  const bool timedOut = ctx->errorWord(rank).load() != 0;
  double best = us[0];
  for (double x : us) best = x < best ? x : best;
  std::printf("{\"rank\": %d, \"flags\": \"%s\", \"kernels\": \"%s\", \"K\": %d, \"us_per_round_trip_best\": %.3f, "
              "\"us_per_round_trip\": [", rank, place.c_str(), shape.c_str(), K, best);
  for (size_t i = 0; i < us.size(); i++) std::printf("%s%.3f", i ? ", " : "", us[i]);
  std::printf("], \"timed_out\": %s}\n", timedOut ? "true" : "false");
  ctx->barrier("done");
  GLOO_AMD_HIP_CHECK(hipGraphExecDestroy(ge));
  GLOO_AMD_HIP_CHECK(hipGraphDestroy(g));
  if (peerMapped) GLOO_AMD_HIP_CHECK(hipIpcCloseMemHandle(peerMapped));
  ctx->barrier("closed");
  if (mine) GLOO_AMD_HIP_CHECK(hipFree(mine));
  return timedOut ? 1 : 0;
}

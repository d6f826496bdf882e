// stale_line_probe.hip — MEASUREMENT / DIAGNOSIS ONLY: the mechanism of
// GPUTEST_r05's red BCUBE case, reduced to one buffer.
//
// A ranks-as-threads collective on one GPU moves a message like this: the
// receiver's kernels read its inbox (stream R), the sender's copy overwrites
// the inbox (stream S), the host sees the sender's arrival counter, then the
// receiver's next kernel reads the inbox again (stream R).  Here, per trial:
//   1. `reader` on stream R: 2048 workgroups (every XCD) read the whole inbox
//      (its lines may now sit in every XCD's L2);
//   2. the inbox is overwritten with this trial's pattern on stream S, by
//      hipMemcpyAsync (the thread route's SEND) or by a copy kernel;
//   3. hipStreamSynchronize(S) on the host (the counter bump);
//   4. `checker` on stream R: 2048 workgroups each compare the whole inbox with
//      the pattern and count mismatching words.
// Inboxes: plain hipMalloc (coarse-grained, the thread route's arena before
// round 6) and hipExtMallocWithFlags fine-grained (every route's now).
// One JSON line per (inbox, writer): trials, trials with any stale word,
// stale words.   stale_line_probe [trials] [bytes]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CHECK(x)                                                                                       \
  do {                                                                                                 \
    hipError_t e_ = (x);                                                                               \
    if (e_ != hipSuccess) {                                                                            \
      std::printf("{\"fatal\": \"%s:%d %s: %s\"}\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                                    \
    }                                                                                                  \
  } while (0)

__global__ void reader(const uint32_t* p, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) acc += p[i];
  if (acc == 0xdeadbeefu) sink[0] = acc;  // keeps the loads
}

__global__ void writer(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v ^ (uint32_t)i;
}

__global__ void checker(const uint32_t* p, size_t n, uint32_t v, unsigned long long* bad) {
  unsigned c = 0;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) c += p[i] != (v ^ (uint32_t)i);
  if (c) atomicAdd(bad, (unsigned long long)c);
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? std::atoi(argv[1]) : 2000;
  const size_t bytes = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 4096;
  const size_t n = bytes / 4;
  CHECK(hipSetDevice(0));
  hipStream_t R, S;
  CHECK(hipStreamCreateWithFlags(&R, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
  uint32_t* src;
  uint32_t* sink;
  unsigned long long* bad;
  CHECK(hipMalloc(&src, bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&bad), sizeof(*bad), hipHostMallocCoherent | hipHostMallocMapped));
  for (const char* kind : {"coarse", "fine"}) {
    uint32_t* inbox;
    if (std::string(kind) == "coarse") {
      CHECK(hipMalloc(&inbox, bytes));
    } else {
      CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&inbox), bytes, hipDeviceMallocFinegrained));
    }
    for (const char* how : {"memcpy", "kernel"}) {
      long staleTrials = 0;
      unsigned long long staleWords = 0;
      for (int t = 0; t < trials; t++) {
        const uint32_t v = 0x9e3779b9u * (uint32_t)(t + 1) + (std::string(how) == "kernel" ? 7u : 0u);
        // the pattern in src, complete before anything below
        writer<<<64, 256, 0, S>>>(src, n, v);
        CHECK(hipStreamSynchronize(S));
        reader<<<2048, 256, 0, R>>>(inbox, n, sink);
        CHECK(hipStreamSynchronize(R));
        if (std::string(how) == "memcpy") {
          CHECK(hipMemcpyAsync(inbox, src, bytes, hipMemcpyDeviceToDevice, S));
        } else {
          writer<<<64, 256, 0, S>>>(inbox, n, v);
        }
        CHECK(hipStreamSynchronize(S));
        *bad = 0;
        checker<<<2048, 256, 0, R>>>(inbox, n, v, bad);
        CHECK(hipStreamSynchronize(R));
        if (*bad) {
          staleTrials++;
          staleWords += *bad;
        }
      }
      std::printf("{\"inbox\": \"%s\", \"writer\": \"%s\", \"bytes\": %zu, \"trials\": %d, \"stale_trials\": %ld, "
                  "\"stale_words_seen\": %llu}\n", kind, how, bytes, trials, staleTrials, staleWords);
      std::fflush(stdout);
    }
    CHECK(hipFree(inbox));
  }
  return 0;
}

// stale_busy_probe.hip — MEASUREMENT / DIAGNOSIS ONLY: GPUTEST_r05's red BCUBE
// case with the thread route's exact ordering, which
// `stale_line_probe` simplifies away.  On that route a rank's fold is launched
// onto a stream that is still BUSY (its earlier sends and credits are queued),
// the sender's copy runs on another rank's stream, and the receiver learns of
// the copy from a host function on the sender's stream (a counter bump), not
// from a stream synchronise.  Per trial, on a small inbox (the BCUBE case's
// region is 20 bytes):
//   R: reader (16 workgroups, every XCD caches the inbox) ; host function A ; spin
//   host: wait A ; S: copy of this trial's pattern into the inbox (memcpy or
//         kernel) ; host function B ; wait B
//   R: checker (16 workgroups, each reads it all), queued behind the spin when `busy`.
// With `streams` > 2, that many extra streams are created first and each gets
// one kernel, so R and S share hardware queues (GPU_MAX_HW_QUEUES is 4).
// One JSON line per (inbox, writer, busy, streams): trials with a stale word.
//   stale_busy_probe [trials] [bytes]
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

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
  if (acc == 0xdeadbeefu) sink[0] = acc;
}

__global__ void writer(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v ^ (uint32_t)i;
}

__global__ void spin(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

__global__ void checker(const uint32_t* p, size_t n, uint32_t v, unsigned* bad) {
  unsigned c = 0;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) c += p[i] != (v ^ (uint32_t)i);
  if (c) atomicAdd(bad, c);
}

static void setFlag(void* p) { static_cast<std::atomic<int>*>(p)->store(1, std::memory_order_release); }

static void waitFlag(std::atomic<int>& f) {
  while (!f.load(std::memory_order_acquire)) std::this_thread::yield();
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? std::atoi(argv[1]) : 2000;
  const size_t bytes = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 256;
  const size_t n = bytes / 4;
  CHECK(hipSetDevice(0));
  uint32_t *src, *sink;
  unsigned* bad;
  CHECK(hipMalloc(&src, bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&bad), 64, hipHostMallocCoherent | hipHostMallocMapped));
  for (int streams : {2, 16}) {
    std::vector<hipStream_t> extra;
    for (int i = 2; i < streams; i++) {
      hipStream_t x;
      CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
      spin<<<1, 64, 0, x>>>(100);
      extra.push_back(x);
    }
    hipStream_t R, S;
    CHECK(hipStreamCreateWithFlags(&R, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
    for (const char* kind : {"coarse", "fine"}) {
      uint32_t* inbox;
      if (std::string(kind) == "coarse") {
        CHECK(hipMalloc(&inbox, bytes));
      } else {
        CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&inbox), bytes, hipDeviceMallocFinegrained));
      }
      for (const char* how : {"memcpy", "kernel"}) {
        for (int busy : {0, 1}) {
          long stale = 0;
          for (int t = 0; t < trials; t++) {
            const uint32_t v = 0x9e3779b9u * (uint32_t)(t + 1) + (std::string(how) == "kernel" ? 7u : 0u);
            writer<<<1, 64, 0, S>>>(src, n, v);
            CHECK(hipStreamSynchronize(S));
            *bad = 0;
            std::atomic<int> a{0}, b{0};
            reader<<<16, 64, 0, R>>>(inbox, n, sink);
            CHECK(hipLaunchHostFunc(R, setFlag, &a));
            if (busy) spin<<<1, 64, 0, R>>>(2000);  // 20 us
            waitFlag(a);
            if (std::string(how) == "memcpy") {
              CHECK(hipMemcpyAsync(inbox, src, bytes, hipMemcpyDeviceToDevice, S));
            } else {
              writer<<<1, 64, 0, S>>>(inbox, n, v);
            }
            CHECK(hipLaunchHostFunc(S, setFlag, &b));
            waitFlag(b);
            checker<<<16, 64, 0, R>>>(inbox, n, v, bad);
            CHECK(hipStreamSynchronize(R));
            if (*bad) stale++;
          }
          std::printf("{\"inbox\": \"%s\", \"writer\": \"%s\", \"busy\": %d, \"streams\": %d, \"bytes\": %zu, "
                      "\"trials\": %d, \"stale_trials\": %ld}\n", kind, how, busy, streams, bytes, trials, stale);
          std::fflush(stdout);
        }
      }
      CHECK(hipFree(inbox));
    }
    CHECK(hipStreamDestroy(R));
    CHECK(hipStreamDestroy(S));
    for (auto x : extra) CHECK(hipStreamDestroy(x));
  }
  return 0;
}

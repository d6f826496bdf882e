// hostfn_order_probe.hip — MEASUREMENT / DIAGNOSIS ONLY: does a stream host
// function (hipLaunchHostFunc) run only after the kernels queued before it
// on its stream have finished?  The host-signalled executor route (ranks as
// threads sharing a GPU) publishes its credits that way: a NOTIFY after a
// fold is a host function, and the peer that sees it overwrites the inbox
// the fold read.  If the function ran early, the fold would read the peer's
// next message (GPUTEST_r05's red BCUBE case would look exactly like that).
// Per trial: a one-wave kernel spins for ~`spin_us`, then reads x[0] into
// out; a host function queued behind it on the same stream sets a flag; the
// host thread, on the flag, overwrites x from another stream and waits for
// that copy.  If the kernel read the NEW value the host function ran before
// the kernel was done.  One JSON line per spin length.  Last line: does
// hipStreamSynchronize (and an event recorded behind the host function) return
// only after a slow host function has returned?  (Executor release and
// context close rely on it: a credit's host function writes the context's
// control block.)
//   hostfn_order_probe [trials] [spin_us...]
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
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

__global__ void spin_then_read(const uint32_t* x, uint32_t* out, uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0) out[0] = x[0];
}

static void setFlag(void* p) { static_cast<std::atomic<int>*>(p)->store(1, std::memory_order_release); }
static void slowSetFlag(void* p) {
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  setFlag(p);
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? std::atoi(argv[1]) : 500;
  std::vector<int> spins;
  for (int i = 2; i < argc; i++) spins.push_back(std::atoi(argv[i]));
  if (spins.empty()) spins = {5, 20, 100};
  CHECK(hipSetDevice(0));
  hipStream_t R, S;
  CHECK(hipStreamCreateWithFlags(&R, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
  uint32_t *x, *out, *fresh;
  CHECK(hipMalloc(&x, 4096));
  CHECK(hipMalloc(&fresh, 4096));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&out), 64, hipHostMallocCoherent | hipHostMallocMapped));
  for (int spin : spins) {
    int early = 0;
    double waitUs = 0;
    for (int t = 0; t < trials; t++) {
      const uint32_t oldv = 2 * t + 1, newv = 2 * t + 2;
      CHECK(hipMemcpy(x, &oldv, 4, hipMemcpyHostToDevice));
      CHECK(hipMemcpy(fresh, &newv, 4, hipMemcpyHostToDevice));
      out[0] = 0;
      std::atomic<int> flag{0};
      spin_then_read<<<1, 64, 0, R>>>(x, out, (uint64_t)spin * 100);
      CHECK(hipLaunchHostFunc(R, setFlag, &flag));
      const auto t0 = std::chrono::steady_clock::now();
      while (!flag.load(std::memory_order_acquire)) std::this_thread::yield();
      waitUs += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      CHECK(hipMemcpyAsync(x, fresh, 4, hipMemcpyDeviceToDevice, S));
      CHECK(hipStreamSynchronize(S));
      CHECK(hipStreamSynchronize(R));
      if (out[0] == newv) early++;
      else if (out[0] != oldv) {
        std::printf("{\"fatal\": \"read %u, neither %u nor %u\"}\n", out[0], oldv, newv);
        return 3;
      }
    }
    std::printf("{\"spin_us\": %d, \"trials\": %d, \"host_function_before_kernel_end\": %d, "
                "\"mean_wait_for_host_function_us\": %.1f}\n", spin, trials, early, waitUs / trials);
    std::fflush(stdout);
  }
  int syncEarly = 0, eventEarly = 0;
  const int slowTrials = 20;
  for (int t = 0; t < slowTrials; t++) {
    std::atomic<int> f1{0}, f2{0};
    spin_then_read<<<1, 64, 0, R>>>(x, out, 200);
    CHECK(hipLaunchHostFunc(R, slowSetFlag, &f1));
    CHECK(hipStreamSynchronize(R));
    if (!f1.load(std::memory_order_acquire)) syncEarly++;
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CHECK(hipLaunchHostFunc(R, slowSetFlag, &f2));
    CHECK(hipEventRecord(ev, R));
    CHECK(hipEventSynchronize(ev));
    if (!f2.load(std::memory_order_acquire)) eventEarly++;
    CHECK(hipStreamSynchronize(R));
    CHECK(hipEventDestroy(ev));
  }
  std::printf("{\"slow_host_function_ms\": 20, \"trials\": %d, \"stream_sync_returned_before_it\": %d, "
              "\"event_sync_returned_before_it\": %d}\n", slowTrials, syncEarly, eventEarly);
  return 0;
}

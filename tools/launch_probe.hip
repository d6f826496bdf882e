// launch_probe.hip — what a small collective's host side costs on this box,
// and what a persistent interpreter fed through stream memory operations
// would cost instead (DESIGN.md §8 "Remaining").  One process, one GPU.
// Prints one JSON line per measurement: p50 / p90 in µs over ITERS rounds.
//
//   launch_sync     one-wave nop kernel + hipStreamSynchronize
//   launch_enqueue  the host time of that launch alone
//   launch_query    the launch, then hipStreamQuery spun until the stream is idle
//   launch_event    the launch + hipEventRecord, then hipEventQuery spun
//   launch_flag     a kernel that stores a flag into coherent host memory, the
//                   host spinning on the flag (then a non-blocking stream query)
//   write_sync      hipStreamWriteValue64 + hipStreamSynchronize
//   wait_sync       hipStreamWaitValue64 (already met) + hipStreamSynchronize
//   persistent_ops  a resident one-workgroup kernel on another stream polls a
//                   doorbell; per round the host enqueues WriteValue(door, i)
//                   and WaitValue(done >= i) on its stream and synchronises it
//   persistent_host the same kernel, the host writing the doorbell and polling
//                   `done` itself (no HIP call per round: the floor)
//
// The resident kernel leaves its loop on a quit value or after a wall-clock
// bound (wall_clock64, 100 MHz), whichever comes first, so the grid always
// drains.  Stores are vector (global) atomics.
//   launch_probe [ITERS]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

constexpr uint64_t kQuit = ~uint64_t(0);

__global__ void nop_kernel() {}

__global__ void flag_kernel(uint64_t* flag, uint64_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void resident_kernel(const uint64_t* door, uint64_t* done, uint64_t maxTicks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  uint64_t seen = 0;
  for (;;) {
    const uint64_t d = __hip_atomic_load(door, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (d == kQuit) break;
    if (d != seen) {
      seen = d;
      __hip_atomic_store(done, d, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (wall_clock64() - t0 > maxTicks) break;
    __builtin_amdgcn_s_sleep(1);
  }
}

using Clock = std::chrono::steady_clock;

static void report(const char* what, std::vector<double>& us) {
  std::sort(us.begin(), us.end());
  std::printf("{\"measure\": \"%s\", \"rounds\": %zu, \"us_p50\": %.2f, \"us_p90\": %.2f, \"us_min\": %.2f}\n", what,
              us.size(), us[us.size() / 2], us[us.size() * 9 / 10], us[0]);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  // launch_probe ITERS spin: hipDeviceScheduleSpin (host waits spin instead of yielding)
  if (argc > 2 && std::string(argv[2]) == "spin") CHECK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  CHECK(hipSetDevice(0));
  int canWait = 0;
  CHECK(hipDeviceGetAttribute(&canWait, hipDeviceAttributeCanUseStreamWaitValue, 0));
  std::printf("{\"can_use_stream_wait_value\": %d}\n", canWait);
  hipStream_t s, r;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&r, hipStreamNonBlocking));
  // the doorbell in fine-grained device memory, `done` in coherent pinned host memory
  uint64_t* door = nullptr;
  CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&door), 64, hipDeviceMallocFinegrained));
  CHECK(hipMemset(door, 0, 64));
  uint64_t* done = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&done), 64, hipHostMallocCoherent | hipHostMallocMapped));
  *done = 0;
  uint64_t* hdoor = nullptr;  // a host-memory doorbell for persistent_host
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&hdoor), 64, hipHostMallocCoherent | hipHostMallocMapped));
  *hdoor = 0;
  CHECK(hipDeviceSynchronize());
  std::vector<double> a, b;

  for (int i = 0; i < 100; i++) nop_kernel<<<1, 64, 0, s>>>();
  CHECK(hipStreamSynchronize(s));
  for (int i = 0; i < iters; i++) {
    const auto t0 = Clock::now();
    nop_kernel<<<1, 64, 0, s>>>();
    const auto t1 = Clock::now();
    CHECK(hipStreamSynchronize(s));
    const auto t2 = Clock::now();
    a.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
    b.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  report("launch_sync", a);
  report("launch_enqueue", b);

  // the same with a second stream of this process that ran one kernel and is idle now
  nop_kernel<<<1, 64, 0, r>>>();
  CHECK(hipStreamSynchronize(r));
  a.clear();
  for (int i = 0; i < iters; i++) {
    const auto t0 = Clock::now();
    nop_kernel<<<1, 64, 0, s>>>();
    CHECK(hipStreamSynchronize(s));
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  report("launch_sync_second_stream_idle", a);
  // ... and alternating launches between the two streams, each synchronised
  a.clear();
  for (int i = 0; i < iters; i++) {
    hipStream_t x = (i & 1) ? r : s;
    const auto t0 = Clock::now();
    nop_kernel<<<1, 64, 0, x>>>();
    CHECK(hipStreamSynchronize(x));
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  report("launch_sync_alternating_streams", a);

  a.clear();
  for (int i = 0; i < iters; i++) {
    const auto t0 = Clock::now();
    nop_kernel<<<1, 64, 0, s>>>();
    hipError_t q;
    while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    CHECK(q);
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  report("launch_query", a);

  hipEvent_t ev;
  CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  a.clear();
  for (int i = 0; i < iters; i++) {
    const auto t0 = Clock::now();
    nop_kernel<<<1, 64, 0, s>>>();
    CHECK(hipEventRecord(ev, s));
    hipError_t q;
    while ((q = hipEventQuery(ev)) == hipErrorNotReady) {
    }
    CHECK(q);
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  report("launch_event", a);

  a.clear();
  *done = 0;
  for (int i = 0; i < iters; i++) {
    const uint64_t v = (uint64_t)i + 1;
    const auto t0 = Clock::now();
    flag_kernel<<<1, 64, 0, s>>>(done, v);
    const auto dl = Clock::now() + std::chrono::seconds(5);
    while (__atomic_load_n(done, __ATOMIC_ACQUIRE) < v) {
      if (Clock::now() > dl) {
        std::fprintf(stderr, "flag never arrived\n");
        return 3;
      }
    }
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  CHECK(hipStreamSynchronize(s));
  report("launch_flag", a);

  a.clear();
  for (int i = 0; i < iters; i++) {
    const auto t0 = Clock::now();
    CHECK(hipStreamWriteValue64(s, door, (uint64_t)i + 1, 0));
    CHECK(hipStreamSynchronize(s));
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  report("write_sync", a);

  a.clear();
  *done = ~uint64_t(0) >> 1;
  for (int i = 0; i < iters; i++) {
    const auto t0 = Clock::now();
    CHECK(hipStreamWaitValue64(s, done, (uint64_t)i + 1, hipStreamWaitValueGte));
    CHECK(hipStreamSynchronize(s));
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  report("wait_sync", a);

  // persistent_ops: the resident kernel on stream r, bounded to 30 s
  CHECK(hipMemset(door, 0, 64));
  *done = 0;
  CHECK(hipDeviceSynchronize());
  resident_kernel<<<1, 64, 0, r>>>(door, done, 30ull * 100000000ull);
  CHECK(hipGetLastError());
  a.clear();
  bool ok = true;
  for (int i = 0; i < iters && ok; i++) {
    const uint64_t v = (uint64_t)i + 1;
    const auto t0 = Clock::now();
    CHECK(hipStreamWriteValue64(s, door, v, 0));
    CHECK(hipStreamWaitValue64(s, done, v, hipStreamWaitValueGte));
    CHECK(hipStreamSynchronize(s));
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    if (a.back() > 2e6) ok = false;  // the resident kernel is gone
  }
  CHECK(hipStreamWriteValue64(s, door, kQuit, 0));
  CHECK(hipStreamSynchronize(s));
  CHECK(hipStreamSynchronize(r));
  if (ok) report("persistent_ops", a);

  // persistent_host: the doorbell in host memory, written and polled by the host
  *hdoor = 0;
  *done = 0;
  resident_kernel<<<1, 64, 0, r>>>(hdoor, done, 30ull * 100000000ull);
  CHECK(hipGetLastError());
  a.clear();
  const auto deadline = Clock::now() + std::chrono::seconds(20);
  for (int i = 0; i < iters && ok; i++) {
    const uint64_t v = (uint64_t)i + 1;
    const auto t0 = Clock::now();
    __atomic_store_n(hdoor, v, __ATOMIC_RELEASE);
    while (__atomic_load_n(done, __ATOMIC_ACQUIRE) < v) {
      if (Clock::now() > deadline) {
        ok = false;
        break;
      }
    }
    a.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  __atomic_store_n(hdoor, kQuit, __ATOMIC_RELEASE);
  CHECK(hipStreamSynchronize(r));
  if (ok) report("persistent_host", a);

  CHECK(hipFree(door));
  CHECK(hipHostFree(done));
  CHECK(hipHostFree(hdoor));
  return ok ? 0 : 3;
}

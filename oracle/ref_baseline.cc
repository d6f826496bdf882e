// ref_baseline.cc — ORACLE / MEASUREMENT INFRASTRUCTURE ONLY (bench.py's
// `cpu_baseline` leg).  Times the reference's own gloo::sum<float>
// (gloo/math.h:15-28) compiled from /root/reference exactly as the reference
// ships it (-O3 -DNDEBUG, no -march), in its own .so so no
// differently-flagged instantiation of the template can be picked by the
// linker.  Gloo calls it single-threaded; `nthreads` > 1 partitions the range
// over std::threads for the all-cores figure.
#include <thread>
#include <vector>

#include "gloo/math.h"

namespace {

template <typename F>
void split(size_t n, int nthreads, F&& fn) {
  if (nthreads <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const size_t per = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; t++) {
    const size_t lo = per * t;
    if (lo >= n) break;
    const size_t len = (lo + per > n) ? n - lo : per;
    ts.emplace_back([=] { fn(lo, len); });
  }
  for (auto& t : ts) t.join();
}

}  // namespace

extern "C" {

// The 3-operand form gloo::sum<T>(void* c, const void* a, const void* b,
// size_t n) (gloo/math.h:15-23); c may alias a.
void ref_base_sum_f32(float* c, const float* a, const float* b, size_t n, int nthreads) {
  split(n, nthreads, [=](size_t lo, size_t len) { gloo::sum<float>(c + lo, a + lo, b + lo, len); });
}

// The in-place 2-operand form gloo::sum<T>(T* a, const T* b, size_t n)
// (gloo/math.h:25-28), the pointer ReductionFunction<T>::sum holds
// (gloo/algorithm.h:84-86).
void ref_base_sum2_f32(float* a, const float* b, size_t n, int nthreads) {
  split(n, nthreads, [=](size_t lo, size_t len) { gloo::sum<float>(a + lo, b + lo, len); });
}

}  // extern "C"

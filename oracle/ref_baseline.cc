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

extern "C" {

void ref_base_sum_f32(float* c, const float* a, const float* b, size_t n, int nthreads) {
  if (nthreads <= 1) {
    gloo::sum<float>(c, a, b, n);
    return;
  }
  std::vector<std::thread> ts;
  const size_t per = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; t++) {
    const size_t lo = per * t;
    if (lo >= n) break;
    const size_t len = (lo + per > n) ? n - lo : per;
    ts.emplace_back([=] { gloo::sum<float>(c + lo, a + lo, b + lo, len); });
  }
  for (auto& t : ts) t.join();
}

}  // extern "C"

// plan.h — per-rank schedules (see include/gloo_amd.h "Schedules").
#pragma once

#include <cstdint>
#include <vector>

#include "gloo_amd.h"

namespace gloo_amd {

using Step = gloo_hip_step_t;

struct Plan {
  std::vector<Step> steps;
  uint64_t arena = 0;  // inbox arena, elements
};

// Build rank `rank`'s plan.  recvElems: reduce-scatter only.
Plan makePlan(int algo, int rank, int size, uint64_t count, int nptrs,
              const std::vector<int>& recvElems = {});

// New-style collective parameters (gloo/allreduce.h:89-193, gloo/reduce.h:19-110).
struct NewStyleOptions {
  int ninputs = 0;
  int noutputs = 1;
  size_t elemSize = 4;
  size_t maxSegmentBytes = 1024 * 1024;  // kMaxSegmentSize, gloo/allreduce.h:78, gloo/reduce.h:98
  int root = 0;                          // gloo::reduce only (ReduceOptions::setRoot)
};
// algo: GLOO_HIP_ALGO_ALLREDUCE_RING, GLOO_HIP_ALGO_ALLREDUCE_BCUBE or
// GLOO_HIP_ALGO_REDUCE, optionally | GLOO_HIP_ALGO_MESH (mesh.h).
Plan makeNewStylePlan(int algo, int rank, int size, uint64_t count, const NewStyleOptions& o);
inline bool isNewStyle(int algo) {
  algo &= ~GLOO_HIP_ALGO_MESH;
  return algo == GLOO_HIP_ALGO_ALLREDUCE_RING || algo == GLOO_HIP_ALGO_ALLREDUCE_BCUBE ||
         algo == GLOO_HIP_ALGO_REDUCE;
}

}  // namespace gloo_amd

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

// New-style allreduce parameters (gloo/allreduce.h:89-193).
struct NewStyleOptions {
  int ninputs = 0;
  int noutputs = 1;
  size_t elemSize = 4;
  size_t maxSegmentBytes = 1024 * 1024;  // kMaxSegmentSize, gloo/allreduce.h:78
};
Plan makeAllreducePlan(int rank, int size, uint64_t count, const NewStyleOptions& o);

}  // namespace gloo_amd

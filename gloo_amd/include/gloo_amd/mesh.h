// mesh.h — a reference schedule's result with mesh data movement.
//
// makeMeshPlan(algo, ...) runs every rank's plan of `algo` (plan.h)
// symbolically, finds the expression tree the reference evaluates for each
// output range and the rank that finishes it, and returns rank `rank`'s plan
// that moves raw inputs straight to that rank (every peer at once), evaluates
// the same trees there and, for allreduce, sends the results to every rank.
// Identical trees, identical bits.  Throws when the schedule has no such form
// (e.g. AllreduceRing, whose ranks finish with different association orders).
#pragma once

#include <vector>

#include "gloo_amd/plan.h"

namespace gloo_amd {

// ns: the options of a new-style algorithm (ALLREDUCE_RING, ALLREDUCE_BCUBE,
// REDUCE), nullptr for the class-style ones.
Plan makeMeshPlan(int algo, int rank, int size, uint64_t count, int nptrs, const std::vector<int>& recvElems,
                  const NewStyleOptions* ns = nullptr);

}  // namespace gloo_amd

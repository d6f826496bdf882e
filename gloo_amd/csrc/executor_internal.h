// executor_internal.h — helpers shared by the executor's construction
// (executor.cc) and its runs (executor_run.cc): launch-mode thresholds and
// the sliced interpreter's step splitting (executor_modes.cc).  Internal to
// the library.
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "gloo_amd/plan.h"

namespace gloo_amd {
namespace exec {

// Throws EnforceNotMet naming `what` and gloo_hip_last_error() unless rc is
// GLOO_HIP_OK.
void checkRc(int rc, const char* what);

// Largest message whose wait / body / notify chain is fused into one launch
// (GLOO_AMD_FUSE_BYTES).
size_t fuseBytes();
// Largest message below which GLOO_AMD_GRAPH=auto replays a mesh plan as a
// hipGraph (4 MiB, fixed since round 6).
size_t graphBytes();
// Largest message of a plan the one-launch interpreter runs (0: never).
size_t interpBytes();
// Bytes of the largest message per sliced-interpreter workgroup, and their cap.
size_t sliceBytes();
size_t sliceCapBytes();
// Most workgroups of a sliced launch (<= kMaxSlices).
int maxSlices();
// The slice cap for `ranksHere` ranks sharing `device`: min(maxSlices(),
// its CU count / ranksHere), at least 1.
int coResidentSlices(int device, int ranksHere);
// A GPU's PCI domain / bus / device as one number (the same GPU in every
// process, whatever its device index there).
int64_t gpuLocation(int device);

// A range of one of a rank's buffers, symbolically: output j = j, input j =
// kIn + j, the inbox arena = kArena.
struct Access {
  int buf;
  size_t off, len;
};
constexpr int kIn = 1 << 20, kArena = -1;

// The boundaries the plan's steps use in the user buffers, and [off, off+len)
// cut at them: where the sliced form splits its whole-range local steps.
std::vector<size_t> userCuts(const Plan& plan);
std::vector<std::pair<size_t, size_t>> cutRange(const std::vector<size_t>& cuts, size_t off, size_t len);
// Whether the plan can run as slices, given the ranges peers write into this
// rank's buffers.
bool sliceable(const Plan& plan, int nin, int nout, const std::vector<Access>& remoteWrites);
// Device step-list entries of the plan's sliced form.
size_t slicedInterpSteps(const Plan& plan, int nin, int nout);

}  // namespace exec
}  // namespace gloo_amd

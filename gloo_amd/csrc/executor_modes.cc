// executor_modes.cc — launch-mode thresholds and the sliced interpreter's
// step splitting, shared by executor.cc and executor_run.cc
// (executor_internal.h).
#include <algorithm>
#include <cstdlib>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "executor_internal.h"
#include "gloo_amd.h"
#include "gloo_amd/common.h"
#include "gloo_amd/errors.h"
#include "gloo_amd/signal.h"

namespace gloo_amd {
namespace exec {

void checkRc(int rc, const char* what) {
  if (rc != GLOO_HIP_OK) throw EnforceNotMet(strcat_(what, " failed (", rc, "): ", gloo_hip_last_error()));
}

// Largest message whose wait / body / notify chain is fused into one launch.
size_t fuseBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_FUSE_BYTES");
    return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)(64 << 10);
  }();
  return v;
}

// Largest message below which GLOO_AMD_GRAPH=auto replays a mesh plan as a
// hipGraph (executor constructor); larger mesh plans are enqueued eagerly
// (7-13 % faster than replay at 16 and 64 MiB per rank).
size_t graphBytes() { return size_t(4) << 20; }

// Largest message of a plan the one-launch interpreter runs (0: never): the
// fused-launch size.
size_t interpBytes() { return fuseBytes(); }

// Workgroups per sliced interpreter launch: about one per this many bytes of
// the plan's largest message.
size_t sliceBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_INTERP_SLICE_BYTES");
    return e ? std::max<size_t>(1, std::strtoull(e, nullptr, 10)) : (size_t)(32 << 10);
  }();
  return v;
}

// Most bytes of the largest message per slice: above maxSlices() slices of
// sliceBytes() the slices grow up to this, so plans with messages up to
// maxSlices() x this run sliced (2 MiB with the defaults).  Measured, HD
// fp32 4 MiB per rank, 2 rank processes on one MI355X: 32 x 64 KiB slices
// 32.8 us against graph replay 40.9 us; at 8 MiB messages 128 x 64 KiB
// slices lose to graph replay (profiles/round3/r3y_latency_*).
size_t sliceCapBytes() { return 2 * sliceBytes(); }

// The sliced form splits a plan's whole-range local steps (LOCAL_REDUCE /
// LOCAL_BCAST over [0, n)) at every boundary the other steps use in the
// user buffers, so that the pieces later steps read are exactly pieces that
// were written.  Element-wise, so the bytes are the same.
std::vector<size_t> userCuts(const Plan& plan) {
  std::set<size_t> c;
  auto add = [&](size_t off, size_t len) {
    c.insert(off);
    c.insert(off + len);
  };
  for (const Step& t : plan.steps) {
    switch (t.kind) {
      case GLOO_HIP_STEP_SEND:
      case GLOO_HIP_STEP_FOLD_SRC:
        if (!(t.flags & GLOO_HIP_SRC_ARENA)) add(t.src_off, t.length);
        break;
      case GLOO_HIP_STEP_REDUCE:
        add(t.dst_off, t.length);
        break;
      case GLOO_HIP_STEP_COPY:
        if (!(t.flags & GLOO_HIP_SRC_ARENA)) add(t.src_off, t.length);
        if (!(t.flags & GLOO_HIP_DST_ARENA)) add(t.dst_off, t.length);
        break;
      case GLOO_HIP_STEP_FOLD:
        if (!(t.flags & GLOO_HIP_DST_ARENA)) add(t.dst_off, t.length);
        break;
      default:
        break;
    }
  }
  return std::vector<size_t>(c.begin(), c.end());
}

// [off, off + len) cut at `cuts` (sorted): the (offset, length) pieces.
std::vector<std::pair<size_t, size_t>> cutRange(const std::vector<size_t>& cuts, size_t off, size_t len) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t at = off;
  for (size_t c : cuts)
    if (c > at && c < off + len) {
      out.push_back({at, c - at});
      at = c;
    }
  if (off + len > at) out.push_back({at, off + len - at});
  return out;
}

// Can the plan run as slices (signal.h, sliced interpreter)?  Workgroup g
// handles slice g of every step and never meets the others, so every step
// must read exactly the ranges earlier steps wrote: a read overlapping an
// earlier write (a peer's message into the arena counts as one, written
// before anything) must be that same range, and a write overlapping any
// earlier access must be that same range.  Reads of data nobody wrote this
// run (the user's buffers) may overlap freely.
bool sliceable(const Plan& plan, int nin, int nout, const std::vector<Access>& remoteWrites) {
  const std::vector<size_t> cuts = userCuts(plan);
  std::map<int, std::vector<Access>> reads, writes;
  auto clash = [](const Access& a, const Access& b) {
    const bool overlap = a.off < b.off + b.len && b.off < a.off + a.len;
    return overlap && !(a.off == b.off && a.len == b.len);
  };
  auto write = [&](const Access& w) {
    if (!w.len) return true;
    for (const Access& x : reads[w.buf])
      if (clash(x, w)) return false;
    for (const Access& x : writes[w.buf])
      if (clash(x, w)) return false;
    writes[w.buf].push_back(w);
    return true;
  };
  auto read = [&](const Access& r) {
    if (!r.len) return true;
    for (const Access& x : writes[r.buf])
      if (clash(x, r)) return false;
    reads[r.buf].push_back(r);
    return true;
  };
  for (const Access& w : remoteWrites)
    if (!write(w)) return false;
  auto sendBuf = [](const Step& t) {
    return t.flags & GLOO_HIP_SRC_ARENA ? kArena : t.flags & GLOO_HIP_FROM_INPUTS ? kIn : 0;
  };
  for (const Step& t : plan.steps) {
    const size_t L = t.length;
    bool ok = true;
    switch (t.kind) {
      case GLOO_HIP_STEP_SEND:
      case GLOO_HIP_STEP_FOLD_SRC:
        ok = read({sendBuf(t), t.src_off, L});
        break;
      case GLOO_HIP_STEP_REDUCE:
        ok = read({t.flags & GLOO_HIP_FROM_INPUTS ? kIn : 0, t.dst_off, L}) && read({kArena, t.src_off, L}) &&
             write({0, t.dst_off, L});
        break;
      case GLOO_HIP_STEP_COPY:
        ok = read({t.flags & GLOO_HIP_SRC_ARENA ? kArena : 0, t.src_off, L}) &&
             write({t.flags & GLOO_HIP_DST_ARENA ? kArena : 0, t.dst_off, L});
        break;
      case GLOO_HIP_STEP_FOLD:
        ok = write({t.flags & GLOO_HIP_DST_ARENA ? kArena : 0, t.dst_off, L});
        break;
      case GLOO_HIP_STEP_LOCAL_REDUCE: {
        const bool fromIn = t.flags & GLOO_HIP_FROM_INPUTS;
        for (const auto& pc : cutRange(cuts, t.dst_off, L)) {
          for (int j = 0; j < (fromIn ? nin : nout) && ok; j++)
            ok = read({(fromIn ? kIn : 0) + j, pc.first, pc.second});
          ok = ok && write({0, pc.first, pc.second});
        }
        break;
      }
      case GLOO_HIP_STEP_LOCAL_BCAST:
        for (const auto& pc : cutRange(cuts, t.dst_off, L)) {
          ok = ok && read({0, pc.first, pc.second});
          for (int j = 1; j < nout && ok; j++) ok = write({j, pc.first, pc.second});
        }
        break;
      default:
        break;
    }
    if (!ok) return false;
  }
  return true;
}

// Upper bound on the interpreter steps buildInterp() emits for the sliced
// form of `plan`: it mirrors buildInterp's pushes, with the whole-range local
// steps counted once per piece.  A plan over the device list's capacity
// (kInterpMaxSteps) must not be proposed for slicing, because a sliced plan
// has no other route (many small segments of a large new-style call).
size_t slicedInterpSteps(const Plan& plan, int nin, int nout) {
  const std::vector<size_t> cuts = userCuts(plan);
  size_t k = 0;
  for (const Step& t : plan.steps) {
    switch (t.kind) {
      case GLOO_HIP_STEP_DECL_RECV:
      case GLOO_HIP_STEP_WAIT_SEND:
      case GLOO_HIP_STEP_FOLD_SRC:
        break;
      case GLOO_HIP_STEP_LOCAL_REDUCE: {
        const size_t srcs = (size_t)std::max(1, t.flags & GLOO_HIP_FROM_INPUTS ? nin : nout);
        const size_t per =
            srcs <= GLOO_HIP_MAX_SRCS ? 1 : 1 + (srcs - GLOO_HIP_MAX_SRCS + GLOO_HIP_MAX_SRCS - 2) / (GLOO_HIP_MAX_SRCS - 1);
        k += cutRange(cuts, t.dst_off, t.length).size() * per;
        break;
      }
      case GLOO_HIP_STEP_LOCAL_BCAST:
        k += cutRange(cuts, t.dst_off, t.length).size() * (size_t)std::max(0, nout - 1);
        break;
      default:
        k += 1;
        break;
    }
  }
  return k;
}

// Most workgroups of a sliced launch (<= kMaxSlices).  Ranks that share a
// GPU each bring this many, and a slice spins until its peer slice runs, so
// the default keeps 8 ranks on one GPU co-resident.
int maxSlices() {
  static const int v = [] {
    const char* e = std::getenv("GLOO_AMD_INTERP_MAX_SLICES");
    return e ? std::min(kMaxSlices, std::max(1, std::atoi(e))) : 32;
  }();
  return v;
}

int coResidentSlices(int device, int ranksHere) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) {
    (void)hipGetLastError();
    return std::min(maxSlices(), 32);
  }
  return std::max(1, std::min(maxSlices(), cus / std::max(1, ranksHere)));
}

int64_t gpuLocation(int device) {
  int dom = 0, bus = 0, dev = 0;
  if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess ||
      hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess) {
    (void)hipGetLastError();
    return -1 - device;  // unknown: the device index
  }
  return ((int64_t)dom << 32) | ((int64_t)bus << 8) | (int64_t)dev;
}

}  // namespace exec
}  // namespace gloo_amd

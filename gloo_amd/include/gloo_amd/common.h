// common.h — errors and checks (mirrors gloo/common/error.h:24-48 and
// gloo/common/logging.h:32-59: failures surface as C++ exceptions inside the
// library; the C-ABI converts them to status codes).
#pragma once

#include <hip/hip_runtime_api.h>

#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>

namespace gloo_amd {

struct Exception : std::runtime_error {
  explicit Exception(const std::string& m) : std::runtime_error(m) {}
};
// GLOO_ENFORCE failures (gloo::EnforceNotMet).
struct EnforceNotMet : Exception {
  explicit EnforceNotMet(const std::string& m) : Exception(m) {}
};
// Transport failures and timeouts (gloo::IoException).
struct IoException : Exception {
  explicit IoException(const std::string& m) : Exception(m) {}
};

// gloo::CudaShared (gloo/cuda.h:40-54): the mutex that serialises this
// library's device allocations, frees and IPC mappings with those of the
// host framework (which may install its own allocator's mutex).  Held only
// around the individual HIP calls, never across a rendezvous.
class HipShared {
 public:
  static std::mutex& getMutex();
  static void setMutex(std::mutex* m);
};

template <typename... Args>
std::string strcat_(Args&&... args) {
  std::ostringstream ss;
  (ss << ... << args);
  return ss.str();
}

}  // namespace gloo_amd

#define GLOO_AMD_ENFORCE(cond, ...)                                                    \
  do {                                                                                 \
    if (!(cond))                                                                       \
      throw ::gloo_amd::EnforceNotMet(::gloo_amd::strcat_(__FILE__, ":", __LINE__,     \
                                                          ": ", #cond, " ", ##__VA_ARGS__)); \
  } while (0)

// A HIP allocation / free / mapping call under HipShared's mutex.
#define GLOO_AMD_HIP_ALLOC(expr)                                                       \
  do {                                                                                 \
    std::lock_guard<std::mutex> allocLock_(::gloo_amd::HipShared::getMutex());         \
    GLOO_AMD_HIP_CHECK(expr);                                                          \
  } while (0)
#define GLOO_AMD_HIP_RELEASE(expr)                                                     \
  do {                                                                                 \
    std::lock_guard<std::mutex> allocLock_(::gloo_amd::HipShared::getMutex());         \
    (void)(expr);                                                                      \
  } while (0)

#define GLOO_AMD_HIP_CHECK(expr)                                                       \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      throw ::gloo_amd::EnforceNotMet(::gloo_amd::strcat_(__FILE__, ":", __LINE__, ": ", \
                                                          #expr, ": ", hipGetErrorString(e_))); \
  } while (0)

// errors.cc — see errors.h.
#include "gloo_amd/errors.h"

#include <cstdio>

#include "gloo_amd.h"

namespace gloo_amd {
namespace {
thread_local char g_last_error[1024] = "";
}
int setError(int code, const std::string& msg) {
  std::snprintf(g_last_error, sizeof(g_last_error), "%s", msg.c_str());
  return code;
}
}  // namespace gloo_amd

extern "C" const char* gloo_hip_last_error(void) { return gloo_amd::g_last_error; }

// errors.cc — see errors.h.
#include "gloo_amd/errors.h"

#include <atomic>
#include <cstdio>

#include "gloo_amd.h"
#include "gloo_amd/common.h"

namespace gloo_amd {
namespace {
thread_local char g_last_error[1024] = "";
}
namespace {
std::mutex g_default_mutex;
std::atomic<std::mutex*> g_alloc_mutex{&g_default_mutex};
}  // namespace
std::mutex& HipShared::getMutex() { return *g_alloc_mutex.load(); }
void HipShared::setMutex(std::mutex* m) { g_alloc_mutex.store(m ? m : &g_default_mutex); }

int setError(int code, const std::string& msg) {
  std::snprintf(g_last_error, sizeof(g_last_error), "%s", msg.c_str());
  return code;
}
}  // namespace gloo_amd

extern "C" const char* gloo_hip_last_error(void) { return gloo_amd::g_last_error; }

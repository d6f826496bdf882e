// errors.h — thread-local last-error text behind gloo_hip_last_error().
#pragma once

#include <string>

namespace gloo_amd {
// Records `msg` as the calling thread's last error and returns `code`.
int setError(int code, const std::string& msg);
}  // namespace gloo_amd

// common.hip — error plumbing and version string of librlks.so
#include <hip/hip_runtime.h>

#include <string>

#include "rlks_internal.h"

namespace rlks {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

}  // namespace rlks

extern "C" {

const char* rlks_last_error(void) { return rlks::g_last_error.c_str(); }

const char* rlks_version(void) { return "rlks 0.1.0 gfx950"; }

}  // extern "C"

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

#ifdef RLKS_DEBUG
int dcheck_read_env(unsigned long long*);
int dcheck_read_ppo(unsigned long long*);
int dcheck_read_sgd(unsigned long long*);
#endif

}  // namespace rlks

int rlks_debug_checks(unsigned long long* out) {
#ifdef RLKS_DEBUG
  RLKS_REQUIRE(out, RLKS_ERR_ARG, "rlks_debug_checks: null argument");
  RLKS_HIP(hipDeviceSynchronize());
  int (*readers[])(unsigned long long*) = {rlks::dcheck_read_env, rlks::dcheck_read_ppo, rlks::dcheck_read_sgd};
  out[0] = out[1] = out[2] = 0;
  for (auto rd : readers) {
    unsigned long long v[3];
    RLKS_REQUIRE(rd(v) == 0, RLKS_ERR_HIP, "rlks_debug_checks: counter read failed");
    if (v[0] && !out[0]) { out[1] = v[1]; out[2] = v[2]; }
    out[0] += v[0];
  }
  return RLKS_OK;
#else
  (void)out;
  return rlks::fail(RLKS_ERR_UNSUPPORTED, "rlks_debug_checks: not a debug build (make -C csrc debug)");
#endif
}

extern "C" {

const char* rlks_last_error(void) { return rlks::g_last_error.c_str(); }

const char* rlks_version(void) { return "rlks 0.1.0 gfx950"; }

}  // extern "C"

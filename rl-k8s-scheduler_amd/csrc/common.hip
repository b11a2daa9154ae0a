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
// the counters' readers of every translation unit (registered by their static initialisers; a
// function-local registry, so that the units' initialisation order does not matter)
struct DcheckReaders {
  int (*f[64])(unsigned long long*);
  int n = 0;
};
static DcheckReaders& dcheck_readers() {
  static DcheckReaders r;
  return r;
}
void dcheck_register(int (*reader)(unsigned long long*)) {
  DcheckReaders& r = dcheck_readers();
  if (r.n < 64) r.f[r.n++] = reader;
}
#endif

}  // namespace rlks

int rlks_debug_checks(unsigned long long* out) {
#ifdef RLKS_DEBUG
  RLKS_REQUIRE(out, RLKS_ERR_ARG, "rlks_debug_checks: null argument");
  RLKS_HIP(hipDeviceSynchronize());
  const rlks::DcheckReaders& R = rlks::dcheck_readers();
  // RLKS_N_TU: the Makefile's source count (every TU includes rlks_internal.h and registers once)
  RLKS_REQUIRE(R.n == RLKS_N_TU, RLKS_ERR_HIP, "rlks_debug_checks: registered counter sets != translation units");
  out[0] = out[1] = out[2] = 0;
  for (int i = 0; i < R.n; ++i) {
    unsigned long long v[3];
    RLKS_REQUIRE(R.f[i](v) == 0, RLKS_ERR_HIP, "rlks_debug_checks: counter read failed");
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

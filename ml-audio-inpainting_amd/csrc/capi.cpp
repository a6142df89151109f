// capi.cpp — library identity and error reporting for the ainp C ABI.
#include <rocprofiler-sdk-roctx/roctx.h>
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "common.h"

namespace ainp {
static thread_local char g_last_error[512] = "";

int record_error(hipError_t e, const char* where) {
  snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where,
           hipGetErrorString(e));
  return AINP_ELAUNCH;
}
int record_msg(const char* msg) {
  snprintf(g_last_error, sizeof(g_last_error), "%s", msg);
  return AINP_EINVAL;
}
}  // namespace ainp

extern "C" int ainp_abi_version(void) { return 1; }

// Per-phase trace ranges (SURVEY §5 tracing): roctx ranges of the
// rocprofiler-sdk marker API, recorded by `rocprofv3 --marker-trace`; a no-op
// cost (one call) when no profiler is attached.
extern "C" int ainp_range_push(const char* name) { return roctxRangePushA(name ? name : "?"); }
extern "C" int ainp_range_pop(void) { return roctxRangePop(); }
extern "C" void ainp_mark(const char* name) { roctxMarkA(name ? name : "?"); }
extern "C" const char* ainp_build_target(void) { return "gfx950"; }
extern "C" const char* ainp_last_error(void) { return ainp::g_last_error; }

// Library identity + per-thread error string of the C ABI (include/onetrans_hip.h).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace ot {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace ot

extern "C" int ot_version(void) { return 20000; }   // 2.0.0: ot_rms_epilogue.struct_size (round 4)
extern "C" const char* ot_get_last_error_string(void) { return ot::g_err; }
extern "C" int ot_gemm_tile_rows(void) { return 128; }

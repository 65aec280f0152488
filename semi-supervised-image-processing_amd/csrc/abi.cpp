// C-ABI plumbing: thread-local error string, launch checks, version.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include "../../include/ssip.h"
#include "stop_event.h"

namespace ssip {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

StopEvent& stop_event() {
  static thread_local StopEvent s;
  return s;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return SSIP_ERR_LAUNCH;
  }
  return SSIP_OK;
}
}  // namespace ssip

extern "C" {
const char* ssip_last_error(void) { return ssip::g_err; }
int ssip_version(void) { return SSIP_ABI_VERSION; }
}

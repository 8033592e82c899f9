// Error reporting and version entry points of the mvml_gat C ABI.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace mvml {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return MVML_ERR_LAUNCH;
  }
  return MVML_OK;
}

}  // namespace mvml

extern "C" const char* mvml_last_error(void) { return mvml::g_err; }

extern "C" const char* mvml_version(void) { return "mvml_gat 0.1.0 (gfx950)"; }

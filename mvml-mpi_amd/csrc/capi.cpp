// Error reporting and version entry points of the mvml_gat C ABI.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>

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

// Kernel-path options (include/mvml_gat.h, MVML_OPT_*): environment defaults read once at load.
constexpr int kOptCount = 12;
static std::atomic<int> g_opt[kOptCount];
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
static const bool g_opt_init = [] {
  g_opt[MVML_OPT_BIG_WINDOW] = env_int("MVML_BIG_WINDOW", 1);
  g_opt[MVML_OPT_BWD_ATOMWISE] = env_int("MVML_BWD_ATOMWISE", 0);
  g_opt[MVML_OPT_GEMM_TILE] = env_int("MVML_X3_TILE", 0);
  g_opt[MVML_OPT_GEMM_PERSIST] = env_int("MVML_X3W_PERSIST", 256);  // one per CU (MI355X)
  g_opt[MVML_OPT_GEMM_NSPLIT] = env_int("MVML_GEMM_NSPLIT", 1);
  g_opt[MVML_OPT_GEMM_RING] = env_int("MVML_GEMM_RING", 0);
  g_opt[MVML_OPT_LSTM_TILE] = env_int("MVML_LSTM_TILE", 0);
  g_opt[MVML_OPT_MEAN_SRC] = env_int("MVML_MEAN_SRC", 1);
  g_opt[MVML_OPT_FLAT_SRC] = env_int("MVML_FLAT_SRC", 0);
  g_opt[MVML_OPT_DST_FWD] = env_int("MVML_DST_FWD", 0);
  g_opt[MVML_OPT_DST_UNR] = env_int("MVML_DST_UNR", 0);
  g_opt[MVML_OPT_SMALLK] = env_int("MVML_SMALLK", 1);
  return true;
}();

int option(int i) { return g_opt[i].load(std::memory_order_relaxed); }

}  // namespace mvml

extern "C" int mvml_set_option(int opt, int value) {
  if (opt < 0 || opt >= mvml::kOptCount) return -1;
  return mvml::g_opt[opt].exchange(value, std::memory_order_relaxed);
}

extern "C" int mvml_get_option(int opt) {
  if (opt < 0 || opt >= mvml::kOptCount) return -1;
  return mvml::option(opt);
}

extern "C" const char* mvml_last_error(void) { return mvml::g_err; }

extern "C" const char* mvml_version(void) { return "mvml_gat 0.1.0 (gfx950)"; }

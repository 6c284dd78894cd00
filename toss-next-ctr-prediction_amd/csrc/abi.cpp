// Error plumbing + version for the C ABI (include/ctr_hip.h).
#include <hip/hip_runtime.h>

#include <string>

#include "common.h"
#include "ctr_hip.h"

namespace ctr {
static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return -2;
  }
  return 0;
}
}  // namespace ctr

extern "C" const char* ctr_last_error(void) { return ctr::g_err.c_str(); }

extern "C" int ctr_abi_version(void) { return 1; }

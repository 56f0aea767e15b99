// qb_capi.cpp — library-level C ABI: version, per-thread error text, devices.
#include <cstdarg>
#include <cstdio>

#include "qb_common.h"

namespace qb {

namespace {
thread_local char t_err[512] = "";
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(t_err, sizeof t_err, fmt, ap);
  va_end(ap);
}

int hip_fail(hipError_t e, const char* what) {
  set_error("%s: %s (%d)", what, hipGetErrorString(e), int(e));
  return QB_EHIP;
}

}  // namespace qb

extern "C" int qb_abi_version(void) { return QB_ABI_VERSION; }

extern "C" const char* qb_last_error(void) { return qb::t_err; }

extern "C" int qb_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky error; "no GPU" is not a failure
    return 0;
  }
  return n;
}

// Library-wide C entry points: version, error reporting, device query.
#include "common.hpp"

#include <cstring>

namespace slam {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace slam

extern "C" int slam_abi_version(void) { return SLAM355_ABI_VERSION; }

extern "C" const char* slam_last_error(void) { return slam::g_err; }

extern "C" int slam_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

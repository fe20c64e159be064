// Library-level C-ABI entry points: version string and the thread-local error message.
#include "idn_common.hpp"

#include <string.h>

namespace idn {

static thread_local char g_err[512] = "";

int set_error(int status, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return status;
}

}  // namespace idn

extern "C" int idn_abi_version(void) { return IDN_ABI_VERSION; }

extern "C" const char* idn_version(void) { return "idn 0.4.0 gfx950"; }

extern "C" const char* idn_last_error(void) { return idn::g_err; }

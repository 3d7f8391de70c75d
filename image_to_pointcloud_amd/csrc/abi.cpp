// ABI bookkeeping: version and thread-local last-error string.
#include "common.h"

#include <cstring>

namespace i2pc {

static thread_local char g_err[512] = {0};

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

void clear_error() { g_err[0] = 0; }

}  // namespace i2pc

extern "C" int i2pc_abi_version(void) { return 1; }

extern "C" const char* i2pc_last_error(void) { return i2pc::g_err; }

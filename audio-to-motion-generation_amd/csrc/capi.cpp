// Error reporting shared by every C-ABI entry point.
#include <cstdarg>
#include <cstdio>

#include "../../include/a2m.h"

namespace a2m {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace a2m

extern "C" {

const char* a2m_last_error(void) { return a2m::g_err; }

int a2m_version(void) { return 1; }

}

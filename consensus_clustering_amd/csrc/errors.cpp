// Thread-local error message and version string of libccmi (no exceptions cross the ABI).
#include <string>

#include "ccmi_internal.h"

namespace {
thread_local std::string g_last_error;
}

namespace cc {
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace cc

extern "C" const char* cc_last_error(void) { return g_last_error.c_str(); }

extern "C" const char* cc_version(void) { return "ccmi 0.1.0 (gfx950)"; }

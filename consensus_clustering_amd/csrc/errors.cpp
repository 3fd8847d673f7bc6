// Thread-local error message, version string and build id of libccmi (no exceptions cross
// the ABI).
#include <string>

#include "ccmi_internal.h"

#ifndef CC_BUILD_ID
#define CC_BUILD_ID "unknown"
#endif
#ifndef CC_BUILD_FLAGS
#define CC_BUILD_FLAGS ""
#endif

namespace {
thread_local std::string g_last_error;
}

namespace cc {
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace cc

extern "C" const char* cc_last_error(void) { return g_last_error.c_str(); }

extern "C" const char* cc_version(void) { return "ccmi 0.2.0 (gfx950) flags: " CC_BUILD_FLAGS; }

extern "C" const char* cc_build_id(void) { return CC_BUILD_ID; }

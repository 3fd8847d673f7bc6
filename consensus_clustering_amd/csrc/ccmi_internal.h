// Internal helpers shared by the libccmi translation units (not part of the ABI).
#pragma once

#include <string>

#include "../../include/ccmi.h"

namespace cc {

void set_error(const std::string& msg);

}  // namespace cc

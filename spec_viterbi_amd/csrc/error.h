// svh::Error: a C-ABI status code and a message (thrown inside the library, turned into a status
// at the extern "C" boundary).  No HIP dependency: host-only code (the readers) uses it too.
#pragma once

#include <stdexcept>
#include <string>

namespace svh {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& msg) : std::runtime_error(msg), code(c) {}
};

}  // namespace svh

// HIP error handling for the host side of libzkp_amd: every failing HIP call
// becomes a C++ exception, which the C-ABI layer (capi.cpp) turns into a
// status code + thread-local message.  No exception ever crosses the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>

namespace zkp {

struct HipError : std::runtime_error {
  hipError_t code;
  HipError(hipError_t e, const char* expr, const char* file, int line)
      : std::runtime_error(std::string("HIP error '") + hipGetErrorString(e) + "' in " + expr + " at " + file + ":" +
                           std::to_string(line)),
        code(e) {}
};

}  // namespace zkp

#define HIPX(expr)                                                                  \
  do {                                                                              \
    hipError_t _zkp_e = (expr);                                                     \
    if (_zkp_e != hipSuccess) throw ::zkp::HipError(_zkp_e, #expr, __FILE__, __LINE__); \
  } while (0)

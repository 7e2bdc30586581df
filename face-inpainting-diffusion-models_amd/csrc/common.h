// Shared helpers for the ifd HIP library (gfx950 / MI355X only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>

namespace ifd {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

void set_error(const std::string& msg);
const char* get_error();

#define IFD_CHECK_HIP(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      ::ifd::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" +        \
                       __FILE__ + ":" + std::to_string(__LINE__));                       \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

#define IFD_REQUIRE(cond, msg)                                                           \
  do {                                                                                   \
    if (!(cond)) {                                                                       \
      ::ifd::set_error(std::string("ifd: ") + (msg));                                    \
      return 2;                                                                          \
    }                                                                                    \
  } while (0)

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

}  // namespace ifd

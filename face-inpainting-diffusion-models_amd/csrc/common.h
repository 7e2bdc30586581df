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
void clear_error();

// The status of the launch just issued (hipGetLastError), with the error message set for it, naming `where`
// (callers pass __func__), so a nonzero status never reaches the host with another call's message. A fault of
// an EARLIER asynchronous launch (illegal address, ...) surfaces at the next launch check: the message says so.
inline int launch_status(const char* where) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    std::string m = std::string(where) + ": " + hipGetErrorString(e);
    if (e == hipErrorIllegalAddress || e == hipErrorLaunchFailure || e == hipErrorAssert)
      m += " (a device fault; it may come from an earlier asynchronous launch on this device)";
    set_error(m);
  }
  return (int)e;
}
#define IFD_LAUNCH_STATUS() ::ifd::launch_status(__func__)
// A failed launcher status inside a host routine: the message names what was running and the HIP status.
#define IFD_LAUNCH_OK(e, what)                                                           \
  do {                                                                                   \
    if ((e) != 0) {                                                                      \
      ::ifd::set_error(std::string("ifd: ") + (what) + " launch: " +                     \
                       hipGetErrorString((hipError_t)(e)));                             \
      return (e);                                                                        \
    }                                                                                    \
  } while (0)

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

// Launchers keep one-time per-device state (large-LDS attribute set, CU count). One process may
// drive several devices through several handles, so the state is keyed by the device ordinal.
constexpr int kMaxDevices = 64;
inline int current_device() {
  int d = 0;
  (void)hipGetDevice(&d);
  return (d >= 0 && d < kMaxDevices) ? d : 0;
}
inline int device_cu_count() {
  static int ncu[kMaxDevices] = {};
  const int d = current_device();
  if (!ncu[d]) {
    int n = 0;
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d);
    ncu[d] = n > 0 ? n : 256;
  }
  return ncu[d];
}
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device); `done` is the
// caller's per-kernel table.
inline hipError_t set_lds_attr_once(bool (&done)[kMaxDevices], const void* fn, int bytes) {
  const int d = current_device();
  if (done[d]) return hipSuccess;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done[d] = true;
  return e;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

}  // namespace ifd

// Shared host-side helpers for the i2pc C ABI (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdint>

#include "../../include/i2pc.h"

namespace i2pc {

// Records the message returned by i2pc_last_error(); returns `code`.
int set_error(int code, const char* fmt, ...);
void clear_error();

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(I2PC_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
  return I2PC_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

constexpr int kWave = 64;

}  // namespace i2pc

#define I2PC_REQUIRE(cond, ...)                                  \
  do {                                                           \
    if (!(cond)) return ::i2pc::set_error(I2PC_EINVAL, __VA_ARGS__); \
  } while (0)

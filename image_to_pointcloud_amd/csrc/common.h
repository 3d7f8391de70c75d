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

// two floats -> packed bf16 pair (low = a) in one v_cvt_pk_bf16_f32 (RNE, the same bits as two scalar
// (__bf16) conversions; the scalar pair costs a convert each plus a shift and an or)
__device__ __forceinline__ uint32_t pk2bf(float a, float b) {
  typedef float pk2bf_f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 pk2bf_b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(pk2bf_f2{a, b}, pk2bf_b2));
}

constexpr int kWave = 64;

}  // namespace i2pc

#define I2PC_REQUIRE(cond, ...)                                  \
  do {                                                           \
    if (!(cond)) return ::i2pc::set_error(I2PC_EINVAL, __VA_ARGS__); \
  } while (0)

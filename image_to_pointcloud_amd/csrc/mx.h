// OCP MX fp8 (e4m3fn data + E8M0 scale per 32 elements) device helpers shared by the fp8
// GEMM epilogue (gemm.hip) and the quantising producers (fp8.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace i2pc {
namespace mx {

// E8M0 exponent e of an MX block with max |v| = amax: the smallest e with amax / 2^e <= 448
// (e4m3fn's largest normal, 1.75 * 2^8), clamped to the E8M0 range [-127, 127]; the block's
// values are then v * 2^-e, rounded to e4m3 with no saturation needed.
__device__ __forceinline__ int mx_exponent(float amax) {
  const uint32_t b = __float_as_uint(amax);
  const int ex = (int)((b >> 23) & 0xff) - 127;
  int e = ex - 8 + ((b & 0x7fffff) > 0x600000 ? 1 : 0);
  if (amax == 0.f) e = -127;
  return e < -127 ? -127 : e > 127 ? 127 : e;
}
__device__ __forceinline__ float exp2i(int x) {   // 2^x for x in [-127, 127]
  return x >= -126 ? __uint_as_float((uint32_t)(x + 127) << 23) : __uint_as_float(0x00400000u);
}
// four floats (already scaled into e4m3 range) -> four e4m3fn bytes, round to nearest even
__device__ __forceinline__ uint32_t pack_e4m3(float a, float b, float c, float d) {
  const float L = 448.f;
  a = fminf(fmaxf(a, -L), L); b = fminf(fmaxf(b, -L), L);
  c = fminf(fmaxf(c, -L), L); d = fminf(fmaxf(d, -L), L);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

}  // namespace mx
}  // namespace i2pc

// Shader-clock probe of the running chip (bench.py's clock_ghz_run).
//
// The chip lowers its clock under load and devices differ (MI355X_MICROARCH.md, "DVFS give-back"), so
// a kernel's fraction of the 2.5 PF peak says little without the clock it ran at.  k_clock_probe runs
// one 256-thread workgroup per CU (4 waves, one per SIMD) through a fixed chain of dense bf16 MFMAs on
// random operands and stamps s_memtime (shader clock ticks) against s_memrealtime (the 100 MHz
// constant clock) around it (the guide's item 6).  bench.py launches it right before and right after
// its timed steps, so the figure is the clock THIS box held under dense MFMA load in THIS run.
#include "common.h"

namespace i2pc {
namespace probe {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t mix32(uint32_t x) {   // lowbias32
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__device__ __forceinline__ bf16x8 rand8(uint32_t seed) {
  bf16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    // random sign and mantissa, exponent near 1.0: dense bit activity, no overflow over the chain
    const uint32_t h = mix32(seed * 8u + (uint32_t)e);
    const uint16_t b = (uint16_t)((h & 0x807fu) | 0x3f00u);
    v[e] = __builtin_bit_cast(__bf16, b);
  }
  return v;
}

// out[2 * blockIdx.x] = shader ticks, out[2 * blockIdx.x + 1] = 100 MHz ticks of the MFMA chain
__global__ __launch_bounds__(256) void k_clock_probe(int iters, unsigned long long* __restrict__ out) {
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  const bf16x8 a0 = rand8(gid * 4u), a1 = rand8(gid * 4u + 1u);
  const bf16x8 b0 = rand8(gid * 4u + 2u), b1 = rand8(gid * 4u + 3u);
  f32x16 c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int e = 0; e < 16; ++e) c[k][e] = 0.f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    // four independent accumulators keep the SIMD's matrix pipe full
    c[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, c[0], 0, 0, 0);
    c[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, c[1], 0, 0, 0);
    c[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, c[2], 0, 0, 0);
    c[3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, c[3], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += c[k][e];
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r1 - r0;
  }
  if (s == 1234.5f) out[0] = 0;   // keeps the chain live (never true on these operands in practice)
}

}  // namespace probe
}  // namespace i2pc

extern "C" int i2pc_clock_probe(int workgroups, int iters, unsigned long long* out, void* stream) {
  using namespace i2pc;
  clear_error();
  I2PC_REQUIRE(out, "NULL pointer");
  I2PC_REQUIRE(workgroups >= 1 && workgroups <= 4096 && iters >= 1, "clock_probe: workgroups 1..4096, iters >= 1");
  hipLaunchKernelGGL(probe::k_clock_probe, dim3(workgroups), dim3(256), 0, as_stream(stream), iters, out);
  return check_launch("clock_probe");
}

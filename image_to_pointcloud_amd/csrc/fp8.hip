// MX fp8 producers of the DPT-Hybrid fp8 path (gfx950): activations are quantised once,
// by the kernel that already holds them, into the operand format of i2pc_gemm_fp8 --
// e4m3fn bytes [rows][K] plus one E8M0 scale byte per 32 consecutive k, stored as uint32
// [rows][K / 128] (byte b of dword kt = block 4 kt + b).  Block scale: the smallest power
// of two with max |v| / 2^e <= 448 (mx.h), so no value saturates; e4m3 rounding is the
// hardware's round-to-nearest-even (v_cvt_pk_fp8_f32).
//   k_quant_rows      : bf16 / fp32 rows (optional ReLU, optional row remap) -> fp8 rows
//   k_layernorm_fp8   : LayerNorm (modeling_dpt.py:233-234) written straight as fp8 rows
#include "common.h"
#include "mx.h"

namespace i2pc {
namespace f8 {

using namespace ::i2pc::mx;

__device__ __forceinline__ float bf2f(uint32_t lo16) { return __uint_as_float(lo16 << 16); }

// one thread per (row, 32-element block); output row r reads input row
// (r / g) * gs + r % g + o (g = 0: r + o)
template <bool F32>
__global__ __launch_bounds__(256) void k_quant_rows(const void* __restrict__ x, int64_t ldx, int rows, int nb, int relu,
                                                    int g, int gs, int o, uint8_t* __restrict__ y, int64_t ldy,
                                                    uint8_t* __restrict__ ys, int64_t ldys_bytes) {
  const int64_t total = (int64_t)rows * nb;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / nb);
    const int blk = (int)(i - (int64_t)r * nb);
    const int64_t src = g > 0 ? (int64_t)(r / g) * gs + (r % g) + o : (int64_t)r + o;
    float v[32];
    if (F32) {
      const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(x) + src * ldx + blk * 32);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 t = p[q];
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
      }
    } else {
      const uint4* p = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(x) + src * ldx + blk * 32);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 t = p[q];
        const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[8 * q + 2 * e] = bf2f(w[e] & 0xffffu);
          v[8 * q + 2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
        }
      }
    }
    float am = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      if (relu) v[e] = fmaxf(v[e], 0.f);
      am = fmaxf(am, fabsf(v[e]));
    }
    const int ex = mx_exponent(am);
    const float mul = exp2i(-ex);
    uint32_t d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = pack_e4m3(v[4 * q] * mul, v[4 * q + 1] * mul, v[4 * q + 2] * mul, v[4 * q + 3] * mul);
    uint4* out = reinterpret_cast<uint4*>(y + (int64_t)r * ldy + blk * 32);
    out[0] = make_uint4(d[0], d[1], d[2], d[3]);
    out[1] = make_uint4(d[4], d[5], d[6], d[7]);
    ys[(int64_t)r * ldys_bytes + blk] = (uint8_t)(ex + 127);
  }
}

__device__ __forceinline__ float wave_sum(float x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// one wave per row, V float4 per lane (dim = 256 V), two-pass variance as k_layernorm;
// a 32-element block = 8 consecutive lanes' float4s
template <int V>
__global__ __launch_bounds__(256) void k_layernorm_fp8(const float* __restrict__ x, int64_t ldx, const float* __restrict__ gm,
                                                       const float* __restrict__ bt, float eps, int rows, int dim,
                                                       uint8_t* __restrict__ y, int64_t ldy, uint8_t* __restrict__ ys,
                                                       int64_t ldys_bytes) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float4* xr = reinterpret_cast<const float4*>(x + row * ldx);
  float4 v[V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    v[i] = xr[i * 64 + lane];
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = wave_sum(s) / (float)dim;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float a = v[i].x - mean, c = v[i].y - mean, d = v[i].z - mean, e = v[i].w - mean;
    q += (a * a + c * c) + (d * d + e * e);
  }
  const float var = wave_sum(q) / (float)dim;
  const float rstd = 1.0f / sqrtf(var + eps);
  const float4* g4 = reinterpret_cast<const float4*>(gm);
  const float4* b4 = reinterpret_cast<const float4*>(bt);
  uint32_t* yr = reinterpret_cast<uint32_t*>(y + row * ldy);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float4 gg = g4[i * 64 + lane], bb = b4[i * 64 + lane];
    const float o0 = (v[i].x - mean) * rstd * gg.x + bb.x, o1 = (v[i].y - mean) * rstd * gg.y + bb.y;
    const float o2 = (v[i].z - mean) * rstd * gg.z + bb.z, o3 = (v[i].w - mean) * rstd * gg.w + bb.w;
    float am = fmaxf(fmaxf(fabsf(o0), fabsf(o1)), fmaxf(fabsf(o2), fabsf(o3)));
    am = fmaxf(am, __shfl_xor(am, 1));
    am = fmaxf(am, __shfl_xor(am, 2));
    am = fmaxf(am, __shfl_xor(am, 4));
    const int ex = mx_exponent(am);
    const float mul = exp2i(-ex);
    yr[i * 64 + lane] = pack_e4m3(o0 * mul, o1 * mul, o2 * mul, o3 * mul);
    if ((lane & 7) == 0) ys[(int64_t)row * ldys_bytes + (i * 64 + lane) / 8] = (uint8_t)(ex + 127);
  }
}

}  // namespace f8
}  // namespace i2pc

using namespace i2pc;

extern "C" int i2pc_quant_fp8(const void* x, int x_f32, int64_t ldx, int rows, int k, int relu, int row_group,
                              int row_group_stride, int row_offset, void* y, int64_t ldy, void* y_scale,
                              int64_t ldy_scale, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && y && y_scale, "NULL pointer");
  I2PC_REQUIRE(rows > 0 && k > 0 && k % 32 == 0, "quant_fp8: rows > 0 and k %% 32 == 0 required (k=%d)", k);
  I2PC_REQUIRE(ldx % 8 == 0 && ldy % 16 == 0 && ldy >= k && ldy_scale * 128 >= k,
               "quant_fp8: ldx %% 8, ldy %% 16, ldy >= k, ldy_scale >= k/128 required");
  const int nb = k / 32;
  const int64_t total = (int64_t)rows * nb;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  auto* yy = static_cast<uint8_t*>(y);
  auto* ys = static_cast<uint8_t*>(y_scale);
  if (x_f32)
    hipLaunchKernelGGL(f8::k_quant_rows<true>, dim3(grid), dim3(256), 0, as_stream(stream), x, ldx, rows, nb, relu,
                       row_group, row_group_stride, row_offset, yy, ldy, ys, ldy_scale * 4);
  else
    hipLaunchKernelGGL(f8::k_quant_rows<false>, dim3(grid), dim3(256), 0, as_stream(stream), x, ldx, rows, nb, relu,
                       row_group, row_group_stride, row_offset, yy, ldy, ys, ldy_scale * 4);
  return check_launch("quant_fp8");
}

extern "C" int i2pc_layernorm_fp8(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps,
                                  int rows, int dim, void* y, int64_t ldy, void* y_scale, int64_t ldy_scale,
                                  void* stream) {
  clear_error();
  I2PC_REQUIRE(x && gamma && beta && y && y_scale, "NULL pointer");
  I2PC_REQUIRE(rows > 0 && dim % 256 == 0 && dim >= 256 && dim <= 2048, "layernorm_fp8: dim %% 256 == 0, <= 2048 (dim=%d)", dim);
  I2PC_REQUIRE(ldx % 4 == 0 && ldy % 16 == 0 && ldy_scale * 128 >= dim, "layernorm_fp8: strides");
  const int V = dim / 256;
  dim3 grid((rows + 3) / 4), block(256);
  hipStream_t s = as_stream(stream);
  auto* yy = static_cast<uint8_t*>(y);
  auto* ys = static_cast<uint8_t*>(y_scale);
  const int64_t lds = ldy_scale * 4;
  switch (V) {
    case 1: hipLaunchKernelGGL(f8::k_layernorm_fp8<1>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, ys, lds); break;
    case 2: hipLaunchKernelGGL(f8::k_layernorm_fp8<2>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, ys, lds); break;
    case 3: hipLaunchKernelGGL(f8::k_layernorm_fp8<3>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, ys, lds); break;
    case 4: hipLaunchKernelGGL(f8::k_layernorm_fp8<4>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, ys, lds); break;
    case 5: hipLaunchKernelGGL(f8::k_layernorm_fp8<5>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, ys, lds); break;
    case 6: hipLaunchKernelGGL(f8::k_layernorm_fp8<6>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, ys, lds); break;
    case 7: hipLaunchKernelGGL(f8::k_layernorm_fp8<7>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, ys, lds); break;
    default: hipLaunchKernelGGL(f8::k_layernorm_fp8<8>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, ys, lds); break;
  }
  return check_launch("layernorm_fp8");
}

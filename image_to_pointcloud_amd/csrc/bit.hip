// BiT-ResNet stem of DPT-Hybrid (transformers modeling_bit.py, called from
// modeling_dpt.py:89-182) on gfx950, NHWC bf16.  The convolutions themselves run on the
// MFMA GEMM engine (weight standardisation is folded into the weights at load); this file
// holds the memory-bound glue around them:
//   k_stem_im2col : 7x7 stride-2 "SAME" stem conv input (BitEmbeddings.convolution,
//                   modeling_bit.py:234-241, DynamicPad2d :148-196) as bf16 GEMM rows
//                   [pixel][(ky, kx, c) padded to a multiple of 64]
//   k_gn_stats    : GroupNorm statistics (nn.functional.group_norm, modeling_bit.py:142-146):
//                   per (image, group) sum and sum of squares, fp32 per workgroup, fp64 atomics
//   k_gn_apply    : y = act(gn(x) + shortcut), shortcut = none | bf16 | gn(r) of a second map
//                   (BitBottleneckLayer.forward, modeling_bit.py:429-447)
//   k_maxpool     : 3x3 stride-2 max pool after dynamic SAME padding with value 0
//                   (BitMaxPool2d, modeling_bit.py:199-223)
#include "common.h"

#include <algorithm>

namespace i2pc {
namespace bit {

typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ bf16_t f2bf(float x) {
  __bf16 b = (__bf16)x;
  return *reinterpret_cast<bf16_t*>(&b);
}

// out[m][k] for m = (b, oy, ox), k = (ky * 7 + kx) * 3 + c (< 147, zero beyond): input pixel
// (oy * 2 - pt + ky, ox * 2 - pl + kx) of channel c, zero outside the image
__global__ __launch_bounds__(256) void k_stem_im2col(const float* __restrict__ x, int B, int H, int W, int OH, int OW,
                                                     int pt, int pl, int ks, int kp, bf16_t* __restrict__ out) {
  const int KK = ks * ks * 3;
  const int64_t total = (int64_t)B * OH * OW * (kp / 8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / (kp / 8);
    const int k0 = (int)(i - m * (kp / 8)) * 8;
    const int b = (int)(m / ((int64_t)OH * OW));
    const int rem = (int)(m - (int64_t)b * OH * OW);
    const int oy = rem / OW, ox = rem - (rem / OW) * OW;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      float v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = k0 + e + h;
        v[h] = 0.f;
        if (k < KK) {
          const int tap = k / 3, c = k - tap * 3;
          const int ky = tap / ks, kx = tap - ky * ks;
          const int iy = oy * 2 - pt + ky, ix = ox * 2 - pl + kx;
          if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
            v[h] = x[(((int64_t)b * 3 + c) * H + iy) * W + ix];
        }
      }
      w[e / 2] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    }
    *reinterpret_cast<uint4*>(out + m * kp + k0) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// One workgroup = one image x PIX pixels; thread t owns 8 consecutive channels of pixels
// t / (C / 8) + j * (256 / (C / 8)).  Per-channel partial sums reduce through LDS, then one
// thread per group adds them to the fp64 accumulators acc[b][g][2].
constexpr int PIX = 128;
__global__ __launch_bounds__(256) void k_gn_stats(const bf16_t* __restrict__ x, int HW, int C, int G,
                                                  double* __restrict__ acc) {
  __shared__ float ss[2][1024];
  const int chunks = C / 8;
  const int per_it = 256 / chunks;                 // pixels per iteration (C <= 2048)
  const int tiles = (HW + PIX - 1) / PIX;
  const int b = blockIdx.x / tiles;
  const int p0 = (blockIdx.x - b * tiles) * PIX;
  const int ch = (threadIdx.x % chunks) * 8;
  const int pl = threadIdx.x / chunks;
  float s[8] = {}, q[8] = {};
  if (pl < per_it) {
    const bf16_t* xb = x + (int64_t)b * HW * C;
    for (int p = p0 + pl; p < min(p0 + PIX, HW); p += per_it) {
      const uint4 u = *reinterpret_cast<const uint4*>(xb + (int64_t)p * C + ch);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = __uint_as_float(w[e] << 16), c = __uint_as_float(w[e] & 0xffff0000u);
        s[2 * e] += a; q[2 * e] += a * a;
        s[2 * e + 1] += c; q[2 * e + 1] += c * c;
      }
    }
  }
  for (int i = threadIdx.x; i < 2 * 1024; i += 256) (&ss[0][0])[i] = 0.f;
  __syncthreads();
  if (pl < per_it) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      atomicAdd(&ss[0][ch + e], s[e]);
      atomicAdd(&ss[1][ch + e], q[e]);
    }
  }
  __syncthreads();
  const int cg = C / G;
  for (int g = threadIdx.x; g < G; g += 256) {
    double a = 0.0, c = 0.0;
    for (int k = 0; k < cg; ++k) { a += ss[0][g * cg + k]; c += ss[1][g * cg + k]; }
    atomicAdd(&acc[((int64_t)b * G + g) * 2], a);
    atomicAdd(&acc[((int64_t)b * G + g) * 2 + 1], c);
  }
}

struct GnOperand {
  const bf16_t* x;
  const double* acc;        // [B][G][2] sums (null: x is used raw)
  const float* gamma;
  const float* beta;
};

__device__ __forceinline__ void gn_load(const GnOperand& o, int64_t off, int b, int c0, int C, int G, float inv_n,
                                        float eps, float v[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(o.x + off);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(w[e] << 16);
    v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
  if (!o.acc) return;
  const int cg = C / G;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    const int g = c / cg;
    const double sum = o.acc[((int64_t)b * G + g) * 2], sq = o.acc[((int64_t)b * G + g) * 2 + 1];
    const double mean = sum * inv_n;
    const double var = fmax(sq * inv_n - mean * mean, 0.0);
    const float rstd = 1.0f / sqrtf((float)var + eps);
    v[e] = (v[e] - (float)mean) * rstd * o.gamma[c] + o.beta[c];
  }
}

__global__ __launch_bounds__(256) void k_gn_apply(GnOperand a, GnOperand r, int has_r, int B, int HW, int C, int G,
                                                  float eps, int relu, bf16_t* __restrict__ y) {
  const int64_t total = (int64_t)B * HW * (C / 8);
  const float inv_n = 1.0f / ((float)HW * (float)(C / G));
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t off = i * 8;
    const int c0 = (int)(off % C);
    const int b = (int)(off / ((int64_t)HW * C));
    float v[8], w[8];
    gn_load(a, off, b, c0, C, G, inv_n, eps, v);
    if (has_r) {
      gn_load(r, off, b, c0, C, G, inv_n, eps, w);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += w[e];
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    uint4 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(y + off) = o;
  }
}

// 3x3 stride-2 max over the zero-padded map (pad pt top / pl left, zero beyond the
// bottom/right edge as DynamicPad2d pads there), 8 channels per thread
__global__ __launch_bounds__(256) void k_maxpool(const bf16_t* __restrict__ x, int B, int H, int W, int C, int OH, int OW,
                                                 int pt, int pl, bf16_t* __restrict__ y) {
  const int cv = C / 8;
  const int64_t total = (int64_t)B * OH * OW * cv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cv) * 8;
    const int64_t pix = i / cv;
    const int b = (int)(pix / ((int64_t)OH * OW));
    const int rem = (int)(pix - (int64_t)b * OH * OW);
    const int oy = rem / OW, ox = rem - (rem / OW) * OW;
    float m[8];
    bool any_pad = false;
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    for (int ky = 0; ky < 3; ++ky)
      for (int kx = 0; kx < 3; ++kx) {
        const int iy = oy * 2 - pt + ky, ix = ox * 2 - pl + kx;
        if ((unsigned)iy >= (unsigned)H || (unsigned)ix >= (unsigned)W) { any_pad = true; continue; }
        const uint4 u = *reinterpret_cast<const uint4*>(x + (((int64_t)b * H + iy) * W + ix) * C + c0);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          m[2 * e] = fmaxf(m[2 * e], __uint_as_float(w[e] << 16));
          m[2 * e + 1] = fmaxf(m[2 * e + 1], __uint_as_float(w[e] & 0xffff0000u));
        }
      }
    if (any_pad) {
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], 0.f);
    }
    uint4 o;
    o.x = (uint32_t)f2bf(m[0]) | ((uint32_t)f2bf(m[1]) << 16);
    o.y = (uint32_t)f2bf(m[2]) | ((uint32_t)f2bf(m[3]) << 16);
    o.z = (uint32_t)f2bf(m[4]) | ((uint32_t)f2bf(m[5]) << 16);
    o.w = (uint32_t)f2bf(m[6]) | ((uint32_t)f2bf(m[7]) << 16);
    *reinterpret_cast<uint4*>(y + pix * C + c0) = o;
  }
}

static int grid_for(int64_t work) { return (int)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 16384)); }

}  // namespace bit
}  // namespace i2pc

using namespace i2pc;
using namespace i2pc::bit;

extern "C" int i2pc_bit_stem_im2col(const float* pixels, int batch, int h, int w, int out_h, int out_w, int pad_top,
                                    int pad_left, int ksize, int k_pitch, void* out, void* stream) {
  clear_error();
  I2PC_REQUIRE(pixels && out && batch > 0 && h > 0 && w > 0 && out_h > 0 && out_w > 0, "bad arguments");
  I2PC_REQUIRE(k_pitch % 8 == 0 && k_pitch >= ksize * ksize * 3, "k_pitch %d must be >= %d and %% 8", k_pitch, ksize * ksize * 3);
  const int64_t work = (int64_t)batch * out_h * out_w * (k_pitch / 8);
  hipLaunchKernelGGL(k_stem_im2col, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), pixels, batch, h, w, out_h,
                     out_w, pad_top, pad_left, ksize, k_pitch, static_cast<bf16_t*>(out));
  return check_launch("bit_stem_im2col");
}

extern "C" int i2pc_groupnorm_stats(const void* x, int batch, int hw, int c, int groups, double* acc, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && acc && batch > 0 && hw > 0, "bad arguments");
  I2PC_REQUIRE(c % 8 == 0 && c <= 1024 && groups > 0 && c % groups == 0, "groupnorm: C=%d (%% 8, <= 1024) / groups %d", c, groups);
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(acc, 0, sizeof(double) * 2 * batch * groups, s) != hipSuccess) return set_error(I2PC_ELAUNCH, "memset failed");
  const int tiles = (hw + PIX - 1) / PIX;
  hipLaunchKernelGGL(k_gn_stats, dim3(batch * tiles), dim3(256), 0, s, static_cast<const bf16_t*>(x), hw, c, groups, acc);
  return check_launch("groupnorm_stats");
}

extern "C" int i2pc_groupnorm_apply(const void* x, const double* acc, const float* gamma, const float* beta,
                                    const void* r, const double* r_acc, const float* r_gamma, const float* r_beta,
                                    int batch, int hw, int c, int groups, float eps, int relu, void* y, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && y && batch > 0 && hw > 0 && c % 8 == 0 && groups > 0 && c % groups == 0, "bad arguments");
  I2PC_REQUIRE(!acc || (gamma && beta), "groupnorm: gamma/beta required with statistics");
  I2PC_REQUIRE(!r_acc || (r && r_gamma && r_beta), "groupnorm: shortcut gamma/beta required with its statistics");
  GnOperand a{static_cast<const bf16_t*>(x), acc, gamma, beta};
  GnOperand rr{static_cast<const bf16_t*>(r), r_acc, r_gamma, r_beta};
  const int64_t work = (int64_t)batch * hw * (c / 8);
  hipLaunchKernelGGL(k_gn_apply, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), a, rr, r ? 1 : 0, batch, hw, c,
                     groups, eps, relu, static_cast<bf16_t*>(y));
  return check_launch("groupnorm_apply");
}

extern "C" int i2pc_maxpool3s2(const void* x, int batch, int h, int w, int c, int out_h, int out_w, int pad_top,
                               int pad_left, void* y, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && y && batch > 0 && h > 0 && w > 0 && c % 8 == 0 && out_h > 0 && out_w > 0, "bad arguments");
  const int64_t work = (int64_t)batch * out_h * out_w * (c / 8);
  hipLaunchKernelGGL(k_maxpool, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), static_cast<const bf16_t*>(x), batch,
                     h, w, c, out_h, out_w, pad_top, pad_left, static_cast<bf16_t*>(y));
  return check_launch("maxpool3s2");
}

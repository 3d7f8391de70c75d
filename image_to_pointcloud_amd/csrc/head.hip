// Fused DPT depth head tail on MI355X:
//   bilinear resize (align_corners=True) of the head's first conv output to (H, W)
//   -> 3x3 conv C -> 32 + bias + ReLU -> 1x1 conv 32 -> 1 + bias + ReLU -> depth fp32.
// (transformers DPTDepthEstimationHead / DepthAnythingDepthEstimationHead: head[1..5],
//  modeling_dpt.py:679-716.)  Unfused, the resize writes a C-channel map at (H, W) in bf16
// (1.2 GB for DPT-Large at B=32) that the im2col conv then reads nine times.  Here a
// workgroup builds the resized halo of its 8 x 32 output tile straight into LDS (64
// channels at a time), with the same index rules and arithmetic as k_resize (bf16 rounding
// included), and runs the conv on the MFMA cores:
//   v_mfma_f32_16x16x32_bf16, A = 16 halo pixels x 32 channels (ds_read_b128, 16-B chunk
//   index XOR (pixel & 7): conflict-free), B = 32 channels x 16 output channels from the
//   LDS weight slice (chunk XOR (co & 7)); each wave owns 2 output rows = 4 m-tiles x 2 n-tiles.
// The epilogue rounds relu(acc + b2) to bf16 (the unfused conv stores bf16), multiplies by
// the 1x1 weights, reduces the 32 channels across lanes, adds b4 and applies ReLU.
#include "common.h"

#include <algorithm>

namespace i2pc {
namespace head {

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTileH = 8, kTileW = 32;              // output pixels per workgroup
constexpr int kHaloH = kTileH + 2, kHaloW = kTileW + 2;
constexpr int kChunk = 64;                          // input channels per LDS pass
constexpr int kCo = 32;
constexpr int kHaloBytes = kHaloH * kHaloW * kChunk * 2;   // 43,520
constexpr int kWBytes = kCo * 9 * kChunk * 2;               // 36,864

__device__ __forceinline__ bf16_t f2bf(float x) {
  __bf16 b = (__bf16)x;
  return *reinterpret_cast<bf16_t*>(&b);
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 per pair (RNE, as the scalar conversions)
__device__ __forceinline__ uint32_t pack2(f32x2 v) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2)); }
// the two bf16 of a dword as floats
__device__ __forceinline__ f32x2 unpack2(uint32_t u) {
  return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}

__global__ __launch_bounds__(256, 2) void k_head_upconv(const bf16_t* __restrict__ x, int h, int w, int C, int H,
                                                        int W, int tiles_w, int tiles_h,
                                                        const bf16_t* __restrict__ w2, const float* __restrict__ b2,
                                                        const float* __restrict__ w4, float b4,
                                                        float* __restrict__ depth) {
  __shared__ __attribute__((aligned(16))) uint8_t s_halo[kHaloBytes];
  __shared__ __attribute__((aligned(16))) uint8_t s_w[kWBytes];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int bid = blockIdx.x;
  const int tx = bid % tiles_w;
  bid /= tiles_w;
  const int ty = bid % tiles_h;
  const int b = bid / tiles_h;
  const int oy0 = ty * kTileH, ox0 = tx * kTileW;
  // k_resize's source-index rules (align_corners=True)
  const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  const bf16_t* xb = x + (int64_t)b * h * w * C;

  f32x4 acc[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[j][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = 0; c0 < C; c0 += kChunk) {
    // resized halo: (kHaloH * kHaloW) pixels x 8 chunks of 8 channels, four items per thread
    // in flight (all loads unconditional at clamped coordinates; padding is selected after)
    constexpr int kItems = kHaloH * kHaloW * 8;
    constexpr int kIter = (kItems + 255) / 256;
    for (int i0 = 0; i0 < kIter; i0 += 4) {
      uint4 q[4][4];
      float wy[4], wx[4];
      bool inside[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int it = min((i0 + u) * 256 + (int)threadIdx.x, kItems - 1);
        const int pix = it >> 3, c8 = it & 7;
        const int hy = oy0 - 1 + pix / kHaloW, hx = ox0 - 1 + pix % kHaloW;
        inside[u] = hy >= 0 && hy < H && hx >= 0 && hx < W;
        const float fy = sh * min(max(hy, 0), H - 1), fx = sw * min(max(hx, 0), W - 1);
        const int y0 = (int)fy, xx0 = (int)fx;
        const int y1 = y0 + (y0 < h - 1 ? 1 : 0), xx1 = xx0 + (xx0 < w - 1 ? 1 : 0);
        wy[u] = fy - y0;
        wx[u] = fx - xx0;
        const bf16_t* base = xb + c0 + c8 * 8;
        q[u][0] = *reinterpret_cast<const uint4*>(base + ((int64_t)y0 * w + xx0) * C);
        q[u][1] = *reinterpret_cast<const uint4*>(base + ((int64_t)y0 * w + xx1) * C);
        q[u][2] = *reinterpret_cast<const uint4*>(base + ((int64_t)y1 * w + xx0) * C);
        q[u][3] = *reinterpret_cast<const uint4*>(base + ((int64_t)y1 * w + xx1) * C);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int it = (i0 + u) * 256 + (int)threadIdx.x;
        if (it >= kItems) break;
        const int pix = it >> 3, c8 = it & 7;
        const float ly1 = wy[u], lx1 = wx[u];
        const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
        const uint32_t* p00 = reinterpret_cast<const uint32_t*>(&q[u][0]);
        const uint32_t* p01 = reinterpret_cast<const uint32_t*>(&q[u][1]);
        const uint32_t* p10 = reinterpret_cast<const uint32_t*>(&q[u][2]);
        const uint32_t* p11 = reinterpret_cast<const uint32_t*>(&q[u][3]);
        uint4 out;
        uint32_t* po = reinterpret_cast<uint32_t*>(&out);
        // channel pairs on the packed FP32 pipe (v_pk_mul/v_pk_fma): half the VALU issue
        const f32x2 vx0 = {lx0, lx0}, vx1 = {lx1, lx1}, vy0 = {ly0, ly0}, vy1 = {ly1, ly1};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2 t0 = __builtin_elementwise_fma(vx1, unpack2(p01[k]), vx0 * unpack2(p00[k]));
          const f32x2 t1 = __builtin_elementwise_fma(vx1, unpack2(p11[k]), vx0 * unpack2(p10[k]));
          const f32x2 r = __builtin_elementwise_fma(vy1, t1, vy0 * t0);
          po[k] = inside[u] ? pack2(r) : 0u;
        }
        *reinterpret_cast<uint4*>(s_halo + pix * 128 + ((c8 ^ (pix & 7)) << 4)) = out;
      }
    }
    // weight slice [co][tap][64 channels]: 9 loads per thread issued together
    {
      uint4 wv9[9];
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        const int it = u * 256 + threadIdx.x;
        const int c8 = it & 7, rest = it >> 3;
        const int tap = rest % 9, co = rest / 9;
        wv9[u] = *reinterpret_cast<const uint4*>(w2 + ((int64_t)co * 9 + tap) * C + c0 + c8 * 8);
      }
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        const int it = u * 256 + threadIdx.x;
        const int c8 = it & 7, rest = it >> 3;
        const int tap = rest % 9, co = rest / 9;
        *reinterpret_cast<uint4*>(s_w + (co * 9 + tap) * 128 + ((c8 ^ (co & 7)) << 4)) = wv9[u];
      }
    }
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap % 3;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c8 = kk * 4 + (lane >> 4);
        bf16x8 bw[2];
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int co = 16 * n + (lane & 15);
          bw[n] = *reinterpret_cast<const bf16x8*>(s_w + (co * 9 + tap) * 128 + ((c8 ^ (co & 7)) << 4));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 2 * wid + (j >> 1), c = 16 * (j & 1) + (lane & 15);
          const int pix = (r + dy) * kHaloW + (c + dx);
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(s_halo + pix * 128 + ((c8 ^ (pix & 7)) << 4));
#pragma unroll
          for (int n = 0; n < 2; ++n) acc[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[n], acc[j][n], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // epilogue: lane holds output channel co = 16 n + (lane & 15) of pixels 4 (lane >> 4) + e
  float bias[2], wv[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    bias[n] = b2[16 * n + (lane & 15)];
    wv[n] = w4[16 * n + (lane & 15)];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float s[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = 0.f;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float v = fmaxf(acc[j][n][e] + bias[n], 0.f);
        t += __uint_as_float((uint32_t)f2bf(v) << 16) * wv[n];
      }
      s[e] = t;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int e = 0; e < 4; ++e) s[e] += __shfl_xor(s[e], o);
    if ((lane & 15) == 0) {
      const int r = 2 * wid + (j >> 1);
      const int oy = oy0 + r;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ox = ox0 + 16 * (j & 1) + 4 * (lane >> 4) + e;
        if (oy < H && ox < W) depth[((int64_t)b * H + oy) * W + ox] = fmaxf(s[e] + b4, 0.f);
      }
    }
  }
}

}  // namespace head
}  // namespace i2pc

using namespace i2pc;

extern "C" int i2pc_head_upconv(const void* x, int batch, int h, int w, int c, int out_h, int out_w, const void* w2,
                                const float* b2, const float* w4, float b4, float* depth, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && w2 && b2 && w4 && depth, "head_upconv: NULL pointer");
  I2PC_REQUIRE(batch > 0 && h > 0 && w > 0 && out_h > 0 && out_w > 0, "head_upconv: empty shape");
  I2PC_REQUIRE(c > 0 && c % head::kChunk == 0, "head_upconv: channels %d must be a multiple of %d", c, head::kChunk);
  I2PC_REQUIRE((int64_t)batch * h * w * c < (1ll << 31) && (int64_t)batch * out_h * out_w < (1ll << 31),
               "head_upconv: tensor too large");
  const int tw = (out_w + head::kTileW - 1) / head::kTileW, th = (out_h + head::kTileH - 1) / head::kTileH;
  const int64_t blocks = (int64_t)batch * tw * th;
  I2PC_REQUIRE(blocks < (1ll << 31), "head_upconv: grid too large");
  hipLaunchKernelGGL(head::k_head_upconv, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     static_cast<const uint16_t*>(x), h, w, c, out_h, out_w, tw, th, static_cast<const uint16_t*>(w2),
                     b2, w4, b4, depth);
  return check_launch("head_upconv");
}

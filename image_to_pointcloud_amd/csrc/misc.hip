// Memory-bound helpers of the depth network (gfx950): LayerNorm, bilinear 2x
// upsample (align_corners=True), ViT stem CLS/pos row, fp32->bf16, head output.
// All are HBM-bound: 16-byte vector loads/stores, one wave per row where a row
// reduction is needed.
#include "common.h"
#include "mx.h"

#include <cstdlib>

#include <algorithm>
#include <cstring>

namespace i2pc {
namespace misc {

typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ bf16_t f2bf(float x) {
  __bf16 b = (__bf16)x;
  return *reinterpret_cast<bf16_t*>(&b);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) { return pk2bf(a, b); }

__device__ __forceinline__ float wave_sum(float x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// one wave per row, D/256 float4 per lane held in registers (two-pass variance)
template <int V>
__global__ __launch_bounds__(256) void k_layernorm(const float* __restrict__ x, int64_t ldx,
                                                   const float* __restrict__ g, const float* __restrict__ b,
                                                   float eps, int rows, int dim, bf16_t* __restrict__ y, int64_t ldy,
                                                   float* __restrict__ mean_out) {
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
  if (mean_out && lane == 0) mean_out[row] = mean;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float a = v[i].x - mean, c = v[i].y - mean, d = v[i].z - mean, e = v[i].w - mean;
    q += (a * a + c * c) + (d * d + e * e);
  }
  const float var = wave_sum(q) / (float)dim;
  const float rstd = 1.0f / sqrtf(var + eps);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  uint2* yr = reinterpret_cast<uint2*>(y + row * ldy);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float4 gg = g4[i * 64 + lane], bb = b4[i * 64 + lane];
    uint2 o;
    o.x = pack2((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y);
    o.y = pack2((v[i].z - mean) * rstd * gg.z + bb.z, (v[i].w - mean) * rstd * gg.w + bb.w);
    yr[i * 64 + lane] = o;
  }
}

// dim % 128 == 0 but not % 256 (Depth-Anything-V2-Small's 384): one wave per row, V float2 per
// lane, every load unconditional and in flight together (k_layernorm_any's runtime-bounded loop
// predicates each load and waits for it: 3.7 TB/s at dim 384)
template <int V>
__global__ __launch_bounds__(256) void k_layernorm2(const float* __restrict__ x, int64_t ldx,
                                                    const float* __restrict__ g, const float* __restrict__ b,
                                                    float eps, int rows, int dim, bf16_t* __restrict__ y, int64_t ldy,
                                                   float* __restrict__ mean_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float2* xr = reinterpret_cast<const float2*>(x + row * ldx);
  float2 v[V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = xr[i * 64 + lane];
#pragma unroll
  for (int i = 0; i < V; ++i) s += v[i].x + v[i].y;
  const float mean = wave_sum(s) / (float)dim;
  if (mean_out && lane == 0) mean_out[row] = mean;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float a = v[i].x - mean, c = v[i].y - mean;
    q += a * a + c * c;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)dim + eps);
  const float2* g2 = reinterpret_cast<const float2*>(g);
  const float2* b2 = reinterpret_cast<const float2*>(b);
  uint32_t* yr = reinterpret_cast<uint32_t*>(y + row * ldy);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float2 gg = g2[i * 64 + lane], bb = b2[i * 64 + lane];
    yr[i * 64 + lane] = pack2((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y);
  }
}

// generic row width (dim % 64 == 0, dim <= 2048): E scalars per lane, stride 64 (coalesced)
__global__ __launch_bounds__(256) void k_layernorm_any(const float* __restrict__ x, int64_t ldx,
                                                       const float* __restrict__ g, const float* __restrict__ b,
                                                       float eps, int rows, int dim, bf16_t* __restrict__ y, int64_t ldy,
                                                   float* __restrict__ mean_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int E = dim / 64;
  const float* xr = x + row * ldx;
  float v[32];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    v[i] = i < E ? xr[i * 64 + lane] : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)dim;
  if (mean_out && lane == 0) mean_out[row] = mean;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i)
    if (i < E) { const float a = v[i] - mean; q += a * a; }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)dim + eps);
  bf16_t* yr = y + row * ldy;
#pragma unroll
  for (int i = 0; i < 32; ++i)
    if (i < E) yr[i * 64 + lane] = f2bf((v[i] - mean) * rstd * g[i * 64 + lane] + b[i * 64 + lane]);
}

// NHWC bf16, 8 channels (16 B) per thread; torch upsample_bilinear2d, align_corners=True.
// Bilinear resize of an NHWC bf16 map to (H, W) with torch's upsample_bilinear2d
// source-index rules (float scale; align_corners: s = (in-1)/(out-1) * dst, else
// s = max(in/out * (dst + 0.5) - 0.5, 0)); 8 channels per lane (16 B loads).
// I: the flat index type -- uint32_t whenever B*H*W*c/8 < 2^31 (every DPT map), so the three
// index divisions per 16-B output are 32-bit instead of the emulated 64-bit sequences that made
// this kernel VALU-bound (2.1-2.6 TB/s)
template <typename I>
__global__ __launch_bounds__(256) void k_resize(const bf16_t* __restrict__ x, int B, int h, int w, int c, int H, int W,
                                                int align, const bf16_t* __restrict__ add, bf16_t* __restrict__ y) {
  const I cv = (I)(c / 8);
  const I total = (I)B * (I)H * (I)W * cv;
  float sh, sw;
  if (align) {
    sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
    sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  } else {
    sh = (float)h / (float)H;
    sw = (float)w / (float)W;
  }
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cv);
    I pix = i / cv;
    const int ox = (int)(pix % (I)W);
    pix /= (I)W;
    const int oy = (int)(pix % (I)H);
    const int b = (int)(pix / (I)H);
    const float fy = align ? sh * oy : fmaxf(sh * (oy + 0.5f) - 0.5f, 0.f);
    const float fx = align ? sw * ox : fmaxf(sw * (ox + 0.5f) - 0.5f, 0.f);
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly1 = fy - y0, lx1 = fx - x0;
    const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
const bf16_t* base = x + (int64_t)b * h * w * c + ch * 8;
    const uint4 a00 = *reinterpret_cast<const uint4*>(base + ((int64_t)y0 * w + x0) * c);
    const uint4 a01 = *reinterpret_cast<const uint4*>(base + ((int64_t)y0 * w + x1) * c);
    const uint4 a10 = *reinterpret_cast<const uint4*>(base + ((int64_t)y1 * w + x0) * c);
    const uint4 a11 = *reinterpret_cast<const uint4*>(base + ((int64_t)y1 * w + x1) * c);
    const uint32_t* p00 = reinterpret_cast<const uint32_t*>(&a00);
    const uint32_t* p01 = reinterpret_cast<const uint32_t*>(&a01);
    const uint32_t* p10 = reinterpret_cast<const uint32_t*>(&a10);
    const uint32_t* p11 = reinterpret_cast<const uint32_t*>(&a11);
    uint4 addv = make_uint4(0, 0, 0, 0);
    if (add) addv = *reinterpret_cast<const uint4*>(add + (int64_t)i * 8);
    const uint32_t* pa = reinterpret_cast<const uint32_t*>(&addv);
    uint4 out;
    uint32_t* po = reinterpret_cast<uint32_t*>(&out);
    // channel pairs on the packed FP32 pipe; one cvt_pk_bf16 per pair
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    auto g2 = [](uint32_t u) { return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)}; };
    const f32x2 vx0 = {lx0, lx0}, vx1 = {lx1, lx1}, vy0 = {ly0, ly0}, vy1 = {ly1, ly1};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x2 t0 = __builtin_elementwise_fma(vx1, g2(p01[k]), vx0 * g2(p00[k]));
      const f32x2 t1 = __builtin_elementwise_fma(vx1, g2(p11[k]), vx0 * g2(p10[k]));
      f32x2 r = __builtin_elementwise_fma(vy1, t1, vy0 * t0);
      if (add) r += g2(pa[k]);
      po[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2));
    }
    *reinterpret_cast<uint4*>(y + (int64_t)i * 8) = out;
  }
}

// k_resize / k_upsample2x_fp8 mapped by output row (r05): a workgroup walks output rows (b, oy), and
// inside a row each thread keeps one 8-channel chunk (ch = thread % (c / 8), c a power of two) and
// steps over the pixels -- no per-output index divisions (≈ 20 VALU per value in the flat-index
// kernels, PMC), one row's vertical taps computed once, and every tap load lane-consecutive (the
// 32-channel-block form put 8 lanes 64 B apart).  Same arithmetic as k_resize (bit-identical).  F8:
// the block's four lanes (a quad) share the amax by DPP and write k_quant_rows' bytes.
template <bool F8>
__global__ __launch_bounds__(256) void k_resize_rowmap(const bf16_t* __restrict__ x, int B, int h, int w, int c,
                                                       int lgcv, int H, int W, int align,
                                                       const bf16_t* __restrict__ add, bf16_t* __restrict__ y,
                                                       uint8_t* __restrict__ y8, int64_t ldy8,
                                                       uint8_t* __restrict__ ys, int64_t ldys) {
  const int cv = 1 << lgcv;
  const int ch = threadIdx.x & (cv - 1);
  const int px0 = threadIdx.x >> lgcv, pstep = 256 >> lgcv;
  float sh, sw;
  if (align) {
    sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
    sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  } else {
    sh = (float)h / (float)H;
    sw = (float)w / (float)W;
  }
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  auto g2 = [](uint32_t u) { return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)}; };
  for (int row = blockIdx.x; row < B * H; row += gridDim.x) {
    const int b = row / H, oy = row - (row / H) * H;
    const float fy = align ? sh * oy : fmaxf(sh * (oy + 0.5f) - 0.5f, 0.f);
    const int y0 = (int)fy;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0);
    const float ly1 = fy - y0, ly0 = 1.f - ly1;
    const f32x2 vy0 = {ly0, ly0}, vy1 = {ly1, ly1};
    const bf16_t* r0 = x + ((int64_t)b * h + y0) * w * c + ch * 8;
    const bf16_t* r1 = x + ((int64_t)b * h + y1) * w * c + ch * 8;
    for (int ox = px0; ox < W; ox += pstep) {
      const float fx = align ? sw * ox : fmaxf(sw * (ox + 0.5f) - 0.5f, 0.f);
      const int x0 = (int)fx;
      const int x1 = x0 + (x0 < w - 1 ? 1 : 0);
      const float lx1 = fx - x0, lx0 = 1.f - lx1;
      const f32x2 vx0 = {lx0, lx0}, vx1 = {lx1, lx1};
      const uint4 a00 = *reinterpret_cast<const uint4*>(r0 + (int64_t)x0 * c);
      const uint4 a01 = *reinterpret_cast<const uint4*>(r0 + (int64_t)x1 * c);
      const uint4 a10 = *reinterpret_cast<const uint4*>(r1 + (int64_t)x0 * c);
      const uint4 a11 = *reinterpret_cast<const uint4*>(r1 + (int64_t)x1 * c);
      const int64_t o = ((int64_t)row * W + ox) * c + ch * 8;
      uint4 addv = make_uint4(0, 0, 0, 0);
      if (add) addv = *reinterpret_cast<const uint4*>(add + o);
      const uint32_t p00[4] = {a00.x, a00.y, a00.z, a00.w}, p01[4] = {a01.x, a01.y, a01.z, a01.w};
      const uint32_t p10[4] = {a10.x, a10.y, a10.z, a10.w}, p11[4] = {a11.x, a11.y, a11.z, a11.w};
      const uint32_t pa[4] = {addv.x, addv.y, addv.z, addv.w};
      uint32_t po[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x2 t0 = __builtin_elementwise_fma(vx1, g2(p01[k]), vx0 * g2(p00[k]));
        const f32x2 t1 = __builtin_elementwise_fma(vx1, g2(p11[k]), vx0 * g2(p10[k]));
        f32x2 r = __builtin_elementwise_fma(vy1, t1, vy0 * t0);
        if (add) r += g2(pa[k]);
        po[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2));
      }
      if constexpr (!F8) {
        *reinterpret_cast<uint4*>(y + o) = make_uint4(po[0], po[1], po[2], po[3]);
      } else {
        float v[8];
        float am = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] = __uint_as_float(po[k] << 16);
          v[2 * k + 1] = __uint_as_float(po[k] & 0xffff0000u);
          am = fmaxf(am, fmaxf(fabsf(v[2 * k]), fabsf(v[2 * k + 1])));
        }
        // the 32-channel block = this quad of lanes (ch & ~3 .. ch | 3): max by quad_perm xor 1, xor 2
        am = fmaxf(am, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(am), 0xB1, 0xF, 0xF, true)));
        am = fmaxf(am, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(am), 0x4E, 0xF, 0xF, true)));
        const int ex = ::i2pc::mx::mx_exponent(am);
        const float mul = ::i2pc::mx::exp2i(-ex);
        const int64_t pix = (int64_t)row * W + ox;
        *reinterpret_cast<uint2*>(y8 + pix * ldy8 + ch * 8) =
            make_uint2(::i2pc::mx::pack_e4m3(v[0] * mul, v[1] * mul, v[2] * mul, v[3] * mul),
                       ::i2pc::mx::pack_e4m3(v[4] * mul, v[5] * mul, v[6] * mul, v[7] * mul));
        if ((ch & 3) == 0) ys[pix * ldys + (ch >> 2)] = (uint8_t)(ex + 127);
      }
    }
  }
}

// 2x bilinear upsample (align_corners, as k_resize) written as MX fp8 rows -- i2pc_gemm_fp8's operand:
// e4m3 bytes [pixel][c] + one E8M0 scale byte per 32 channels (scale dwords [pixel][ldys / 4]).  One
// thread per (output pixel, 32-channel block): the four taps' 64-B runs, the same bf16 rounding of each
// value as k_resize, then the block quantised exactly as k_quant_rows quantises a bf16 row (so the bytes
// equal quant_fp8(upsample2x(x))) and stored as 32 B + 1 scale byte; the bf16 map is never written.
__global__ __launch_bounds__(256) void k_upsample2x_fp8(const bf16_t* __restrict__ x, int B, int h, int w, int c,
                                                        const bf16_t* __restrict__ add, uint8_t* __restrict__ y8,
                                                        int64_t ldy8, uint8_t* __restrict__ ys, int64_t ldys) {
  const int H = 2 * h, W = 2 * w;
  const uint32_t nb = (uint32_t)(c / 32);
  const uint32_t total = (uint32_t)B * (uint32_t)H * (uint32_t)W * nb;
  const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  auto g2 = [](uint32_t u) { return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)}; };
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int blk = (int)(i % nb);
    uint32_t pix = i / nb;
    const int ox = (int)(pix % (uint32_t)W);
    const uint32_t t = pix / (uint32_t)W;
    const int oy = (int)(t % (uint32_t)H);
    const int b = (int)(t / (uint32_t)H);
    const float fy = sh * oy, fx = sw * ox;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly1 = fy - y0, lx1 = fx - x0;
    const f32x2 vx0 = {1.f - lx1, 1.f - lx1}, vx1 = {lx1, lx1}, vy0 = {1.f - ly1, 1.f - ly1}, vy1 = {ly1, ly1};
    const bf16_t* base = x + (int64_t)b * h * w * c + blk * 32;
    const uint4* p00 = reinterpret_cast<const uint4*>(base + ((int64_t)y0 * w + x0) * c);
    const uint4* p01 = reinterpret_cast<const uint4*>(base + ((int64_t)y0 * w + x1) * c);
    const uint4* p10 = reinterpret_cast<const uint4*>(base + ((int64_t)y1 * w + x0) * c);
    const uint4* p11 = reinterpret_cast<const uint4*>(base + ((int64_t)y1 * w + x1) * c);
    const uint4* pa = add ? reinterpret_cast<const uint4*>(add + (int64_t)pix * c + blk * 32) : nullptr;
    float v[32];
    float am = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 a00 = p00[q], a01 = p01[q], a10 = p10[q], a11 = p11[q];
      const uint4 aa = pa ? pa[q] : make_uint4(0, 0, 0, 0);
      const uint32_t w00[4] = {a00.x, a00.y, a00.z, a00.w}, w01[4] = {a01.x, a01.y, a01.z, a01.w};
      const uint32_t w10[4] = {a10.x, a10.y, a10.z, a10.w}, w11[4] = {a11.x, a11.y, a11.z, a11.w};
      const uint32_t wa[4] = {aa.x, aa.y, aa.z, aa.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x2 t0 = __builtin_elementwise_fma(vx1, g2(w01[k]), vx0 * g2(w00[k]));
        const f32x2 t1 = __builtin_elementwise_fma(vx1, g2(w11[k]), vx0 * g2(w10[k]));
        f32x2 r = __builtin_elementwise_fma(vy1, t1, vy0 * t0);
        if (pa) r += g2(wa[k]);
        const f32x2 rb = g2(__builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2)));   // k_resize's bf16 value
        v[8 * q + 2 * k] = rb.x;
        v[8 * q + 2 * k + 1] = rb.y;
        am = fmaxf(am, fmaxf(fabsf(rb.x), fabsf(rb.y)));
      }
    }
    const int ex = ::i2pc::mx::mx_exponent(am);
    const float mul = ::i2pc::mx::exp2i(-ex);
    uint32_t d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      d[q] = ::i2pc::mx::pack_e4m3(v[4 * q] * mul, v[4 * q + 1] * mul, v[4 * q + 2] * mul, v[4 * q + 3] * mul);
    uint4* out = reinterpret_cast<uint4*>(y8 + (int64_t)pix * ldy8 + blk * 32);
    out[0] = make_uint4(d[0], d[1], d[2], d[3]);
    out[1] = make_uint4(d[4], d[5], d[6], d[7]);
    ys[(int64_t)pix * ldys + blk] = (uint8_t)(ex + 127);
  }
}

__global__ void k_cls_pos(const float* cls, const float* pos0, int B, int T, int D, float* x) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * D) return;
  const int b = i / D, d = i - b * D;
  x[(int64_t)b * T * D + d] = cls[d] + pos0[d];
}

__global__ void k_f32_to_bf16(const float4* __restrict__ x, int64_t n4, uint2* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    y[i] = make_uint2(pack2(v.x, v.y), pack2(v.z, v.w));
  }
}

// one thread per pixel: C (<= 64, multiple of 8) bf16 channels -> 1 fp32
__global__ __launch_bounds__(256) void k_head_out(const bf16_t* __restrict__ x, int64_t P, int C,
                                                  const float* __restrict__ w, float bias, float* __restrict__ d) {
  __shared__ float sw[64];
  if (threadIdx.x < C) sw[threadIdx.x] = w[threadIdx.x];
  __syncthreads();
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < P; p += (int64_t)gridDim.x * blockDim.x) {
    const uint4* src = reinterpret_cast<const uint4*>(x + p * C);
    float acc = 0.f;
    for (int k = 0; k < C / 8; ++k) {
      const uint4 u = src[k];
      const uint32_t* q = reinterpret_cast<const uint32_t*>(&u);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc += __uint_as_float(q[t] << 16) * sw[k * 8 + 2 * t];
        acc += __uint_as_float(q[t] & 0xffff0000u) * sw[k * 8 + 2 * t + 1];
      }
    }
    d[p] = fmaxf(acc + bias, 0.f);
  }
}

// Sum over the 16 lanes of a DPP row by one DPP move per step (lane ^ 1, lane ^ 2 inside a quad, then
// the half-row mirror 7 - i and the row mirror 15 - i, whose partners hold the other quad's / half's
// sum by then) instead of ds_bpermute round trips; every lane ends with the row's sum.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return v;
}

// LayerNorm row statistics from the cw-column chunk partials (cw = 64 or 32) an i2pc_gemm producer
// epilogue wrote ((mean, M2) per chunk of out - shift): Chan's combination for equal chunk counts,
// mean = avg(mean_c), M2 = sum M2_c + cw sum (mean_c - mean)^2, var = M2 / (cw P) (biased, as
// nn.LayerNorm), out = (rstd, -rstd * mean), shift_out = shift_in + mean.  16 lanes per row (coalesced 8-byte
// partials, partial c on lane c % 16).
// 64 rows per workgroup: each 16-lane row group takes four rows (16 apart), all of their loads issued
// before any reduction (r06; one row per group was a 1154-workgroup launch with one load per thread in
// flight, ~4.7 us for 2.4 MB).  Per row the same operations in the same order as before.
__global__ __launch_bounds__(256) void k_ln_rowstats(const float2* __restrict__ part, int rows, int P, float cw, float eps,
                                                     float2* __restrict__ out, const float* shift_in,
                                                     float* shift_out) {
  constexpr int RPT = 4;
  const int l = threadIdx.x & 15;
  float2 v[RPT][4];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = blockIdx.x * 64 + k * 16 + (threadIdx.x >> 4);
    const float2* q = part + (int64_t)(r < rows ? r : 0) * P;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[k][j] = (l + 16 * j < P) ? q[l + 16 * j] : make_float2(0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = blockIdx.x * 64 + k * 16 + (threadIdx.x >> 4);
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) sm += v[k][j].x;
    sm = row16_sum(sm);
    const float mean = sm / (float)P;
    float m2 = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (l + 16 * j < P) {
        const float d = v[k][j].x - mean;
        m2 += v[k][j].y + cw * d * d;
      }
    m2 = row16_sum(m2);
    if (r < rows && l == 0) {
      const float rstd = 1.0f / sqrtf(m2 / (cw * (float)P) + eps);
      out[r] = make_float2(rstd, -rstd * mean);
      if (shift_out) shift_out[r] = (shift_in ? shift_in[r] : 0.f) + mean;
    }
  }
}

// LayerNorm of a bf16 row block from its row statistics (i2pc_ln_apply): y = bf16(gamma * (rs.x * x +
// rs.y) + beta) with rs = (rstd, -rstd * mean) of the rows as ln_rowstats gives them (x = the shifted
// bf16 residual stream: the statistics were taken of the same shifted values).  8 columns per thread
// (one 16-B load and store), one workgroup row per matrix row.
__global__ __launch_bounds__(256) void k_ln_apply(const uint4* __restrict__ x, int64_t ldx8, const float2* __restrict__ rs,
                                                  const float4* __restrict__ gamma, const float4* __restrict__ beta,
                                                  int d8, uint4* __restrict__ y, int64_t ldy8) {
  // one 8-column group per thread: row r = blockIdx.y, group c = blockIdx.x * 256 + threadIdx.x
  const int r = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < d8) {
    const uint4 v = x[r * ldx8 + c];
    // the row statistics are rewritten by the k_ln_rowstats launch right before this one: read them
    // with agent-scope loads (sc1: past any non-coherent line another XCD's L2 may hold), by
    // construction rather than by the compiler's choice of a scalar load (the r04
    // two-process nondeterminism)
    const float* sp = reinterpret_cast<const float*>(rs + r);
    float2 s;
    s.x = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s.y = __hip_atomic_load(sp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float4 g0 = gamma[2 * c], g1 = gamma[2 * c + 1], b0 = beta[2 * c], b1 = beta[2 * c + 1];
    const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    const uint32_t q[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float lo = __builtin_fmaf(g[2 * t], __builtin_fmaf(__uint_as_float(q[t] << 16), s.x, s.y), b[2 * t]);
      const float hi = __builtin_fmaf(g[2 * t + 1], __builtin_fmaf(__uint_as_float(q[t] & 0xffff0000u), s.x, s.y), b[2 * t + 1]);
      o[t] = pk2bf(lo, hi);
    }
    y[r * ldy8 + c] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// DIAGNOSTIC (r05 root-cause of the r04 nondeterminism): the r04 grid-stride form, knob "ln_apply_gs".
__global__ __launch_bounds__(256) void k_ln_apply_gs(const uint4* __restrict__ x, int64_t ldx8, const float2* __restrict__ rs,
                                                     const float4* __restrict__ gamma, const float4* __restrict__ beta,
                                                     int rows, int d8, uint4* __restrict__ y, int64_t ldy8, int mode) {
  // mode 1: as r04; 2: agent-scope acquire fence first; 3: x and rs read by agent-scope relaxed atomic loads;
  // 4: the vector L1 of the CU invalidated first (buffer_inv sc0); 5: rs read by agent-scope loads only
  if (mode == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (mode == 4) asm volatile("buffer_inv sc0" ::: "memory");
  const int64_t n = (int64_t)rows * d8;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int r = (int)(i / d8);
    const int c = (int)(i - (int64_t)r * d8);
    uint4 v;
    float2 s;
    if (mode == 5) {
      v = x[r * ldx8 + c];
      const float* sp = reinterpret_cast<const float*>(rs + r);
      s.x = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s.y = __hip_atomic_load(sp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (mode == 3) {
      const uint32_t* xp = reinterpret_cast<const uint32_t*>(x + r * ldx8 + c);
      v.x = __hip_atomic_load(xp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v.y = __hip_atomic_load(xp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v.z = __hip_atomic_load(xp + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v.w = __hip_atomic_load(xp + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const float* sp = reinterpret_cast<const float*>(rs + r);
      s.x = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s.y = __hip_atomic_load(sp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      v = x[r * ldx8 + c];
      s = rs[r];
    }
    const float4 g0 = gamma[2 * c], g1 = gamma[2 * c + 1], b0 = beta[2 * c], b1 = beta[2 * c + 1];
    const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    const uint32_t q[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float lo = __builtin_fmaf(g[2 * t], __builtin_fmaf(__uint_as_float(q[t] << 16), s.x, s.y), b[2 * t]);
      const float hi = __builtin_fmaf(g[2 * t + 1], __builtin_fmaf(__uint_as_float(q[t] & 0xffff0000u), s.x, s.y), b[2 * t + 1]);
      o[t] = pk2bf(lo, hi);
    }
    y[r * ldy8 + c] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

static int grid_for(int64_t work, int per_block = 256) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((work + per_block - 1) / per_block, 256 * 16));
}

}  // namespace misc
}  // namespace i2pc

using namespace i2pc;
using namespace i2pc::misc;

static thread_local int g_ln2 = 1;   // "ln_f2": the float2 row kernel for dim 384
static thread_local int g_resize_rows = 1;   // "resize_rows": k_resize_rowmap where it applies (0 = the flat kernels)
static int pow2_log(int v) { return v > 0 && (v & (v - 1)) == 0 ? __builtin_ctz((unsigned)v) : -1; }
static thread_local int g_ln_apply_gs = 0;   // "ln_apply_gs": DIAGNOSTIC, the r04 grid-stride ln_apply

bool i2pc_misc_tune(const char* name, int value) {
  if (std::strcmp(name, "ln_f2") == 0) { g_ln2 = value; return true; }
  if (std::strcmp(name, "ln_apply_gs") == 0) { g_ln_apply_gs = value; return true; }
  if (std::strcmp(name, "resize_rows") == 0) { g_resize_rows = value; return true; }
  return false;
}

extern "C" int i2pc_ln_rowstats_w(const float* part, int rows, int parts, int chunk_cols, float eps, float* rows_out,
                                  const float* shift_in, float* shift_out, void* stream) {
  clear_error();
  I2PC_REQUIRE(part && rows_out, "NULL pointer");
  I2PC_REQUIRE(rows > 0 && parts >= 1 && parts <= 64, "ln_rowstats: parts=%d must be 1..64", parts);
  I2PC_REQUIRE(chunk_cols == 32 || chunk_cols == 64, "ln_rowstats: chunk_cols=%d must be 32 or 64", chunk_cols);
  hipLaunchKernelGGL(k_ln_rowstats, dim3((rows + 63) / 64), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float2*>(part), rows, parts, (float)chunk_cols, eps,
                     reinterpret_cast<float2*>(rows_out), shift_in, shift_out);
  return check_launch("ln_rowstats");
}

extern "C" int i2pc_ln_apply(const void* x, int64_t ldx, const float* rows_stats, const float* gamma, const float* beta,
                             int rows, int dim, void* y, int64_t ldy, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && rows_stats && gamma && beta && y, "NULL pointer");
  I2PC_REQUIRE(rows > 0 && dim > 0 && dim % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && ldx >= dim && ldy >= dim,
               "ln_apply: dim, ldx, ldy must be multiples of 8 (ld >= dim)");
  I2PC_REQUIRE((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) % 16 == 0 &&
                   (reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta)) % 16 == 0,
               "ln_apply: 16-byte aligned operands");
  const int d8 = dim / 8;
  if (g_ln_apply_gs) {
    hipLaunchKernelGGL(k_ln_apply_gs, dim3(grid_for((int64_t)rows * d8)), dim3(256), 0, as_stream(stream),
                       static_cast<const uint4*>(x), ldx / 8, reinterpret_cast<const float2*>(rows_stats),
                       reinterpret_cast<const float4*>(gamma), reinterpret_cast<const float4*>(beta), rows, d8,
                       static_cast<uint4*>(y), ldy / 8, g_ln_apply_gs);
    return check_launch("ln_apply");
  }
  for (int r0 = 0; r0 < rows; r0 += 65535) {   // (grid y <= 65535 rows per launch)
    const int nr = std::min(rows - r0, 65535);
    hipLaunchKernelGGL(k_ln_apply, dim3((d8 + 255) / 256, nr), dim3(256), 0, as_stream(stream),
                       static_cast<const uint4*>(x) + (int64_t)r0 * (ldx / 8), ldx / 8,
                       reinterpret_cast<const float2*>(rows_stats) + r0, reinterpret_cast<const float4*>(gamma),
                       reinterpret_cast<const float4*>(beta), d8, static_cast<uint4*>(y) + (int64_t)r0 * (ldy / 8),
                       ldy / 8);
  }
  return check_launch("ln_apply");
}

extern "C" int i2pc_ln_rowstats(const float* part, int rows, int parts, float eps, float* rows_out,
                                const float* shift_in, float* shift_out, void* stream) {
  return i2pc_ln_rowstats_w(part, rows, parts, 64, eps, rows_out, shift_in, shift_out, stream);
}

static int layernorm_impl(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps, int rows,
                          int dim, void* y, int64_t ldy, float* mean_out, void* stream);

extern "C" int i2pc_layernorm(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps,
                              int rows, int dim, void* y, int64_t ldy, void* stream) {
  clear_error();
  return layernorm_impl(x, ldx, gamma, beta, eps, rows, dim, y, ldy, nullptr, stream);
}

extern "C" int i2pc_layernorm_stats(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps,
                                    int rows, int dim, void* y, int64_t ldy, float* row_mean, void* stream) {
  clear_error();
  I2PC_REQUIRE(row_mean, "layernorm_stats: NULL row_mean");
  return layernorm_impl(x, ldx, gamma, beta, eps, rows, dim, y, ldy, row_mean, stream);
}

static int layernorm_impl(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps, int rows,
                          int dim, void* y, int64_t ldy, float* mean_out, void* stream) {
  I2PC_REQUIRE(x && gamma && beta && y, "NULL pointer");
  I2PC_REQUIRE(rows > 0 && dim > 0 && dim % 64 == 0 && dim <= 2048, "layernorm: dim=%d must be a multiple of 64 <= 2048", dim);
  I2PC_REQUIRE(ldx % 4 == 0 && ldy % 4 == 0, "layernorm: row strides must be multiples of 4");
  hipStream_t s = as_stream(stream);
  const dim3 grid((rows + 3) / 4), block(256);
  bf16_t* yy = static_cast<bf16_t*>(y);
  if (dim == 384 && g_ln2) {
    hipLaunchKernelGGL(k_layernorm2<3>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out);
    return check_launch("layernorm");
  }
  if (dim % 256 != 0) {
    hipLaunchKernelGGL(k_layernorm_any, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out);
    return check_launch("layernorm");
  }
  switch (dim / 256) {
    case 1: hipLaunchKernelGGL(k_layernorm<1>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out); break;
    case 2: hipLaunchKernelGGL(k_layernorm<2>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out); break;
    case 3: hipLaunchKernelGGL(k_layernorm<3>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out); break;
    case 4: hipLaunchKernelGGL(k_layernorm<4>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out); break;
    case 5: hipLaunchKernelGGL(k_layernorm<5>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out); break;
    case 6: hipLaunchKernelGGL(k_layernorm<6>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out); break;
    case 7: hipLaunchKernelGGL(k_layernorm<7>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out); break;
    case 8: hipLaunchKernelGGL(k_layernorm<8>, grid, block, 0, s, x, ldx, gamma, beta, eps, rows, dim, yy, ldy, mean_out); break;
  }
  return check_launch("layernorm");
}

extern "C" int i2pc_resize_bilinear(const void* x, int batch, int h, int w, int c, int out_h, int out_w,
                                    int align_corners, const void* add, void* y, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && y, "NULL pointer");
  I2PC_REQUIRE(batch > 0 && h > 0 && w > 0 && c > 0 && c % 8 == 0 && out_h > 0 && out_w > 0,
               "resize_bilinear: bad shape (c %% 8 == 0)");
  const int lgcv = pow2_log(c / 8);
  if (g_resize_rows && lgcv >= 0 && lgcv <= 8 && (int64_t)batch * out_h < (1ll << 31)) {
    const int rows = batch * out_h;
    hipLaunchKernelGGL(k_resize_rowmap<false>, dim3(std::min(rows, 16384)), dim3(256), 0, as_stream(stream),
                       static_cast<const bf16_t*>(x), batch, h, w, c, lgcv, out_h, out_w, align_corners ? 1 : 0,
                       static_cast<const bf16_t*>(add), static_cast<bf16_t*>(y), nullptr, 0, nullptr, 0);
    return check_launch("resize_bilinear");
  }
  const int64_t work = (int64_t)batch * out_h * out_w * (c / 8);
  // 32-bit indices when the flat index and its grid-stride successor stay below 2^31
  if (work + (int64_t)grid_for(work) * 256 < ((int64_t)1 << 31))
    hipLaunchKernelGGL(k_resize<uint32_t>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream),
                       static_cast<const bf16_t*>(x), batch, h, w, c, out_h, out_w, align_corners ? 1 : 0,
                       static_cast<const bf16_t*>(add), static_cast<bf16_t*>(y));
  else
    hipLaunchKernelGGL(k_resize<int64_t>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream),
                       static_cast<const bf16_t*>(x), batch, h, w, c, out_h, out_w, align_corners ? 1 : 0,
                       static_cast<const bf16_t*>(add), static_cast<bf16_t*>(y));
  return check_launch("resize_bilinear");
}

extern "C" int i2pc_upsample2x(const void* x, int batch, int h, int w, int c, const void* add, void* y, void* stream) {
  return i2pc_resize_bilinear(x, batch, h, w, c, 2 * h, 2 * w, 1, add, y, stream);
}

extern "C" int i2pc_upsample2x_fp8(const void* x, int batch, int h, int w, int c, const void* add, void* y, int64_t ldy,
                                   void* y_scale, int64_t ldy_scale, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && y && y_scale, "NULL pointer");
  I2PC_REQUIRE(batch > 0 && h > 0 && w > 0 && c > 0 && c % 32 == 0, "upsample2x_fp8: bad shape (c %% 32 == 0)");
  I2PC_REQUIRE(ldy % 16 == 0 && ldy >= c && ldy_scale * 128 >= c, "upsample2x_fp8: ldy %% 16, ldy >= c, ldy_scale >= c/128");
  const int H = 2 * h, W = 2 * w;
  const int64_t work = (int64_t)batch * H * W * (c / 32);
  I2PC_REQUIRE(work + (int64_t)grid_for(work) * 256 < ((int64_t)1 << 32), "upsample2x_fp8: map too large for 32-bit indexing");
  const int lgcv = pow2_log(c / 8);
  if (g_resize_rows && lgcv >= 2 && lgcv <= 8) {
    const int rows = batch * H;
    hipLaunchKernelGGL(k_resize_rowmap<true>, dim3(std::min(rows, 16384)), dim3(256), 0, as_stream(stream),
                       static_cast<const bf16_t*>(x), batch, h, w, c, lgcv, H, W, 1, static_cast<const bf16_t*>(add),
                       nullptr, static_cast<uint8_t*>(y), ldy, static_cast<uint8_t*>(y_scale), ldy_scale * 4);
    return check_launch("upsample2x_fp8");
  }
  hipLaunchKernelGGL(k_upsample2x_fp8, dim3(grid_for(work)), dim3(256), 0, as_stream(stream),
                     static_cast<const bf16_t*>(x), batch, h, w, c, static_cast<const bf16_t*>(add),
                     static_cast<uint8_t*>(y), ldy, static_cast<uint8_t*>(y_scale), ldy_scale * 4);
  return check_launch("upsample2x_fp8");
}

extern "C" int i2pc_cls_pos(const float* cls, const float* pos0, int batch, int tokens, int dim, float* x, void* stream) {
  clear_error();
  I2PC_REQUIRE(cls && pos0 && x && batch > 0 && tokens > 0 && dim > 0, "cls_pos: bad args");
  hipLaunchKernelGGL(k_cls_pos, dim3((batch * dim + 255) / 256), dim3(256), 0, as_stream(stream), cls, pos0, batch, tokens, dim, x);
  return check_launch("cls_pos");
}

extern "C" int i2pc_f32_to_bf16(const float* x, int64_t n, void* y, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && y && n > 0 && n % 4 == 0, "f32_to_bf16: n must be a positive multiple of 4");
  hipLaunchKernelGGL(k_f32_to_bf16, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(x), n / 4, static_cast<uint2*>(y));
  return check_launch("f32_to_bf16");
}

extern "C" int i2pc_head_out(const void* x, int64_t pixels, int c, const float* w, float bias, float* depth, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && w && depth && pixels > 0 && c > 0 && c <= 64 && c % 8 == 0, "head_out: bad args");
  hipLaunchKernelGGL(k_head_out, dim3(grid_for(pixels)), dim3(256), 0, as_stream(stream),
                     static_cast<const bf16_t*>(x), pixels, c, w, bias, depth);
  return check_launch("head_out");
}

// BiT-ResNet stem of DPT-Hybrid (transformers modeling_bit.py, called from
// modeling_dpt.py:89-182) on gfx950, NHWC bf16.  The convolutions themselves run on the
// MFMA GEMM engine (weight standardisation is folded into the weights at load); this file
// holds the memory-bound glue around them:
//   k_stem_im2col : 7x7 stride-2 "SAME" stem conv input (BitEmbeddings.convolution,
//                   modeling_bit.py:234-241, DynamicPad2d :148-196) as bf16 GEMM rows
//                   [pixel][(ky, kx, c) padded to a multiple of 64]
//   k_gn_partial / k_gn_finalize : GroupNorm statistics (nn.functional.group_norm,
//                   modeling_bit.py:142-146): per-tile fp32 sums, fp64 combine -> (mean, rstd)
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
// I: flat index type, uint32_t when the index space stays below 2^31 (32-bit divisions)
template <typename I>
__global__ __launch_bounds__(256) void k_stem_im2col(const float* __restrict__ x, int B, int H, int W, int OH, int OW,
                                                     int pt, int pl, int ks, int kp, bf16_t* __restrict__ out) {
  const int KK = ks * ks * 3;
  const I total = (I)B * (I)OH * (I)OW * (I)(kp / 8);
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const I m = i / (I)(kp / 8);
    const int k0 = (int)(i - m * (I)(kp / 8)) * 8;
    const int b = (int)(m / ((I)OH * (I)OW));
    const int rem = (int)(m - (I)b * (I)OH * (I)OW);
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
      w[e / 2] = pk2bf(v[0], v[1]);
    }
    *reinterpret_cast<uint4*>(out + (int64_t)m * kp + k0) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// GroupNorm statistics in two launches, no atomics:
//  k_gn_partial: one workgroup = one image x PIX pixels; thread t owns 8 consecutive channels
//    of pixel lane t / (C / 8) and accumulates their sums / sums of squares over the tile in
//    registers (fp32) SHIFTED by each channel's value at the tile's first pixel (so a mean far
//    above the spread -- BiT activations after a residual -- does not cancel E[x^2] - mean^2
//    away); the pixel lanes reduce through LDS and the workgroup writes one (mean, M2) pair per
//    group to part[b][tile][g] (channels combined by Chan's formula).
//  k_gn_finalize: one wave per (image, group) merges the tile pairs in fp64 (Chan's parallel
//    formula) and writes (mean, rstd) as float: stats[b][g] (biased variance, as
//    nn.functional.group_norm).
// pixels per workgroup: a function of the image size only (~32 tiles per image, 32..512 pixels), so an
// image's statistics -- partial sums over its tiles -- are the same bits whatever batch it is in
// (r06: the r05 rule sized tiles by batch * hw, so DPT-Hybrid's depth of one image moved by 3-4 %
// between a batch of 64 and a batch of 3 once the fp8 roundings amplified the different partial sums;
// the rule below is r05's at batch 64, so the C5 step is unchanged)
static int gn_pix(int /*batch*/, int hw) {
  const int64_t want = ((int64_t)hw + 31) / 32;
  return (int)std::max<int64_t>(32, std::min<int64_t>(512, (want + 31) / 32 * 32));
}

__global__ __launch_bounds__(256) void k_gn_partial(const bf16_t* __restrict__ x, int HW, int C, int G, int tiles,
                                                    int PIX, float* __restrict__ part) {
  __shared__ float red[2][2048];
  const int chunks = C / 8;
  const int per_it = 256 / chunks;                 // pixel lanes (C <= 2048)
  const int b = blockIdx.x / tiles;
  const int tile = blockIdx.x - b * tiles;
  const int p0 = tile * PIX;
  const int cc = threadIdx.x % chunks;
  const int pl = threadIdx.x / chunks;
  float s[8] = {}, q[8] = {}, k8[8];
  {
    // the shift: channel value at the tile's first pixel (the same for every pixel lane)
    uint4 u0 = *reinterpret_cast<const uint4*>(x + ((int64_t)b * HW + p0) * C + cc * 8);
    const uint32_t w0[4] = {u0.x, u0.y, u0.z, u0.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) { k8[2 * e] = __uint_as_float(w0[e] << 16); k8[2 * e + 1] = __uint_as_float(w0[e] & 0xffff0000u); }
  }
  const int p1 = min(p0 + PIX, HW);
  if (pl < per_it) {
    const bf16_t* xb = x + (int64_t)b * HW * C + cc * 8;
    constexpr int U = 8;                           // 8 independent 16-B loads in flight
    for (int pb = p0 + pl; pb < p1; pb += U * per_it) {
      uint4 u[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int p = pb + k * per_it;
        u[k] = *reinterpret_cast<const uint4*>(xb + (int64_t)min(p, p1 - 1) * C);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (pb + k * per_it >= p1) continue;      // (past the tile: loaded clamped, not counted)
        const uint32_t w[4] = {u[k].x, u[k].y, u[k].z, u[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = __uint_as_float(w[e] << 16) - k8[2 * e], c = __uint_as_float(w[e] & 0xffff0000u) - k8[2 * e + 1];
          s[2 * e] += a; q[2 * e] = fmaf(a, a, q[2 * e]);
          s[2 * e + 1] += c; q[2 * e + 1] = fmaf(c, c, q[2 * e + 1]);
        }
      }
    }
  }
  // per channel: sum over the pixel lanes through the lane-major LDS image [per_it][C]
  // (per_it * C <= 2048 because per_it = 256 / (C / 8))
  if (pl < per_it) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[0][pl * C + cc * 8 + e] = s[e];
      red[1][pl * C + cc * 8 + e] = q[e];
    }
  }
  __syncthreads();
  // per channel: mean and M2 over the tile's pixels from the shifted sums
  const float nt = (float)(p1 - p0);
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f, d = 0.f;
    for (int l = 0; l < per_it; ++l) { a += red[0][l * C + c]; d += red[1][l * C + c]; }
    const bf16_t kc = x[((int64_t)b * HW + p0) * C + c];
    const float m = a / nt;
    red[0][c] = __uint_as_float((uint32_t)kc << 16) + m;   // (only this thread reads column c, and row 0 is its own slot)
    red[1][c] = fmaxf(d - a * m, 0.f);
  }
  __syncthreads();
  const int cg = C / G;
  for (int g = threadIdx.x; g < G; g += 256) {
    float mg = 0.f;
    for (int k = 0; k < cg; ++k) mg += red[0][g * cg + k];
    mg /= (float)cg;
    float m2 = 0.f;
    for (int k = 0; k < cg; ++k) {
      const float dm = red[0][g * cg + k] - mg;
      m2 += red[1][g * cg + k] + nt * dm * dm;
    }
    part[(((int64_t)b * tiles + tile) * G + g) * 2] = mg;
    part[(((int64_t)b * tiles + tile) * G + g) * 2 + 1] = m2;
  }
}

// one wave per (image, group): the lanes add the tile partials in fp64 (lane t takes tiles
// t, t + 64, ...), then a butterfly over the wave.  (A thread per (image, group) walking the
// tiles serially was latency-bound: 8.8 us per call, 52 calls per DPT-Hybrid step.)
__global__ __launch_bounds__(256) void k_gn_finalize(const float* __restrict__ part, int B, int G, int tiles,
                                                     int HW, int PIX, int cg, float eps, float* __restrict__ stats) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= B * G) return;
  const int b = i / G, g = i - (i / G) * G;
  // Chan: (n, mean, M2) of two parts -> the union's
  double n = 0.0, mean = 0.0, m2 = 0.0;
  auto merge = [&](double nb, double mb, double m2b) {
    if (nb == 0.0) return;
    const double nn = n + nb, dlt = mb - mean;
    mean += dlt * (nb / nn);
    m2 += m2b + dlt * dlt * (n * nb / nn);
    n = nn;
  };
  for (int t = lane; t < tiles; t += 64) {
    const float2 pr = *reinterpret_cast<const float2*>(part + (((int64_t)b * tiles + t) * G + g) * 2);
    merge((double)(min(PIX, HW - t * PIX) * cg), pr.x, pr.y);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    merge(__shfl_xor(n, o), __shfl_xor(mean, o), __shfl_xor(m2, o));
  if (lane == 0) {
    const double var = fmax(m2 / n, 0.0);
    stats[2 * i] = (float)mean;
    stats[2 * i + 1] = 1.0f / sqrtf((float)var + eps);
  }
}

struct GnOperand {
  const bf16_t* x;
  const float* stats;       // [B][G] (mean, rstd) (null: x is used raw)
  const float* gamma;
  const float* beta;
};

// per-channel affine of one operand for image b: v * sc + sh (identity when raw)
__device__ __forceinline__ void gn_coeffs(const GnOperand& o, int b, int c0, int C, int G, float sc[8], float sh[8]) {
  if (!o.stats) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = 1.f; sh[e] = 0.f; }
    return;
  }
  const int cg = C / G;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    const float2 st = *reinterpret_cast<const float2*>(o.stats + ((int64_t)b * G + c / cg) * 2);
    sc[e] = st.y * o.gamma[c];
    sh[e] = o.beta[c] - st.x * sc[e];
  }
}

__device__ __forceinline__ void unpack8(const uint4& u, float v[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(w[e] << 16);
    v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}

// One workgroup = one image x PIX pixels; thread = (channel chunk, pixel lane) as in
// k_gn_partial, so every thread derives its 8 channels' scale / shift once.
// (x - mean) * rstd * gamma + beta is evaluated as x * (rstd * gamma) + (beta - mean * rstd * gamma).
__global__ __launch_bounds__(256) void k_gn_apply(GnOperand a, GnOperand r, int has_r, int HW, int C, int G, int tiles,
                                                  int PIX, int relu, bf16_t* __restrict__ y) {
  const int chunks = C / 8;
  const int per_it = 256 / chunks;
  const int b = blockIdx.x / tiles;
  const int p0 = (blockIdx.x - b * tiles) * PIX;
  const int cc = threadIdx.x % chunks;
  const int pl = threadIdx.x / chunks;
  if (pl >= per_it) return;
  const int c0 = cc * 8;
  float as[8], ah[8], rs[8], rh[8];
  gn_coeffs(a, b, c0, C, G, as, ah);
  if (has_r) gn_coeffs(r, b, c0, C, G, rs, rh);
  const int64_t base = (int64_t)b * HW * C + c0;
  const int p1 = min(p0 + PIX, HW);
  constexpr int U = 4;
  for (int pb = p0 + pl; pb < p1; pb += U * per_it) {
    uint4 ux[U], ur[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int p = pb + k * per_it;
      const int64_t off = base + (int64_t)min(p, p1 - 1) * C;
      ux[k] = *reinterpret_cast<const uint4*>(a.x + off);
      if (has_r) ur[k] = *reinterpret_cast<const uint4*>(r.x + off);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int p = pb + k * per_it;
      if (p >= p1) break;
      float v[8], w[8];
      unpack8(ux[k], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(v[e], as[e], ah[e]);
      if (has_r) {
        unpack8(ur[k], w);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += fmaf(w[e], rs[e], rh[e]);
      }
      if (relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      uint4 o;
      o.x = pk2bf(v[0], v[1]);
      o.y = pk2bf(v[2], v[3]);
      o.z = pk2bf(v[4], v[5]);
      o.w = pk2bf(v[6], v[7]);
      *reinterpret_cast<uint4*>(y + base + (int64_t)p * C) = o;
    }
  }
}

// The same im2col with the input window staged in LDS: a workgroup owns 64 consecutive output
// pixels of one output row; it loads the ks input rows x (2 * 63 + ks) columns x 3 channels they
// read (coalesced along x, zero outside the image) once, then writes the 64 x kp output chunks
// (16 B per thread, consecutive threads consecutive chunks).  The per-lane gathers of
// k_stem_im2col read 8 scattered floats per 16-B output.  Same values (bit-identical).
constexpr int kStemOX = 64, kStemMaxK = 7;
constexpr int kStemCols = 2 * (kStemOX - 1) + kStemMaxK;
__global__ __launch_bounds__(256) void k_stem_im2col_lds(const float* __restrict__ x, int B, int H, int W, int OH, int OW,
                                                         int pt, int pl, int ks, int kp, bf16_t* __restrict__ out) {
  __shared__ float win[3 * kStemMaxK * kStemCols];   // [c][row][col]
  __shared__ int koff[256];                           // window offset of k, -1 beyond ks*ks*3
  const int segs = (OW + kStemOX - 1) / kStemOX;
  const int seg = blockIdx.x % segs;
  const int oy = (blockIdx.x / segs) % OH;
  const int b = blockIdx.x / (segs * OH);
  const int ox0 = seg * kStemOX;
  const int nox = min(kStemOX, OW - ox0);
  const int iy0 = oy * 2 - pt, ix0 = ox0 * 2 - pl;
  const int ncols = 2 * (nox - 1) + ks;
  const int KK = ks * ks * 3;
  if ((int)threadIdx.x < kp) {
    const int k = threadIdx.x;
    const int tap = k / 3, c = k - tap * 3;
    const int ky = tap / ks, kx = tap - ky * ks;
    koff[k] = k < KK ? (c * ks + ky) * kStemCols + kx : -1;
  }
  // every (c, row) of the window by the first kStemCols threads, all loads in flight before the
  // first LDS write (a per-row load -> store loop serialised 21 memory latencies per workgroup)
  if ((int)threadIdx.x < kStemCols) {
    const int col = threadIdx.x;
    const int ix = ix0 + col;
    const bool cin = col < ncols && (unsigned)ix < (unsigned)W;
    float v[3 * kStemMaxK];
#pragma unroll
    for (int rowi = 0; rowi < 3 * kStemMaxK; ++rowi) {
      v[rowi] = 0.f;
      if (rowi < 3 * ks) {
        const int c = rowi / ks, r = rowi - c * ks;
        const int iy = iy0 + r;
        if (cin && (unsigned)iy < (unsigned)H) v[rowi] = x[(((int64_t)b * 3 + c) * H + iy) * W + ix];
      }
    }
#pragma unroll
    for (int rowi = 0; rowi < 3 * kStemMaxK; ++rowi)
      if (rowi < 3 * ks) win[rowi * kStemCols + col] = v[rowi];
  }
  __syncthreads();
  // thread t: chunk kc = t % cpm of output pixels ml = t / cpm + j * (256 / cpm) (consecutive
  // threads write consecutive 16-B chunks)
  const int cpm = kp / 8;
  const int per = 256 / cpm;
  const int ml0 = threadIdx.x / cpm, kc = threadIdx.x - ml0 * cpm;
  if (ml0 >= per) return;
  int off[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) off[e] = koff[kc * 8 + e];
  bf16_t* ob = out + (((int64_t)b * OH + oy) * OW + ox0) * kp + kc * 8;
  for (int ml = ml0; ml < nox; ml += per) {
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const float v0 = off[e] >= 0 ? win[off[e] + 2 * ml] : 0.f;
      const float v1 = off[e + 1] >= 0 ? win[off[e + 1] + 2 * ml] : 0.f;
      w[e / 2] = pk2bf(v0, v1);
    }
    *reinterpret_cast<uint4*>(ob + (int64_t)ml * kp) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// 3x3 stride-2 max over the zero-padded map (pad pt top / pl left, zero beyond the
// bottom/right edge as DynamicPad2d pads there), 8 channels per thread
template <typename I>
__global__ __launch_bounds__(256) void k_maxpool(const bf16_t* __restrict__ x, int B, int H, int W, int C, int OH, int OW,
                                                 int pt, int pl, bf16_t* __restrict__ y) {
  const I cv = (I)(C / 8);
  const I total = (I)B * (I)OH * (I)OW * cv;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cv) * 8;
    const I pix = i / cv;
    const int b = (int)(pix / ((I)OH * (I)OW));
    const int rem = (int)(pix - (I)b * (I)OH * (I)OW);
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
    o.x = pk2bf(m[0], m[1]);
    o.y = pk2bf(m[2], m[3]);
    o.z = pk2bf(m[4], m[5]);
    o.w = pk2bf(m[6], m[7]);
    *reinterpret_cast<uint4*>(y + (int64_t)pix * C + c0) = o;
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
  if (ksize <= kStemMaxK && k_pitch <= 256)
    hipLaunchKernelGGL(k_stem_im2col_lds, dim3(batch * out_h * ((out_w + kStemOX - 1) / kStemOX)), dim3(256), 0,
                       as_stream(stream), pixels, batch, h, w, out_h, out_w, pad_top, pad_left, ksize, k_pitch,
                       static_cast<bf16_t*>(out));
  else if (work + (int64_t)grid_for(work) * 256 < ((int64_t)1 << 31))
    hipLaunchKernelGGL(k_stem_im2col<uint32_t>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), pixels, batch, h,
                       w, out_h, out_w, pad_top, pad_left, ksize, k_pitch, static_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL(k_stem_im2col<int64_t>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), pixels, batch, h,
                       w, out_h, out_w, pad_top, pad_left, ksize, k_pitch, static_cast<bf16_t*>(out));
  return check_launch("bit_stem_im2col");
}

extern "C" size_t i2pc_groupnorm_workspace_bytes(int batch, int hw, int groups) {
  const int pix = gn_pix(batch, hw);
  return sizeof(float) * 2 * (size_t)batch * ((hw + pix - 1) / pix) * groups;
}

extern "C" int i2pc_groupnorm_stats(const void* x, int batch, int hw, int c, int groups, float eps, float* stats,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && stats && workspace && batch > 0 && hw > 0, "bad arguments");
  I2PC_REQUIRE(c % 8 == 0 && c <= 2048 && groups > 0 && c % groups == 0, "groupnorm: C=%d (%% 8, <= 2048) / groups %d", c, groups);
  const int pix = gn_pix(batch, hw);
  const int tiles = (hw + pix - 1) / pix;
  I2PC_REQUIRE(workspace_bytes >= i2pc_groupnorm_workspace_bytes(batch, hw, groups), "groupnorm: workspace too small");
  hipStream_t s = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(k_gn_partial, dim3(batch * tiles), dim3(256), 0, s, static_cast<const bf16_t*>(x), hw, c, groups,
                     tiles, pix, part);
  const int n = batch * groups;
  hipLaunchKernelGGL(k_gn_finalize, dim3((n + 3) / 4), dim3(256), 0, s, part, batch, groups, tiles, hw, pix,
                     c / groups, eps, stats);
  return check_launch("groupnorm_stats");
}

extern "C" int i2pc_groupnorm_apply(const void* x, const float* stats, const float* gamma, const float* beta,
                                    const void* r, const float* r_stats, const float* r_gamma, const float* r_beta,
                                    int batch, int hw, int c, int groups, int relu, void* y, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && y && batch > 0 && hw > 0 && c % 8 == 0 && groups > 0 && c % groups == 0, "bad arguments");
  I2PC_REQUIRE(!stats || (gamma && beta), "groupnorm: gamma/beta required with statistics");
  I2PC_REQUIRE(!r_stats || (r && r_gamma && r_beta), "groupnorm: shortcut gamma/beta required with its statistics");
  I2PC_REQUIRE(c <= 2048, "groupnorm: C=%d > 2048", c);
  GnOperand a{static_cast<const bf16_t*>(x), stats, gamma, beta};
  GnOperand rr{static_cast<const bf16_t*>(r), r_stats, r_gamma, r_beta};
  const int pix = gn_pix(batch, hw);
  const int tiles = (hw + pix - 1) / pix;
  hipLaunchKernelGGL(k_gn_apply, dim3(batch * tiles), dim3(256), 0, as_stream(stream), a, rr, r ? 1 : 0, hw, c, groups,
                     tiles, pix, relu, static_cast<bf16_t*>(y));
  return check_launch("groupnorm_apply");
}

extern "C" int i2pc_maxpool3s2(const void* x, int batch, int h, int w, int c, int out_h, int out_w, int pad_top,
                               int pad_left, void* y, void* stream) {
  clear_error();
  I2PC_REQUIRE(x && y && batch > 0 && h > 0 && w > 0 && c % 8 == 0 && out_h > 0 && out_w > 0, "bad arguments");
  const int64_t work = (int64_t)batch * out_h * out_w * (c / 8);
  if (work + (int64_t)grid_for(work) * 256 < ((int64_t)1 << 31))
    hipLaunchKernelGGL(k_maxpool<uint32_t>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream),
                       static_cast<const bf16_t*>(x), batch, h, w, c, out_h, out_w, pad_top, pad_left,
                       static_cast<bf16_t*>(y));
  else
    hipLaunchKernelGGL(k_maxpool<int64_t>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream),
                       static_cast<const bf16_t*>(x), batch, h, w, c, out_h, out_w, pad_top, pad_left,
                       static_cast<bf16_t*>(y));
  return check_launch("maxpool3s2");
}

// Fused DPT depth head tail on MI355X:
//   bilinear resize (align_corners=True) of the head's first conv output to (H, W)
//   -> 3x3 conv C -> 32 + bias + ReLU -> 1x1 conv 32 -> 1 + bias + ReLU -> depth fp32.
// (transformers DPTDepthEstimationHead / DepthAnythingDepthEstimationHead: head[1..5],
//  modeling_dpt.py:679-716.)  Unfused, the resize writes a C-channel map at (H, W) in bf16
// (1.2 GB for DPT-Large at B=32) that the im2col conv then reads nine times.
//
// Workgroup = an 8 x 64 output tile, four waves (wave w: the 8 x 16 strip at columns 16w..16w+15),
// two workgroups per CU.  Per pass of 32 input channels:
//  1. the tile's low-resolution source window (at most 7 x 35 pixels for DPT's 2x resize) and the
//     pass's conv weights (9 taps x 32 output x 32 input channels, 18 KB) land in LDS by LDS-DMA
//     (buffer_load ... lds), issued one pass ahead so they travel behind the previous pass's MFMAs;
//  2. each wave reads its B fragments (weights) from LDS into registers, then the resized 10 x 66
//     halo is built from LDS separably: a thread owns (halo column, 8 channels) and walks the ten
//     halo rows; halo row 0 interpolates its two source rows horizontally, every later row
//     interpolates its lower source row and keeps it only if the resize moved down a source row
//     (branch-free, so the compiler issues the LDS reads ahead) -- k_resize's fp32 operations in
//     k_resize's order (t = fma(wx1, p[x1], wx0 * p[x0]) per source row, r = fma(wy1, t1, wy0 * t0)),
//     rounded to bf16 like the unfused map; the two halo columns past the 256 walkers are
//     interpolated directly with the same operations;
//  3. the 3x3 conv on the MFMA cores (v_mfma_f32_16x16x32_bf16, A = 16 halo pixels x 32
//     channels, B = 32 channels x 16 output channels): a halo row's three column-shifted A
//     fragments are read once and feed every output row that uses them (dy = 0..2), 30 LDS reads
//     for a wave's 144 MFMAs.
// Halo layout: rows of 66 pixels, 64 B per pixel, 16-B group q of column c stored at
// q ^ ((c >> 1) & 3): the A reads (16 consecutive pixels x 4 groups) are conflict-free at any column
// offset; the weights use the same swizzle over output channels.
// The epilogue rounds relu(acc + b2) to bf16 (the unfused conv stores bf16), multiplies by the
// 1x1 weights, reduces the 32 channels across lanes (DPP), adds b4 and applies ReLU.
#include "common.h"

#include <algorithm>

namespace i2pc {
namespace head {

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int kTH = 8, kTW = 64;                  // output pixels per workgroup
constexpr int kHH = kTH + 2, kHW = kTW + 2;       // resized halo
constexpr int kKC = 32;                           // input channels per pass
constexpr int kRowBytes = kHW * kKC * 2;          // 4,224
constexpr int kHaloBytes = kHH * kRowBytes;       // 42,240
constexpr int kWBytes = 9 * 32 * kKC * 2;         // 18,432: a pass's weights
constexpr int kSrcMax = 52 * 1024;                // LDS for a pass's source window (any enlarging resize)
constexpr int kBlock = 256;
constexpr int kEdge = kHH * 2 * 4;                // direct items of the last two halo columns

// one v_cvt_pk_bf16_f32 per pair (RNE, as the scalar conversions)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
// halo row i, column col, 16-B channel group q
__device__ __forceinline__ int halo_off(int i, int col, int q) { return i * kRowBytes + col * 64 + ((q ^ ((col >> 1) & 3)) << 4); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// source pixels p0 (x0) and p1 (x1) of one LDS row, channel group g -> 8 horizontally interpolated values
__device__ __forceinline__ void hlerp(const uint8_t* s_row, int p0, int p1, int g, float lx0, float lx1, float* t) {
  const uint4 a = *reinterpret_cast<const uint4*>(s_row + (p0 * 4 + g) * 16);
  const uint4 b = *reinterpret_cast<const uint4*>(s_row + (p1 * 4 + g) * 16);
  const uint32_t pa[4] = {a.x, a.y, a.z, a.w}, pb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    t[2 * k] = __builtin_fmaf(lx1, lo_f(pb[k]), lx0 * lo_f(pa[k]));
    t[2 * k + 1] = __builtin_fmaf(lx1, hi_f(pb[k]), lx0 * hi_f(pa[k]));
  }
}

// 16 B global -> LDS at lds_base + 16 * lane (buffer_load ... lds).  Inline asm: the compiler does
// not see these writes, so it inserts no waits for them (it would put a vmcnt(0) -- which also
// drains the weight loads meant to stay in flight -- in front of every LDS access it cannot prove
// disjoint); the kernel orders them itself with a counted vmcnt and a barrier.  M0 carries the LDS
// base and is declared clobbered (the compiler keeps any M0 value of its own around it).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t lds_base, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs), "s"(soff)
               : "memory", "m0");
}

// keep = all ones inside the image, 0 on the conv's zero padding
__device__ __forceinline__ uint4 vlerp(const float* t0, const float* t1, float ly0, float ly1, uint32_t keep) {
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    o[k] = pack2(__builtin_fmaf(ly1, t1[2 * k], ly0 * t0[2 * k]), __builtin_fmaf(ly1, t1[2 * k + 1], ly0 * t0[2 * k + 1])) &
           keep;
  return uint4{o[0], o[1], o[2], o[3]};
}

// k_resize's index rules (align_corners=True) for output coordinate v of n_out from n_in
struct Tap1 {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ Tap1 tap(float s, int v, int n_out, int n_in) {
  const float f = s * (float)min(max(v, 0), n_out - 1);
  Tap1 t;
  t.i0 = (int)f;
  t.i1 = t.i0 + (t.i0 < n_in - 1 ? 1 : 0);
  t.l1 = f - (float)t.i0;
  t.l0 = 1.f - t.l1;
  return t;
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// sum over the 16 lanes of a row (quad swaps, half-row mirror, row mirror); every lane ends with it
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return v;
}

__global__ __launch_bounds__(kBlock, 2) void k_head_upconv(const bf16_t* __restrict__ x, int h, int w, int C, int cin,
                                                           int H, int W, int tiles_w, int tiles_h, int win_rows,
                                                           int win_cols, const bf16_t* __restrict__ w2,
                                                           const float* __restrict__ b2, const float* __restrict__ w4,
                                                           float b4, float* __restrict__ depth) {
  // separate LDS objects, so the compiler knows the halo stores and the window reads are disjoint
  // (and issues a row's window reads ahead of the previous row's halo store)
  __shared__ __attribute__((aligned(16))) uint8_t s_halo[kHaloBytes];
  __shared__ __attribute__((aligned(16))) uint8_t s_w[kWBytes];
  // halo row i's source rows (byte offsets in the window) and vertical weights, per tile
  __shared__ __attribute__((aligned(16))) u32x4 s_rows[kHH];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_src[];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, m = lane & 15;
  int bid = blockIdx.x;
  const int tx = bid % tiles_w;
  bid /= tiles_w;
  const int ty = bid % tiles_h;
  const int b = bid / tiles_h;
  const int oy0 = ty * kTH, ox0 = tx * kTW;
  const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  // the tile's source window: the taps of its first and last (clamped) halo rows / columns
  const int sy0 = tap(sh, oy0 - 1, H, h).i0, sy1 = tap(sh, oy0 + kTH, H, h).i1;
  const int sx0 = tap(sw, ox0 - 1, W, w).i0, sx1 = tap(sw, ox0 + kTW, W, w).i1;
  const int sc = sx1 - sx0 + 1, sr = sy1 - sy0 + 1;
  if (sr > win_rows || sc > win_cols) {
    // (cannot happen: the host sized the window with this arithmetic) -- NaN, not a fault
    for (int p = threadIdx.x; p < kTH * kTW; p += kBlock) {
      const int oy = oy0 + p / kTW, ox = ox0 + p % kTW;
      if (oy < H && ox < W) depth[((int64_t)b * H + oy) * W + ox] = __builtin_nanf("");
    }
    return;
  }
  const int rp = sc * 4;                      // 16-B pieces per window row
  if (threadIdx.x < kHH) {
    const Tap1 t = tap(sh, oy0 - 1 + (int)threadIdx.x, H, h);
    s_rows[threadIdx.x] = u32x4{(uint32_t)((t.i0 - sy0) * rp * 16), (uint32_t)((t.i1 - sy0) * rp * 16),
                                __float_as_uint(t.l0), __float_as_uint(t.l1)};
  }

  // a pass's source window -> LDS: window row r by wave r % 4, 64 pieces per DMA (lane-linear:
  // piece = (column, 16-B group)), the lanes past a row's end masked off
  const __amdgpu_buffer_rsrc_t x_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(x + (((int64_t)b * h + sy0) * w + sx0) * C), 0, ((sr - 1) * w + sc) * C * 2, 0x00020000);
  // a pass's weights -> LDS: slot s = (tap, output channel, swizzled group), 18 DMAs over the waves
  const __amdgpu_buffer_rsrc_t w_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(w2), 0, 32 * 9 * C * 2, 0x00020000);
  auto load_pass = [&](int c0) {
    for (int r = wid; r < sr; r += 4)
      for (int j = 0; j * 64 < rp; ++j) {
        const int pp = j * 64 + lane;
        if (pp < rp)
          dma16(x_rs, __builtin_amdgcn_readfirstlane(lds_addr(s_src + (r * rp + j * 64) * 16)),
                ((pp >> 2) * C + (pp & 3) * 8) * 2, (r * w * C + c0) * 2);
      }
    for (int j = wid; j < kWBytes / 1024; j += 4) {
      const int sl = j * 64 + lane, t = sl >> 7, co = (sl >> 2) & 31, gq = (sl & 3) ^ ((co >> 1) & 3);
      dma16(w_rs, __builtin_amdgcn_readfirstlane(lds_addr(s_w + j * 1024)), ((co * 9 + t) * C + gq * 8) * 2, c0 * 2);
    }
  };

  // walker: halo column hc, channel group g
  const int hc = threadIdx.x >> 2, g = threadIdx.x & 3;
  const Tap1 tcol = tap(sw, ox0 - 1 + hc, W, w);
  const bool in_x = ox0 - 1 + hc >= 0 && ox0 - 1 + hc < W;
  const int cx0 = tcol.i0 - sx0, cx1 = tcol.i1 - sx0;

  f32x4 acc[kTH][2];
#pragma unroll
  for (int r = 0; r < kTH; ++r)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_pass(0);
  for (int c0 = 0; c0 < cin; c0 += kKC) {
    // this wave's DMAs landed, then every wave's; every wave is done with the previous pass's halo
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // the pass's B fragments (in flight behind the walk)
    bf16x8 bw[9][2];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int co = 16 * n + m;
        bw[t][n] = *reinterpret_cast<const bf16x8*>(s_w + ((t * 32 + co) * 4 + (q ^ ((co >> 1) & 3))) * 16);
      }

    // halo rows 0..9, walked: row 0 interpolates both of its source rows; each later row either
    // shares row i-1's pair or moves one source row down (the host checks that a resize step never
    // skips a source row), so it always interpolates its lower source row -- unconditionally, for
    // straight-line code whose LDS reads the compiler can issue ahead -- and keeps it if it moved
    {
      float ta[8], tb[8];
      const u32x4 r0 = s_rows[0];
      hlerp(s_src + r0.x, cx0, cx1, g, tcol.l0, tcol.l1, ta);
      hlerp(s_src + r0.y, cx0, cx1, g, tcol.l0, tcol.l1, tb);
      const uint32_t keep0 = in_x && oy0 - 1 >= 0 ? ~0u : 0u;
      *reinterpret_cast<uint4*>(s_halo + halo_off(0, hc, g)) = vlerp(ta, tb, __uint_as_float(r0.z), __uint_as_float(r0.w), keep0);
      uint32_t prev = __builtin_amdgcn_readfirstlane(r0.x);
#pragma unroll
      for (int i = 1; i < kHH; ++i) {
        const u32x4 rt = s_rows[i];
        float nt[8];
        hlerp(s_src + rt.y, cx0, cx1, g, tcol.l0, tcol.l1, nt);
        const uint32_t o0 = __builtin_amdgcn_readfirstlane(rt.x);
        const bool adv = o0 != prev;
        prev = o0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          ta[k] = adv ? tb[k] : ta[k];
          tb[k] = adv ? nt[k] : tb[k];
        }
        const uint32_t keep = in_x && oy0 - 1 + i < H ? ~0u : 0u;
        *reinterpret_cast<uint4*>(s_halo + halo_off(i, hc, g)) = vlerp(ta, tb, __uint_as_float(rt.z), __uint_as_float(rt.w), keep);
      }
    }
    if (threadIdx.x < kEdge) {
      // direct item: halo row ei, column kTW + 0 / 1, group eg
      const int ei = threadIdx.x >> 3, eh = kTW + ((threadIdx.x >> 2) & 1), eg = threadIdx.x & 3;
      const Tap1 ecol = tap(sw, ox0 - 1 + eh, W, w);
      const u32x4 rt = s_rows[ei];
      const uint32_t e_keep = ox0 - 1 + eh >= 0 && ox0 - 1 + eh < W && oy0 - 1 + ei >= 0 && oy0 - 1 + ei < H ? ~0u : 0u;
      float t0[8], t1[8];
      hlerp(s_src + rt.x, ecol.i0 - sx0, ecol.i1 - sx0, eg, ecol.l0, ecol.l1, t0);
      hlerp(s_src + rt.y, ecol.i0 - sx0, ecol.i1 - sx0, eg, ecol.l0, ecol.l1, t1);
      *reinterpret_cast<uint4*>(s_halo + halo_off(ei, eh, eg)) = vlerp(t0, t1, __uint_as_float(rt.z), __uint_as_float(rt.w), e_keep);
    }
    // halo built, B fragments in registers: the window and weight slots are free for the next pass
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c0 + kKC < cin) load_pass(c0 + kKC);

    // a halo row's three A fragments, the next row's in flight behind this row's MFMAs
    bf16x8 a[2][3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) a[0][dx] = *reinterpret_cast<const bf16x8*>(s_halo + halo_off(0, 16 * wid + dx + m, q));
#pragma unroll
    for (int i = 0; i < kHH; ++i) {
      if (i + 1 < kHH)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
          a[(i + 1) & 1][dx] = *reinterpret_cast<const bf16x8*>(s_halo + halo_off(i + 1, 16 * wid + dx + m, q));
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const int r = i - dy;
          if (r < 0 || r >= kTH) continue;
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 1][dx], bw[dy * 3 + dx][n], acc[r][n], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // epilogue: lane holds output channel co = 16 n + m of pixels 16 wid + 4 q + e
  float bias[2], wv[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    bias[n] = b2[16 * n + m];
    wv[n] = w4[16 * n + m];
  }
  const int ox = ox0 + 16 * wid + 4 * q;
#pragma unroll
  for (int r = 0; r < kTH; ++r) {
    float s[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = 0.f;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float v = fmaxf(acc[r][n][e] + bias[n], 0.f);
        const __bf16 vb = (__bf16)v;
        t += __uint_as_float((uint32_t)__builtin_bit_cast(uint16_t, vb) << 16) * wv[n];
      }
      s[e] = fmaxf(row16_sum(t) + b4, 0.f);
    }
    // lane m == r of each 16-lane group stores row r's four pixels
    const int oy = oy0 + r;
    if (m == r && oy < H) {
      float* d = depth + ((int64_t)b * H + oy) * W + ox;
      if (ox + 3 < W && (W & 3) == 0) {
        *reinterpret_cast<float4*>(d) = float4{s[0], s[1], s[2], s[3]};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (ox + e < W) d[e] = s[e];
      }
    }
  }
}

// Host mirror of the kernel's tap(): true when consecutive output rows never skip a source row
// (the walk's schedule; any enlarging resize)
static bool steps_by_one(int n_out, int n_in) {
  const float s = n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  int prev = 0;
  for (int v = 1; v < n_out; ++v) {
    const int i0 = (int)(s * (float)v);
    if (i0 - prev > 1) return false;
    prev = i0;
  }
  return true;
}

// Host mirror of the kernel's tap(): the largest source window of any tile (pixels per row / column)
static int window_extent(int n_out, int n_in, int tile) {
  const float s = n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  auto i0 = [&](int v) { return (int)(s * (float)std::min(std::max(v, 0), n_out - 1)); };
  int most = 1;
  for (int o = 0; o < n_out; o += tile) {
    const int lo = i0(o - 1), hi0 = i0(o + tile), hi = hi0 + (hi0 < n_in - 1 ? 1 : 0);
    most = std::max(most, hi - lo + 1);
  }
  return most;
}

}  // namespace head
}  // namespace i2pc

using namespace i2pc;

extern "C" int i2pc_head_upconv(const void* x, int batch, int h, int w, int c, int cin, int out_h, int out_w,
                                const void* w2, const float* b2, const float* w4, float b4, float* depth,
                                void* stream) {
  clear_error();
  I2PC_REQUIRE(x && w2 && b2 && w4 && depth, "head_upconv: NULL pointer");
  I2PC_REQUIRE(batch > 0 && h > 0 && w > 0 && out_h > 0 && out_w > 0, "head_upconv: empty shape");
  I2PC_REQUIRE(c > 0 && c % 8 == 0, "head_upconv: channel pitch %d must be a multiple of 8", c);
  I2PC_REQUIRE(cin > 0 && cin % head::kKC == 0 && cin <= c,
               "head_upconv: channels used %d must be a multiple of %d and at most the pitch %d", cin, head::kKC, c);
  I2PC_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(w2) % 16 == 0,
               "head_upconv: x and w2 must be 16-byte aligned");
  I2PC_REQUIRE((int64_t)batch * h * w * c < (1ll << 31) && (int64_t)batch * out_h * out_w < (1ll << 31),
               "head_upconv: tensor too large");
  I2PC_REQUIRE(out_h >= h && head::steps_by_one(out_h, h),
               "head_upconv: the resize must enlarge the rows (%d -> %d; the heads enlarge 2x or 1.75x)", h, out_h);
  // LDS for the source window: the largest over the tiles, by the kernel's own arithmetic (the
  // kernel checks its window against these and writes NaN rather than overrun)
  const int rows = head::window_extent(out_h, h, head::kTH), cols = head::window_extent(out_w, w, head::kTW);
  const size_t src_bytes = (size_t)rows * cols * 64;
  I2PC_REQUIRE(src_bytes <= (size_t)head::kSrcMax,
               "head_upconv: a tile's source window (%d x %d pixels) exceeds LDS: %dx%d -> %dx%d shrinks too much", rows,
               cols, h, w, out_h, out_w);
  const int tw = (out_w + head::kTW - 1) / head::kTW, th = (out_h + head::kTH - 1) / head::kTH;
  const int64_t blocks = (int64_t)batch * tw * th;
  I2PC_REQUIRE(blocks < (1ll << 31), "head_upconv: grid too large");
  const int lds = (int)src_bytes;   // (the halo, the weights and the row table are static LDS)
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(head::k_head_upconv),
                              hipFuncAttributeMaxDynamicSharedMemorySize, head::kSrcMax);
    attr = true;
  }
  hipLaunchKernelGGL(head::k_head_upconv, dim3((unsigned)blocks), dim3(head::kBlock), lds, as_stream(stream),
                     static_cast<const uint16_t*>(x), h, w, c, cin, out_h, out_w, tw, th, rows, cols,
                     static_cast<const uint16_t*>(w2), b2, w4, b4, depth);
  return check_launch("head_upconv");
}

// bf16 MFMA GEMM / implicit-GEMM convolution with fused epilogues (gfx950).
//
// out[m][n] = epilogue( sum_k A[m][k] * W[n][k] )
//   A : bf16, either a dense row-major matrix (optionally with a row remap, e.g.
//       "skip the CLS token") or the implicit im2col of an NHWC bf16 image
//       (3x3 / 1x1 convolutions, stride 1 or 2, zero padding) -- the conv/linear
//       blocks of the DPT network (transformers modeling_dpt.py:119-121,166,196,
//       212,320,373-382,434-451,490,645,697-701).
//   W : bf16 [n][k] (nn.Linear layout; conv weights pre-permuted to [co][ky][kx][ci]).
//   epilogue (fp32): + bias[n] + row_bias[m / g][n] + table[m % rows][n],
//       act (GELU-erf / ReLU), + residual (fp32 or bf16) + second residual (bf16),
//       store bf16 or fp32, row-major with a row remap or as a ConvTranspose
//       (kernel == stride) pixel shuffle into NHWC.
//
// Tiling: 256 threads (4 waves), BM x BN x 64 tile, LDS double buffer filled by
// global_load_lds_dwordx4 (16 B/lane, lane-linear LDS image with the XOR swizzle
// applied to the SOURCE address; fragments read back with ds_read_b128 through
// the same swizzle). MFMA v_mfma_f32_16x16x32_bf16 with the weight tile as the A
// operand, so each lane's four accumulators are four consecutive output columns
// (8-/16-byte epilogue stores). XCD-aware tile order: consecutive tiles (which
// share an activation panel) go to one XCD.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace i2pc {
namespace gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;

constexpr int BK = 64;

__device__ __attribute__((aligned(16))) uint8_t g_zero[512];   // conv zero padding source
#ifdef I2PC_STAMPS
// diagnostic build only: per-block s_memtime stamps (start, after prologue, after K loop, end)
__device__ unsigned long long g_stamps[65536 * 8];
#define STAMP(k)                                                                      \
  do {                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < 65536) {                                     \
      unsigned long long t;                                                           \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");      \
      g_stamps[blockIdx.x * 8 + (k)] = t;                                             \
    }                                                                                 \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

struct Args {
  const bf16_t* A; int64_t lda; int M, N, K;
  int a_g, a_gs, a_o;
  int cb, ch, cw, cc, coh, cow, ck, cs, cp;
  const bf16_t* W; int64_t ldw;
  const float* bias;
  const float* rbias; int rb_g;
  const float* tbl; int tbl_rows;
  int act;
  const void* res; int res_f32; int64_t ldr;
  const bf16_t* res2; int64_t ldr2;
  void* C; int c_f32; int64_t ldc;
  int o_g, o_gs, o_o;
  int ct_s, ct_h, ct_w, ct_c;
  int tiles_m, tiles_n;
  int group_m;
};

__device__ __forceinline__ int remap(int m, int g, int gs, int o) {
  return g > 0 ? (m / g) * gs + (m % g) + o : m + o;
}

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ bf16_t f2bf(float x) {
  __bf16 b = (__bf16)x;
  return *reinterpret_cast<bf16_t*>(&b);
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds_base), 16, 0, 0);
}

// ReLU on 8 packed bf16 (pre-activation residual units): clear negative lanes.
__device__ __forceinline__ bf16x8 relu8(bf16x8 v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 u = __builtin_bit_cast(u32x4, v);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t neg = (u[i] >> 15) & 0x00010001u;
    u[i] &= ~(neg * 0xFFFFu);
  }
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ void tile_coords(const Args& p, int bid, int& tm, int& tn) {
  // 1) XCD-aware: blocks b and b+8 share an XCD, so give each XCD a contiguous range of
  //    linear tiles (bijective for any count); 2) inside the range walk GROUP_M M-tiles per
  //    N column so an XCD's live A and W panels stay L2-resident.
  const int nwg = p.tiles_m * p.tiles_n;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7, idx = bid >> 3;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  const int gsz = p.group_m * p.tiles_n;
  const int g = tile / gsz;
  const int first = g * p.group_m;
  const int gm = min(p.tiles_m - first, p.group_m);
  const int in = tile - g * gsz;
  tm = first + in % gm;
  tn = in / gm;
}

// ---------------------------------------------------------------------------
// Tile epilogue through LDS (the MFMA layout gives each lane 4 columns of one row,
// i.e. 8-byte stores scattered over 16 rows -- issue-bound, ~10k cycles per 128^2
// tile).  Phase 1 (MFMA layout): v = act(acc + bias + row_bias + table) -> fp32 in
// the wave's LDS region (16-B units XOR-swizzled by row).  Phase 2 (row layout):
// each lane owns 8 consecutive columns of one row: + res + res2 with 16/32-B loads,
// then one 16-B (bf16) or 2 x 16-B (fp32) store; a wave writes whole 128-B lines.
template <int RM, int RN>
__device__ __forceinline__ void tile_epilogue(const Args& p, f32x4 (&acc)[RM][RN], int i0, int ni, int mrow0,
                                              int ncol0, float* lds) {
  constexpr int TN = RN * 16;
  constexpr int U = TN / 4;                 // 16-B units per LDS row
  constexpr int SW = U >= 8 ? 7 : U - 1;    // swizzle mask
  const int lane = threadIdx.x & 63;
  const int frow = lane & 15;
  const int fq = lane >> 4;
  // bias depends on the column only: load it once, all loads in flight together
  float4 bias4[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j)
    bias4[j] = p.bias ? *reinterpret_cast<const float4*>(p.bias + ncol0 + j * 16 + fq * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  // phase 1
#pragma unroll
  for (int ii = 0; ii < ni; ++ii) {
    const int i = i0 + ii;
    const int r = ii * 16 + frow;
    const int m = mrow0 + i * 16 + frow;
    const int mc = m < p.M ? m : p.M - 1;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = ncol0 + j * 16 + fq * 4;
      float v[4] = {acc[i][j][0] + bias4[j].x, acc[i][j][1] + bias4[j].y, acc[i][j][2] + bias4[j].z,
                    acc[i][j][3] + bias4[j].w};
      if (p.rbias) {
        const float4 bb = *reinterpret_cast<const float4*>(p.rbias + (int64_t)(mc / p.rb_g) * p.N + n);
        v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      }
      if (p.tbl) {
        const float4 bb = *reinterpret_cast<const float4*>(p.tbl + (int64_t)(mc % p.tbl_rows) * p.N + n);
        v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      }
      if (p.act == 1) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = gelu_erf(v[t]);
      } else if (p.act == 2) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = fmaxf(v[t], 0.f);
      }
      const int u = (j * 4 + fq) ^ (r & SW);
      *reinterpret_cast<float4*>(lds + r * TN + u * 4) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (i0 == 0) STAMP(4);
  // phase 2: lanes per row = TN/8, rows per pass = 64 / (TN/8)
  constexpr int LPR = TN / 8;
  constexpr int RPP = 64 / LPR;
  const int c8 = lane % LPR;
  const int rr = lane / LPR;
  const int rows = ni * 16;
  for (int r0 = 0; r0 < rows; r0 += RPP) {
    const int r = r0 + rr;
    const int m = mrow0 + i0 * 16 + r;
    const int u0 = (2 * c8) ^ (r & SW), u1 = (2 * c8 + 1) ^ (r & SW);
    const float4 a = *reinterpret_cast<const float4*>(lds + r * TN + u0 * 4);
    const float4 b = *reinterpret_cast<const float4*>(lds + r * TN + u1 * 4);
    if (m >= p.M) continue;
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const int n = ncol0 + c8 * 8;
    int64_t off;
    int orow = 0;
    if (p.ct_s > 0) {
      const int hw = p.ct_h * p.ct_w;
      const int bi = m / hw;
      const int rem = m - bi * hw;
      const int iy = rem / p.ct_w;
      const int ix = rem - iy * p.ct_w;
      const int tap = n / p.ct_c;
      const int co = n - tap * p.ct_c;
      const int dy = tap / p.ct_s, dx = tap - dy * p.ct_s;
      const int64_t W2 = (int64_t)p.ct_w * p.ct_s;
      off = ((((int64_t)bi * p.ct_h + iy) * p.ct_s + dy) * W2 + (int64_t)ix * p.ct_s + dx) * p.ct_c + co;
    } else {
      orow = remap(m, p.o_g, p.o_gs, p.o_o);
      off = (int64_t)orow * p.ldc + n;
    }
    if (p.res) {
      const int64_t roff = p.ct_s > 0 ? off : (int64_t)orow * p.ldr + n;
      if (p.res_f32) {
        const float4 x0 = *reinterpret_cast<const float4*>(static_cast<const float*>(p.res) + roff);
        const float4 x1 = *reinterpret_cast<const float4*>(static_cast<const float*>(p.res) + roff + 4);
        v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
        v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
      } else {
        const uint4 x = *reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(p.res) + roff);
        const uint32_t* q = reinterpret_cast<const uint32_t*>(&x);
#pragma unroll
        for (int t = 0; t < 4; ++t) { v[2 * t] += __uint_as_float(q[t] << 16); v[2 * t + 1] += __uint_as_float(q[t] & 0xffff0000u); }
      }
    }
    if (p.res2) {
      const int64_t roff = p.ct_s > 0 ? off : (int64_t)orow * p.ldr2 + n;
      const uint4 x = *reinterpret_cast<const uint4*>(p.res2 + roff);
      const uint32_t* q = reinterpret_cast<const uint32_t*>(&x);
#pragma unroll
      for (int t = 0; t < 4; ++t) { v[2 * t] += __uint_as_float(q[t] << 16); v[2 * t + 1] += __uint_as_float(q[t] & 0xffff0000u); }
    }
    if (p.c_f32) {
      float* c = static_cast<float*>(p.C) + off;
      *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      uint4 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
      o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
      *reinterpret_cast<uint4*>(static_cast<bf16_t*>(p.C) + off) = o;
    }
  }
}

static int group_m_for(int tiles_m);

// Epilogue for one lane: out[m][n..n+3] = epi(v[0..3]).
__device__ __forceinline__ void epilogue4(const Args& p, int m, int n, float v[4]) {
  int orow = 0;
  int64_t off;
  if (p.ct_s > 0) {
    const int hw = p.ct_h * p.ct_w;
    const int b = m / hw;
    const int rem = m - b * hw;
    const int iy = rem / p.ct_w;
    const int ix = rem - iy * p.ct_w;
    const int tap = n / p.ct_c;
    const int co = n - tap * p.ct_c;
    const int dy = tap / p.ct_s, dx = tap - dy * p.ct_s;
    const int64_t W2 = (int64_t)p.ct_w * p.ct_s;
    off = ((((int64_t)b * p.ct_h + iy) * p.ct_s + dy) * W2 + (int64_t)ix * p.ct_s + dx) * p.ct_c + co;
  } else {
    orow = remap(m, p.o_g, p.o_gs, p.o_o);
    off = (int64_t)orow * p.ldc + n;
  }
  if (p.bias) {
    const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
    v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
  }
  if (p.rbias) {
    const float4 bb = *reinterpret_cast<const float4*>(p.rbias + (int64_t)(m / p.rb_g) * p.N + n);
    v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
  }
  if (p.tbl) {
    const float4 bb = *reinterpret_cast<const float4*>(p.tbl + (int64_t)(m % p.tbl_rows) * p.N + n);
    v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
  }
  if (p.act == 1) {
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = gelu_erf(v[t]);
  } else if (p.act == 2) {
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = fmaxf(v[t], 0.f);
  }
  if (p.res) {
    const int64_t roff = p.ct_s > 0 ? off : (int64_t)orow * p.ldr + n;
    if (p.res_f32) {
      const float4 r = *reinterpret_cast<const float4*>(static_cast<const float*>(p.res) + roff);
      v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
    } else {
      const uint2 r = *reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(p.res) + roff);
      v[0] += __uint_as_float(r.x << 16); v[1] += __uint_as_float(r.x & 0xffff0000u);
      v[2] += __uint_as_float(r.y << 16); v[3] += __uint_as_float(r.y & 0xffff0000u);
    }
  }
  if (p.res2) {
    const int64_t roff = p.ct_s > 0 ? off : (int64_t)orow * p.ldr2 + n;
    const uint2 r = *reinterpret_cast<const uint2*>(p.res2 + roff);
    v[0] += __uint_as_float(r.x << 16); v[1] += __uint_as_float(r.x & 0xffff0000u);
    v[2] += __uint_as_float(r.y << 16); v[3] += __uint_as_float(r.y & 0xffff0000u);
  }
  if (p.c_f32) {
    *reinterpret_cast<float4*>(static_cast<float*>(p.C) + off) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(static_cast<bf16_t*>(p.C) + off) = o;
  }
}

// BM x BN x KB tile, WM x WN waves (64*WM*WN threads), LDS double buffer.
// KB = 64: 128-B LDS rows (swizzle chunk ^ (row & 7)); KB = 32: 64-B rows (swizzle
// chunk ^ ((row >> 1) & 3)), half the LDS per block so 4-5 blocks share a CU and
// cover each other's load latency and epilogues.
template <int BM, int BN, int WM, int WN, int KB, bool CONV, bool RELU_A>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm(Args p) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM;            // activation rows per wave
  constexpr int TN = BN / WN;            // output columns per wave
  constexpr int RM = TM / 16;
  constexpr int RN = TN / 16;
  constexpr int ROWB = KB * 2;           // LDS bytes per row
  constexpr int CPR = KB / 8;            // 16-B chunks per row
  constexpr int RPI = 64 / CPR;          // rows per glds wave-instruction
  constexpr int A_LOADS = BM / (RPI * NW);
  constexpr int W_LOADS = BN / (RPI * NW);
  constexpr int A_BYTES = BM * ROWB;
  constexpr int W_BYTES = BN * ROWB;
  constexpr int STAGE = A_BYTES + W_BYTES;
  constexpr int SUB = KB / 32;           // MFMA k-substeps per stage
  static_assert(RM >= 1 && RN >= 1, "tile too small");
  static_assert(A_LOADS >= 1 && W_LOADS >= 1 && A_LOADS * RPI * NW == BM && W_LOADS * RPI * NW == BN, "load split");
  static_assert(KB == 32 || KB == 64, "KB");

  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / WN;
  const int wn = wid % WN;
  auto swz = [](int row) { return KB == 64 ? (row & 7) : ((row >> 1) & 3); };

  int tm, tn;
  tile_coords(p, blockIdx.x, tm, tn);
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  // ---- per-lane source rows for the A and W glds streams
  const int lrow = lane / CPR;         // row inside an RPI-row glds slab
  const int pchunk = lane % CPR;       // physical 16-B chunk this lane fills
  const bf16_t* a_src[A_LOADS];
  int cpix[A_LOADS], cyx[A_LOADS];
#pragma unroll
  for (int j = 0; j < A_LOADS; ++j) {
    const int row = (wid * A_LOADS + j) * RPI + lrow;
    const int lchunk = pchunk ^ swz(row);
    int m = m0 + row;
    if (m > p.M - 1) m = p.M - 1;
    if (!CONV) {
      a_src[j] = p.A + (int64_t)remap(m, p.a_g, p.a_gs, p.a_o) * p.lda + lchunk * 8;
      cpix[j] = cyx[j] = 0;
    } else {
      const int hw = p.coh * p.cow;
      const int b = m / hw;
      const int rem = m - b * hw;
      const int oy = rem / p.cow;
      const int ox = rem - oy * p.cow;
      cpix[j] = b * p.ch * p.cw;
      cyx[j] = ((oy * p.cs - p.cp) << 16) | ((ox * p.cs - p.cp) & 0xffff);
      a_src[j] = p.A + lchunk * 8;
    }
  }
  const bf16_t* w_src[W_LOADS];
#pragma unroll
  for (int j = 0; j < W_LOADS; ++j) {
    const int row = (wid * W_LOADS + j) * RPI + lrow;
    const int lchunk = pchunk ^ swz(row);
    w_src[j] = p.W + (int64_t)(n0 + row) * p.ldw + lchunk * 8;
  }

  auto stage = [&](int buf, int k0) {
    uint8_t* sA = smem + buf * STAGE;
    uint8_t* sW = sA + A_BYTES;
    if (!CONV) {
#pragma unroll
      for (int j = 0; j < A_LOADS; ++j) glds16(a_src[j] + k0, sA + (wid * A_LOADS + j) * RPI * ROWB);
    } else {
      const int kk = k0 / p.cc;
      const int ky = kk / p.ck;
      const int kx = kk - ky * p.ck;
      const int ci0 = k0 - kk * p.cc;
#pragma unroll
      for (int j = 0; j < A_LOADS; ++j) {
        const int yi = (cyx[j] >> 16) + ky, xi = ((int)(short)(cyx[j] & 0xffff)) + kx;
        const bool ok = yi >= 0 && yi < p.ch && xi >= 0 && xi < p.cw;
        const void* src = ok ? (const void*)(a_src[j] + ((int64_t)cpix[j] + (int64_t)yi * p.cw + xi) * p.cc + ci0)
                             : (const void*)(g_zero + pchunk * 16);
        glds16(src, sA + (wid * A_LOADS + j) * RPI * ROWB);
      }
    }
#pragma unroll
    for (int j = 0; j < W_LOADS; ++j) glds16(w_src[j] + k0, sW + (wid * W_LOADS + j) * RPI * ROWB);
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  STAMP(0);
  const int nk = p.K / KB;
  stage(0, 0);
  __syncthreads();   // waits vmcnt(0): tile 0 landed
  STAMP(1);

  const int frow = lane & 15;
  const int fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * KB);
    const uint8_t* sA = smem + cur * STAGE;
    const uint8_t* sW = sA + A_BYTES;
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
      bf16x8 wf[RN];
      const int lchunk = 4 * s + fq;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = wn * TN + j * 16 + frow;
        wf[j] = *reinterpret_cast<const bf16x8*>(sW + row * ROWB + ((lchunk ^ swz(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = wm * TM + i * 16 + frow;
        bf16x8 af = *reinterpret_cast<const bf16x8*>(sA + row * ROWB + ((lchunk ^ swz(row)) << 4));
        if (RELU_A) af = relu8(af);
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af, acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  STAMP(2);

  // ---- epilogue through this wave's LDS region (the K loop ended with a barrier)
  constexpr int EP_RM0 = (2 * STAGE) / (NW * TN * 4 * 16);   // m-tiles per pass that fit
  constexpr int EP_RM = EP_RM0 < RM ? EP_RM0 : RM;
  static_assert(EP_RM >= 1 && RM % EP_RM == 0, "epilogue LDS");
#pragma unroll
  for (int i0 = 0; i0 < RM; i0 += EP_RM) {
    tile_epilogue<RM, RN>(p, acc, i0, EP_RM, m0 + wm * TM, n0 + wn * TN,
                          reinterpret_cast<float*>(smem) + wid * EP_RM * 16 * TN);
    __builtin_amdgcn_wave_barrier();
  }
  STAMP(3);
}

template <int BM, int BN, int WM, int WN, int KB, bool CONV, bool RELU_A>
static void launch(const Args& p, hipStream_t s) {
  Args q = p;
  q.tiles_m = (p.M + BM - 1) / BM;
  q.tiles_n = p.N / BN;
  q.group_m = group_m_for(q.tiles_m);
  const int smem = 2 * (BM + BN) * KB * 2;
  auto kern = k_gemm<BM, BN, WM, WN, KB, CONV, RELU_A>;
  static bool attr = false;
  if (!attr && smem > 64 * 1024) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(q.tiles_m * q.tiles_n), dim3(64 * WM * WN), smem, s, q);
}

// ---------------------------------------------------------------------------
// 256 x 256 x 64 tile, 8 waves (2 M x 4 N, 128 x 64 outputs per wave), 8 phases
// per pair of K-tiles (cdna_hip_programming.md §5 "256^2 8-phase template",
// re-derived for this layout).  Each K-tile buffer is four 16 KiB half-tiles:
//   A0/A1 = the first/second 64 activation rows of every wave's 128,
//   B0/B1 = the first/second 32 weight rows of every wave's 64.
// Phase q (1..4) of a K-tile computes C-quadrant Q_q = (A0,B0) (A0,B1) (A1,B1)
// (A1,B0) from register subtiles, so half-tiles retire early and are refilled
// one phase after their last ds_read:
//   phase 1: read A0,B0 | glds odd.A1 (tile t+1)     phase 5: read A0,B0 (odd) | glds even.A1 (t+2)
//   phase 2: read B1    | glds even.A0 (t+2)         phase 6: read B1          | glds odd.A0 (t+3)
//   phase 3: read A1    | glds even.B0 (t+2)         phase 7: read A1          | glds odd.B0 (t+3)
//   phase 4: -          | glds even.B1, vmcnt(6)     phase 8: -                | glds odd.B1, vmcnt(6)
// Every phase: reads, glds, [vmcnt], lgkmcnt(0), s_barrier, 16 MFMA, s_barrier.
// The counted vmcnt(6) keeps three half-tiles in flight across the barriers.
template <bool CONV, bool RELU_A>
__global__ __launch_bounds__(512) void k_gemm8(Args p) {
  constexpr int HALF = 128 * 128;            // bytes per half-tile
  constexpr int BUF = 4 * HALF;              // A0 A1 B0 B1
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 2;                   // 0..1
  const int wn = wid & 3;                    // 0..3

  int tm, tn;
  tile_coords(p, blockIdx.x, tm, tn);
  const int m0 = tm * 256;
  const int n0 = tn * 256;

  // per-lane glds sources.  Lane fills local row lr0 = wid*16 + lane/8 (+8 for slab 1) of
  // every half; A half h local row wm'*64 + r <-> tile row wm'*128 + h*64 + r, B half h
  // local row wn'*32 + c <-> weight row wn'*64 + h*32 + c.  Dense rows are affine in
  // (h, slab) (the dispatcher sends row-remapped A to the 128-row kernel), so one base
  // pointer per operand suffices; conv rows keep (pixel base, y, x) per (h, slab).
  const int pchunk = lane & 7;
  const int lr0 = wid * 16 + (lane >> 3);                 // slab 0 row; slab 1 = +8 (same lr>>6, lr>>5)
  const int lchunk0 = pchunk ^ (lr0 & 7);                 // (lr0 + 8) & 7 == lr0 & 7
  const bf16_t* a_base;
  int cpix[2][2], cyx[2][2];
  {
    const int mrow = m0 + (lr0 >> 6) * 128 + (lr0 & 63);
    if (!CONV) {
      a_base = p.A + (int64_t)(mrow + p.a_o) * p.lda + lchunk0 * 8;
    } else {
      a_base = p.A + lchunk0 * 8;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          int m = mrow + h * 64 + j * 8;
          if (m > p.M - 1) m = p.M - 1;
          const int hw = p.coh * p.cow;
          const int b = m / hw;
          const int rem = m - b * hw;
          const int oy = rem / p.cow;
          const int ox = rem - oy * p.cow;
          cpix[h][j] = b * p.ch * p.cw;
          cyx[h][j] = ((oy * p.cs - p.cp) << 16) | ((ox * p.cs - p.cp) & 0xffff);
        }
    }
  }
  const bf16_t* w_base = p.W + (int64_t)(n0 + (lr0 >> 5) * 64 + (lr0 & 31)) * p.ldw + lchunk0 * 8;
  const int64_t a_step_h = (int64_t)64 * p.lda, a_step_j = (int64_t)8 * p.lda;
  const int64_t w_step_h = (int64_t)32 * p.ldw, w_step_j = (int64_t)8 * p.ldw;
  const int m_last = p.M - 1;
  const int row_hi = m0 + (lr0 >> 6) * 128 + (lr0 & 63);   // for dense row clamping

  // glds of one half-tile (2 instructions per thread); which: 0 A0, 1 A1, 2 B0, 3 B1
  auto stage_half = [&](int buf, int which, int k0) {
    uint8_t* dst = smem + buf * BUF + which * HALF;
    const int h = which & 1;
    if (which < 2) {
      if (!CONV) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int m = row_hi + h * 64 + j * 8;
          const bf16_t* src = m <= m_last ? a_base + h * a_step_h + j * a_step_j
                                          : a_base + (int64_t)(m_last - row_hi) * p.lda;
          glds16(src + k0, dst + (wid * 2 + j) * 8 * 128);
        }
      } else {
        const int kk = k0 / p.cc;
        const int ky = kk / p.ck;
        const int kx = kk - ky * p.ck;
        const int ci0 = k0 - kk * p.cc;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int yi = (cyx[h][j] >> 16) + ky, xi = ((int)(short)(cyx[h][j] & 0xffff)) + kx;
          const bool ok = yi >= 0 && yi < p.ch && xi >= 0 && xi < p.cw;
          const void* src = ok ? (const void*)(a_base + ((int64_t)cpix[h][j] + (int64_t)yi * p.cw + xi) * p.cc + ci0)
                               : (const void*)(g_zero + pchunk * 16);
          glds16(src, dst + (wid * 2 + j) * 8 * 128);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) glds16(w_base + h * w_step_h + j * w_step_j + k0, dst + (wid * 2 + j) * 8 * 128);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;
  const int fq = lane >> 4;
  bf16x8 af[2][4];     // A subtile: [substep][m-tile of the quadrant]
  bf16x8 b0f[2][2], b1f[2][2];

  auto read_a = [&](int buf, int h) {
    const uint8_t* base = smem + buf * BUF + h * HALF;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int lr = wm * 64 + i * 16 + frow;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(base + lr * 128 + (((4 * s + fq) ^ (lr & 7)) << 4));
        if (RELU_A) v = relu8(v);
        af[s][i] = v;
      }
  };
  auto read_b = [&](int buf, int h, bf16x8 (&bf)[2][2]) {
    const uint8_t* base = smem + buf * BUF + (2 + h) * HALF;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int lr = wn * 32 + j * 16 + frow;
        bf[s][j] = *reinterpret_cast<const bf16x8*>(base + lr * 128 + (((4 * s + fq) ^ (lr & 7)) << 4));
      }
  };
  auto mma = [&](int mh, int nh, const bf16x8 (&bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh * 4 + i][nh * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[s][j], af[s][i], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
#define I2PC_BAR()                             \
  do {                                         \
    __builtin_amdgcn_sched_barrier(0);         \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_s_barrier();              \
    __builtin_amdgcn_sched_barrier(0);         \
  } while (0)
#define I2PC_VMCNT(n)                          \
  do {                                         \
    __builtin_amdgcn_sched_barrier(0);         \
    asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); \
  } while (0)

  const int nk = p.K / BK;        // even (checked by the dispatcher)
  // prologue: tile 0 complete, tile 1 A0 B0 B1 in flight
  stage_half(0, 0, 0); stage_half(0, 2, 0); stage_half(0, 3, 0); stage_half(0, 1, 0);
  if (nk > 1) { stage_half(1, 0, BK); stage_half(1, 2, BK); stage_half(1, 3, BK); I2PC_VMCNT(6); }
  else { I2PC_VMCNT(0); }
  I2PC_BAR();

  for (int t = 0; t < nk; t += 2) {
    const bool more = t + 2 < nk;                 // tiles t+2, t+3 exist
    const int k2 = (t + 2) * BK, k3 = (t + 3) * BK;
    // ---- even buffer (tile t)
    read_a(0, 0); read_b(0, 0, b0f);
    stage_half(1, 1, (t + 1) * BK);
    I2PC_BAR(); mma(0, 0, b0f); I2PC_BAR();
    read_b(0, 1, b1f);
    if (more) stage_half(0, 0, k2);
    I2PC_BAR(); mma(0, 1, b1f); I2PC_BAR();
    read_a(0, 1);
    if (more) stage_half(0, 2, k2);
    I2PC_BAR(); mma(1, 1, b1f); I2PC_BAR();
    if (more) { stage_half(0, 3, k2); I2PC_VMCNT(6); } else { I2PC_VMCNT(0); }
    I2PC_BAR(); mma(1, 0, b0f); I2PC_BAR();
    // ---- odd buffer (tile t+1)
    read_a(1, 0); read_b(1, 0, b0f);
    if (more) stage_half(0, 1, k2);
    I2PC_BAR(); mma(0, 0, b0f); I2PC_BAR();
    read_b(1, 1, b1f);
    if (more) stage_half(1, 0, k3);
    I2PC_BAR(); mma(0, 1, b1f); I2PC_BAR();
    read_a(1, 1);
    if (more) stage_half(1, 2, k3);
    I2PC_BAR(); mma(1, 1, b1f); I2PC_BAR();
    if (more) { stage_half(1, 3, k3); I2PC_VMCNT(6); } else { I2PC_VMCNT(0); }
    I2PC_BAR(); mma(1, 0, b0f); I2PC_BAR();
  }
#undef I2PC_BAR
#undef I2PC_VMCNT

  // epilogue: wave (wm, wn) holds rows wm*128 + i*16, cols wn*64 + j*16 (the generic
  // kernel's 128 x 64 wave tile), staged through LDS in two passes of 4 m-tiles
  __syncthreads();
#pragma unroll
  for (int i0 = 0; i0 < 8; i0 += 4) {
    tile_epilogue<8, 4>(p, acc, i0, 4, m0 + wm * 128, n0 + wn * 64,
                        reinterpret_cast<float*>(smem) + wid * 4 * 16 * 64);
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------
// 256 x 256 x 32 tile, 8 waves (2 M x 4 N; 128 x 64 outputs per wave), a ring of
// four 32 KiB LDS stages with THREE K-steps of global_load_lds in flight: the
// load of step k+3 is issued before step k computes and only step k+1 is waited
// for (counted vmcnt), so L2-miss / MALL latency (~1 us under load) hides behind
// ~3 K-steps of MFMA work (the 2-stage 128^2 kernel stalls on every step).
// Rows are 64 B (32 bf16); fragments read with ds_read_b128 through the
// conflict-free swizzle chunk ^ ((row >> 1) & 3), applied to the glds SOURCE.
template <bool CONV, bool RELU_A>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_gemm_ring(Args p) {
  constexpr int RBK = 32;
  constexpr int ROWB = RBK * 2;              // 64 B per row
  constexpr int PART = 256 * ROWB;           // 16 KiB (A or W of one stage)
  constexpr int STG = 2 * PART;              // 32 KiB
  constexpr int NST = 4;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 2;                   // 0..1  -> activation rows wm*128
  const int wn = wid & 3;                    // 0..3  -> output cols wn*64
  int tm, tn;
  tile_coords(p, blockIdx.x, tm, tn);
  const int m0 = tm * 256;
  const int n0 = tn * 256;

  // glds mapping: wave-instruction = 16 rows x 4 chunks; thread does 2 A + 2 W per stage
  const int pchunk = lane & 3;
  const bf16_t* a_src[2];
  const bf16_t* w_src[2];
  int cpix[2], cyx[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wid * 2 + j) * 16 + (lane >> 2);          // 0..255
    const int lchunk = pchunk ^ ((row >> 1) & 3);
    int m = m0 + row;
    if (m > p.M - 1) m = p.M - 1;
    if (!CONV) {
      a_src[j] = p.A + (int64_t)remap(m, p.a_g, p.a_gs, p.a_o) * p.lda + lchunk * 8;
      cpix[j] = cyx[j] = 0;
    } else {
      const int hw = p.coh * p.cow;
      const int b = m / hw;
      const int rem = m - b * hw;
      const int oy = rem / p.cow;
      const int ox = rem - oy * p.cow;
      cpix[j] = b * p.ch * p.cw;
      cyx[j] = ((oy * p.cs - p.cp) << 16) | ((ox * p.cs - p.cp) & 0xffff);
      a_src[j] = p.A + lchunk * 8;
    }
    w_src[j] = p.W + (int64_t)(n0 + row) * p.ldw + lchunk * 8;
  }
  auto stage = [&](int buf, int k0) {
    uint8_t* sA = smem + buf * STG;
    uint8_t* sW = sA + PART;
    if (!CONV) {
#pragma unroll
      for (int j = 0; j < 2; ++j) glds16(a_src[j] + k0, sA + (wid * 2 + j) * 16 * ROWB);
    } else {
      const int kk = k0 / p.cc;
      const int ky = kk / p.ck;
      const int kx = kk - ky * p.ck;
      const int ci0 = k0 - kk * p.cc;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int yi = (cyx[j] >> 16) + ky, xi = ((int)(short)(cyx[j] & 0xffff)) + kx;
        const bool ok = yi >= 0 && yi < p.ch && xi >= 0 && xi < p.cw;
        const void* src = ok ? (const void*)(a_src[j] + ((int64_t)cpix[j] + (int64_t)yi * p.cw + xi) * p.cc + ci0)
                             : (const void*)(g_zero + pchunk * 16);
        glds16(src, sA + (wid * 2 + j) * 16 * ROWB);
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) glds16(w_src[j] + k0, sW + (wid * 2 + j) * 16 * ROWB);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;
  const int fq = lane >> 4;
  const int nk = p.K / RBK;
  // prologue: stages 0..2 in flight, wait for stage 0
  stage(0, 0);
  if (nk > 1) stage(1, RBK);
  if (nk > 2) stage(2, 2 * RBK);
  __builtin_amdgcn_sched_barrier(0);
  if (nk > 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (nk > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 3 < nk) stage((kt + 3) & (NST - 1), (kt + 3) * RBK);
    const uint8_t* sA = smem + (kt & (NST - 1)) * STG;
    const uint8_t* sW = sA + PART;
    bf16x8 wf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + j * 16 + frow;
      wf[j] = *reinterpret_cast<const bf16x8*>(sW + row * ROWB + ((fq ^ ((row >> 1) & 3)) << 4));
    }
    bf16x8 af[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wm * 128 + i * 16 + frow;
      af[i] = *reinterpret_cast<const bf16x8*>(sA + row * ROWB + ((fq ^ ((row >> 1) & 3)) << 4));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (RELU_A) af[i] = relu8(af[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
    }
    // step kt+1 must have landed; everyone must be done reading stage kt before it is refilled
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 3 < nk) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    else if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }

  // epilogue in two passes of 64 rows through this wave's 16 KiB LDS region
  float* elds = reinterpret_cast<float*>(smem) + wid * 64 * 64;
  tile_epilogue<8, 4>(p, acc, 0, 4, m0 + wm * 128, n0 + wn * 64, elds);
  __builtin_amdgcn_wave_barrier();
  tile_epilogue<8, 4>(p, acc, 4, 4, m0 + wm * 128, n0 + wn * 64, elds);
}

static int group_m_for(int tiles_m) {
  static const int env = [] { const char* e = getenv("I2PC_GEMM_GM"); return e ? atoi(e) : 0; }();
  const int g = env > 0 ? env : 8;
  return std::max(1, std::min(g, tiles_m));
}

template <bool CONV, bool RELU_A>
static void launch_ring(const Args& p, hipStream_t s) {
  Args q = p;
  q.tiles_m = (p.M + 255) / 256;
  q.tiles_n = p.N / 256;
  q.group_m = group_m_for(q.tiles_m);
  const int smem = 4 * 32 * 1024;   // 128 KiB
  auto kern = k_gemm_ring<CONV, RELU_A>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(q.tiles_m * q.tiles_n), dim3(512), smem, s, q);
}

template <bool CONV, bool RELU_A>
static void launch8(const Args& p, hipStream_t s) {
  Args q = p;
  q.tiles_m = (p.M + 255) / 256;
  q.tiles_n = p.N / 256;
  q.group_m = group_m_for(q.tiles_m);
  const int smem = 8 * 128 * 128;   // 128 KiB
  auto kern = k_gemm8<CONV, RELU_A>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(q.tiles_m * q.tiles_n), dim3(512), smem, s, q);
}


template <bool CONV, bool RELU_A>
static int dispatch(const Args& p, hipStream_t s) {
  const int64_t t256 = (int64_t)((p.M + 255) / 256) * (p.N / 256);
  const int64_t t128 = (int64_t)((p.M + 127) / 128) * (p.N / 128);
  static const int force = [] { const char* e = getenv("I2PC_GEMM_TILE"); return e ? atoi(e) : 0; }();
  const bool even_k = (p.K / BK) % 2 == 0;
  const bool big_ok = p.N % 256 == 0 && even_k && (CONV || p.a_g == 0);
  if (force == 8 && big_ok) launch8<CONV, RELU_A>(p, s);
  else if (force == 4 && p.N % 256 == 0) launch_ring<CONV, RELU_A>(p, s);
  else if (force == 256 && p.N % 256 == 0) launch<256, 256, 2, 4, 64, CONV, RELU_A>(p, s);
  else if (force == 25632 && p.N % 256 == 0) launch<256, 256, 2, 4, 32, CONV, RELU_A>(p, s);
  else if (force == 128 && p.N % 128 == 0) launch<128, 128, 2, 2, 64, CONV, RELU_A>(p, s);
  else if (force == 12832 && p.N % 128 == 0) launch<128, 128, 2, 2, 32, CONV, RELU_A>(p, s);
  else if (p.N % 256 == 0 && t256 >= 512) launch<256, 256, 2, 4, 64, CONV, RELU_A>(p, s);
  else if (p.N % 128 == 0 && t128 >= 512) launch<128, 128, 2, 2, 64, CONV, RELU_A>(p, s);
  else if (p.N % 64 == 0) launch<128, 64, 2, 2, 64, CONV, RELU_A>(p, s);
  else if (p.N % 32 == 0) launch<128, 32, 4, 1, 64, CONV, RELU_A>(p, s);
  else return set_error(I2PC_EUNSUPPORTED, "gemm: N=%d must be a multiple of 32", p.N);
  return check_launch("gemm");
}

}  // namespace gemm
}  // namespace i2pc

using namespace i2pc;

#ifdef I2PC_STAMPS
extern "C" int i2pc_debug_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(i2pc::gemm::g_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int i2pc_gemm(const i2pc_gemm_desc* d, void* stream) {
  clear_error();
  I2PC_REQUIRE(d != nullptr, "desc is NULL");
  I2PC_REQUIRE(d->a && d->w && d->c, "NULL operand");
  I2PC_REQUIRE(d->m > 0 && d->n > 0 && d->k > 0, "empty gemm");
  I2PC_REQUIRE(d->k % 64 == 0, "gemm: K=%d must be a multiple of 64", d->k);
  I2PC_REQUIRE(d->n % 4 == 0, "gemm: N must be a multiple of 4");
  gemm::Args p{};
  p.A = static_cast<const gemm::bf16_t*>(d->a);
  p.lda = d->lda; p.M = d->m; p.N = d->n; p.K = d->k;
  p.a_g = d->a_group; p.a_gs = d->a_group_stride; p.a_o = d->a_offset;
  p.W = static_cast<const gemm::bf16_t*>(d->w); p.ldw = d->ldw;
  p.bias = d->bias;
  p.rbias = d->row_bias; p.rb_g = d->row_bias_group > 0 ? d->row_bias_group : 1;
  p.tbl = d->table; p.tbl_rows = d->table_rows > 0 ? d->table_rows : 1;
  p.act = d->act;
  p.res = d->res; p.res_f32 = d->res_f32; p.ldr = d->ldr;
  p.res2 = static_cast<const gemm::bf16_t*>(d->res2); p.ldr2 = d->ldr2;
  p.C = d->c; p.c_f32 = d->c_f32; p.ldc = d->ldc;
  p.o_g = d->out_group; p.o_gs = d->out_group_stride; p.o_o = d->out_offset;
  p.ct_s = d->convt_s; p.ct_h = d->convt_h; p.ct_w = d->convt_w; p.ct_c = d->convt_c;
  hipStream_t s = as_stream(stream);
  if (d->conv) {
    I2PC_REQUIRE(d->conv_c % 64 == 0, "conv: Cin=%d must be a multiple of 64", d->conv_c);
    I2PC_REQUIRE(d->k == d->conv_k * d->conv_k * d->conv_c, "conv: K != k*k*Cin");
    I2PC_REQUIRE(d->m == d->conv_batch * d->conv_oh * d->conv_ow, "conv: M != B*OH*OW");
    p.cb = d->conv_batch; p.ch = d->conv_h; p.cw = d->conv_w; p.cc = d->conv_c;
    p.coh = d->conv_oh; p.cow = d->conv_ow; p.ck = d->conv_k; p.cs = d->conv_stride; p.cp = d->conv_pad;
    return d->conv_relu_in ? gemm::dispatch<true, true>(p, s) : gemm::dispatch<true, false>(p, s);
  }
  return d->conv_relu_in ? gemm::dispatch<false, true>(p, s) : gemm::dispatch<false, false>(p, s);
}

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
#include "mx.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace i2pc {
namespace gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;

constexpr int BK = 64;

// A-fragment look-ahead of the bf16 K-steps: m-subtiles whose LDS reads are issued ahead of their
// MFMAs, the order pinned by scheduling groups (0 = the compiler's own schedule, which at 245 VGPRs
// reused one fragment register: read -> lgkmcnt(0) -> 4 MFMAs per m-subtile, every LDS latency exposed
// to the matrix pipe).  r05, in one box: persistent LN-fold QKV / FC1 7.23 -> 6.89 ms per C2 step
// with 2 (3: equal), step 21.77 -> 21.34 ms, bit-identical.  The tile kernel (I2PC_GEMM_APF_TILE) got
// slower with it: its 320 x 256 O / FC2 calls 6.21 -> 6.62 ms per step at 2 or 3 (DA-v2's 384 x 192
// equal), so it keeps the compiler's schedule.  The fp8 path of the persistent engine with one m-subtile
// of look-ahead (two would spill) measured equal on C5 (26.40 vs 26.37 ms per step), not kept.
// Variants: tools/build_variant.sh.
#ifndef I2PC_GEMM_APF
#define I2PC_GEMM_APF 2
#endif
#ifndef I2PC_GEMM_APF_TILE
#define I2PC_GEMM_APF_TILE 0
#endif

__device__ __attribute__((aligned(16))) uint8_t g_zero[1024];  // conv zero padding / absent-bias source
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
// persistent engine: per (block, tile ordinal < 8) four stamps
#define PSTAMP(ti, k)                                                                 \
  do {                                                                                \
    if (threadIdx.x == 0 && (ti) < 8) {                                               \
      unsigned long long t_;                                                          \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
      g_stamps[(blockIdx.x * 8 + (ti)) * 8 + (k)] = t_;                               \
    }                                                                                 \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#define PSTAMP(ti, k) do {} while (0)
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
  uint32_t a_bytes, w_bytes;   // buffer ranges of A and W (persistent engine)
  // MX fp8 engine: E8M0 scale dwords [rows][K / 128] (byte b = 32-k block b of the 128-k step)
  const uint32_t* As; int64_t ldas;    // A scales, dwords per row (conv: per pixel, Cin / 128)
  const uint32_t* Ws; int64_t ldws;    // W scales
  uint32_t* Cs; int64_t ldcs;          // fp8 output scales (EPI_Q8), dwords per row
  uint32_t as_bytes, ws_bytes;
  int kspan;   // split-K (tile kernel): K-steps per blockIdx.y slice, 0 = the whole K
  // LayerNorm fold (i2pc.h): consumer row scales float2 [M] + column sums [N]; producer chunk
  // partials float2 [M][N / lnc] (lnc = 64 or 32 columns per chunk) + the bf16 copy of the fp32 output
  const float* lnr; const float* csum;
  float* lnp; bf16_t* cbf; int64_t ldcb;
  const float* lnsh;
  int lnc;
  const float* rsh;   // bf16 residual stored relative to rsh[row] (i2pc.h res_shift)
  int stagger;    // persistent engine: waves 4-7 issue the next K-stage's loads half-way through a step
                  // (knob "gemm_stagger")
  int dbg_drop;   // diagnostic (I2PC_GEMM_DROP_STORES=1): the persistent engine's output stores are issued to an
                  // empty buffer range (dropped), to measure what the stores cost the next tile's K-loop
  int resq;       // tile kernel: residual rows through LDS in the epilogue (knob "gemm_resq")
  int simple;     // tile / halo kernels: the compiled-down epilogues where they apply (knob "gemm_simple_epi")
};

__device__ __forceinline__ int g_resq_dev(const Args& p) { return p.resq; }

__device__ __forceinline__ int remap(int m, int g, int gs, int o) {
  return g > 0 ? (m / g) * gs + (m % g) + o : m + o;
}

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ bf16_t f2bf(float x) {
  __bf16 b = (__bf16)x;
  return *reinterpret_cast<bf16_t*>(&b);
}

// GELU with the exact (erf) form, erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far
// below the bf16 rounding of the output): one reciprocal, one exp2, six FMAs instead of
// ocml's branchy erff (which made the fc1 epilogue cost ~half a K-loop).
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y *= t;
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  const float erf_abs = fmaf(-y, e, 1.0f);
  const float erf_v = __builtin_copysignf(erf_abs, x);
  return 0.5f * x * (1.0f + erf_v);
}

// GELU in the tanh form, x * sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)) = x / (1 + exp2(x (c1 + c2 x^2))):
// five VALU and two transcendentals instead of the erf form's ~14 and two (|GELU_tanh - GELU_erf| <=
// 2.2e-4, a few per cent of a bf16 output ulp).  Activation code 3 (knob "gelu_tanh"); the epilogues of
// the short-K GEMMs that take GELU (FC1 at K = 384 / 1024) are VALU-bound when every wave of a tile runs
// its epilogue at once.
__device__ __forceinline__ float gelu_tanh(float x) {
  constexpr float c1 = -2.3022082f;                 // -2 sqrt(2/pi) log2(e)
  constexpr float c2 = -2.3022082f * 0.044715f;
  const float u = x * __builtin_fmaf(x * x, c2, c1);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
}

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds_base), 16, 0, 0);
}

// ReLU on 8 packed bf16 (pre-activation residual units): clear negative lanes.
// As signed 16-bit integers the bf16 values with the sign bit set are exactly the negative ones, so
// max(x, 0) on packed int16 (v_pk_max_i16, one VALU per pair) clears them to +0 and keeps the rest.
__device__ __forceinline__ bf16x8 relu8(bf16x8 v) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 x = __builtin_bit_cast(s16x8, v);
  return __builtin_bit_cast(bf16x8, __builtin_elementwise_max(x, s16x8{0, 0, 0, 0, 0, 0, 0, 0}));
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

// v of another lane by a DPP permutation (0xB1: lane ^ 1, 0x4E: lane ^ 2 inside a quad; 0x141: the
// 8-lane half-row mirror, lane 7 - i)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// ---------------------------------------------------------------------------
// Tile epilogue through LDS (the MFMA layout gives each lane 4 columns of one row,
// i.e. 8-byte stores scattered over 16 rows -- issue-bound, ~10k cycles per 128^2
// tile).  Phase 1 (MFMA layout): v = act(acc + bias + row_bias + table) -> fp32 in
// the wave's LDS region (16-B units XOR-swizzled by row).  Phase 2 (row layout):
// each lane owns 8 consecutive columns of one row: + res + res2 with 16/32-B loads,
// then one 16-B (bf16) or 2 x 16-B (fp32) store; a wave writes whole 128-B lines.
// f(0), f(1), ..., f(N - 1) as straight-line code (each call inlined with a constant argument)
template <int N, int I = 0, class F>
__device__ __forceinline__ void epi_passes(F&& f) {
  if constexpr (I < N) {
    f(I);
    epi_passes<N, I + 1>(f);
  }
}

// Residual rows staged through LDS by the tile epilogue (ResQ; the 8-wave 320 x 256 tile kernel with a
// bf16 residual -- DPT-Large's attention-out / FC2 LayerNorm producers on the bf16 stream).  Read in the
// epilogue's phase 2 by plain loads, each pass's residual load sat behind the previous iteration's
// stores: vmcnt retires in issue order, so every iteration waited for a store's round trip (phase 2 of
// the producer ~57-61 K cycles against ~19-42 K for a plain store epilogue, r04 stamps).  Here pass
// p + 1's residual rows go to LDS by LDS-DMA, issued once pass p's phase 1 is done and before its
// stores, and pass p + 1 waits once (vmcnt(0)) instead of once per iteration.  The DMA is inline asm,
// invisible to the compiler (a builtin LDS-DMA made it wait vmcnt(0) before every later LDS access).
// On the RQ path (tile_epilogue<..., RQP = true>) nothing else is loaded after the first pass: the bias
// comes in registers from the caller (b4) and the wave's row shifts (res_shift, ln_shift) go to LDS by
// one LDS-DMA each before pass 0 (rsl: [rs: TM floats][sh: TM floats]), so a pass's only wait is for its
// residual rows -- counted past the previous pass's stores (full: the wave's rows are all < M, so each
// phase-2 iteration issued at least one store) instead of vmcnt(0), which waited for those stores too.
struct ResQ {
  int on;
  uint8_t* buf;          // [2][NW][EP_RM * 16 rows][128 B] (after the phase-1 staging region)
  uint8_t* rsl;          // this wave's row shifts in LDS (RQP)
  const float4* b4;      // this lane's bias columns (RQP)
  int full;
};

__device__ __forceinline__ void dma16_gemm(__amdgpu_buffer_rsrc_t rs, uint32_t lds_base, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs), "s"(0u)
               : "memory", "m0");
}
// the same with sc1 (agent scope: per-call row shifts written by the launch before)
__device__ __forceinline__ void dma16_gemm_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t lds_base, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen sc1 lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs), "s"(0u)
               : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Spatial output tile of the halo convolution (k_conv3_halo): local row r of the tile is pixel
// (ty0 + r / tw, tx0 + r % tw) of image b; rows outside the output map are skipped.
struct SpTile {
  int base;          // b * oh * ow
  int ty0, tx0, tw, oh, ow;
};

// RQP: the RQ path (struct ResQ).  SIMPLE 1 / 2: bias (+ activation: 2) (+ bf16 residuals) -> bf16 only
// (simple_epilogue).  Both compile out the generic epilogue's other features: the code a call runs
// through is then a fraction of the generic one's, whose runtime-skipped branches made a plain bf16
// store epilogue of the 320 x 256 tile as slow as the LayerNorm producer's (tools/stamps_tile.py).
// which compiled-down epilogue a call can use: 1 / 2 = tile_epilogue<..., SIMPLE> without / with an
// activation, 3 = fp32 rows (+ bias) (+ an fp32 residual), no activation (split-K partial sums, the fp32
// residual stream's attention-out / FC2 of DPT-Hybrid), 0 = the generic one
__device__ __forceinline__ int simple_kind(const Args& p) {
  if (!p.simple) return 0;
  const bool s = !p.rbias && !p.tbl && p.ct_s == 0 && p.o_g == 0 && p.o_o == 0 && !p.lnp && !p.rsh;
  if (s && p.c_f32) return (!p.res || p.res_f32) && !p.res2 && p.act == 0 ? 3 : 0;
  return s && !(p.res && p.res_f32) ? (p.act == 0 ? 1 : 2) : 0;
}

template <int RM, int RN, int NI, bool SPAT = false, bool RQP = false, int SIMPLE = 0>
__device__ __forceinline__ void tile_epilogue(const Args& p, f32x4 (&acc)[RM][RN], int i0, int mrow0,
                                              int ncol0, float* lds, SpTile sp = SpTile{}, ResQ rq = ResQ{}) {
  constexpr bool NO_EXTRA = RQP || SIMPLE != 0;     // no row bias, table, res2, fp32 out, scatter, row map
  constexpr bool NO_ACT = RQP || SIMPLE == 1 || SIMPLE == 3;
  constexpr bool F32_ONLY = SIMPLE == 3;            // fp32 rows (+ an fp32 residual)
  constexpr bool NO_LNP = SIMPLE != 0;
  constexpr int ni = NI;
  constexpr int TN = RN * 16;
  constexpr int U = TN / 4;                 // 16-B units per LDS row
  constexpr int SW = U >= 8 ? 7 : U - 1;    // swizzle mask
  const int lane = threadIdx.x & 63;
  const int frow = lane & 15;
  const int fq = lane >> 4;
  // phase 2 layout: lanes per row = TN/8, rows per pass = 64 / (TN/8)
  constexpr int LPR = TN / 8;
  constexpr int RPP = 64 / LPR;
  constexpr int ITS = (NI * 16 + RPP - 1) / RPP;
  const int c8 = lane % LPR;
  const int rr = lane / LPR;
  // LayerNorm producer: the row shifts of this pass's phase-2 iterations are loaded before any of its
  // stores.  vmcnt retires in issue order, so a load issued behind a store cannot be consumed before
  // that store has completed; loaded in each iteration, they chained every iteration behind the
  // previous one's stores (r04, tools/diag12.sh: O 70 -> 68 us, DA-v2's 384 x 192 producer 100 -> 95 us).
  // Prefetching the residual rows as well was no faster: before phase 1 it pushed the 320 x 256 kernel
  // into scratch, after phase 1 (registers free) it measured 2-3 % slower (tools/diag17.sh).
  constexpr bool PRE_SH = ITS <= 10 && !RQP && SIMPLE == 0;
  const bool pre = p.lnp && p.ct_s == 0;
  float pre_rs[PRE_SH ? ITS : 1], pre_sh[PRE_SH ? ITS : 1];
  if (PRE_SH && pre) {
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
      const int r = it * RPP + rr;
      const int m = mrow0 + i0 * 16 + r;
      if ((LPR * RPP < 64 && (rr >= RPP || r >= ni * 16)) || m >= p.M) continue;
      const int orow = remap(m, p.o_g, p.o_gs, p.o_o);
      // per-call row shifts, written by the launch before: agent-scope loads
      if (p.rsh) pre_rs[it] = __hip_atomic_load(p.rsh + orow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (p.lnsh) pre_sh[it] = __hip_atomic_load(p.lnsh + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // residual rows through LDS (ResQ): one 16-B DMA per lane and 8 rows, [row][128 B] per wave and pass
  constexpr int NPASS = RM / NI;
  const int pass = i0 / NI;
  const int wid_q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t rq_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.res), 0, (uint32_t)((int64_t)p.M * p.ldr * 2), 0x00020000);
  // [NI * 16 rows][TN * 2 B] per wave and pass: element e = 16-B chunk e % LPR of row e / LPR
  constexpr int RQ_ELEMS = NI * 16 * LPR, RQ_BYTES = NI * 16 * TN * 2;
  auto res_dma = [&](int ps) {
    uint8_t* dst = rq.buf + ((ps & 1) * 8 + wid_q) * RQ_BYTES;
#pragma unroll
    for (int j = 0; j < (RQ_ELEMS + 63) / 64; ++j) {
      const int e = j * 64 + lane;
      const int r = e / LPR, ch = e - (e / LPR) * LPR;
      const int m = mrow0 + ps * NI * 16 + r;
      const uint32_t off = (m < p.M && e < RQ_ELEMS) ? (uint32_t)((m * p.ldr + ncol0 + ch * 8) * 2) : 0x7FFFFFF0u;
      dma16_gemm(rq_rs, __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(dst + j * 1024)), off);
    }
  };
  constexpr bool RQ_OK = (TN == 64 || TN == 96) && !SPAT;
  constexpr int TMW = RM * 16;              // the wave's rows
  static_assert(!RQP || (RQ_OK && TMW <= 256), "RQ path");
  if constexpr (RQP) {
    if (pass == 0) {
      // the wave's row shifts, 4 rows per lane, before any store of the epilogue (see ResQ)
      if (lane < TMW / 4) {
        const uint32_t off = (uint32_t)((mrow0 + 4 * lane) * 4);
        const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)rq.rsl;
        if (p.rsh)
          dma16_gemm_sc1(__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.rsh), 0, (uint32_t)(p.M * 4), 0x00020000),
                         __builtin_amdgcn_readfirstlane(base), off);
        if (p.lnsh)
          dma16_gemm_sc1(__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.lnsh), 0, (uint32_t)(p.M * 4), 0x00020000),
                         __builtin_amdgcn_readfirstlane(base + TMW * 4), off);
      }
      res_dma(0);
    }
  } else if constexpr (RQ_OK) {
    if (rq.on && pass == 0) res_dma(0);
  }
  // bias depends on the column only: load it once, all loads in flight together
  float4 bias4[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j)
    bias4[j] = RQP ? rq.b4[j]
                   : p.bias ? *reinterpret_cast<const float4*>(p.bias + ncol0 + j * 16 + fq * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
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
      if (!NO_EXTRA && p.rbias) {
        const float4 bb = *reinterpret_cast<const float4*>(p.rbias + (int64_t)(mc / p.rb_g) * p.N + n);
        v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      }
      if (!NO_EXTRA && p.tbl) {
        const float4 bb = *reinterpret_cast<const float4*>(p.tbl + (int64_t)(mc % p.tbl_rows) * p.N + n);
        v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      }
      if (NO_ACT) {
      } else if (p.act == 1) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = gelu_erf(v[t]);
      } else if (p.act == 3) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = gelu_tanh(v[t]);
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
  const uint8_t* rq_cur = nullptr;
  if constexpr (RQP) {
    // this pass's rows landed: issued before the previous pass's >= ITS stores, which may stay in flight
    if (pass == 1) STAMP(6);
    if (pass > 0 && rq.full) wait_vm<ITS>();
    else wait_vm<0>();
    if (pass == 1) STAMP(5);
    if (pass == NPASS - 1) STAMP(7);
    if (pass + 1 < NPASS) res_dma(pass + 1);
    rq_cur = rq.buf + ((pass & 1) * 8 + wid_q) * RQ_BYTES;
  } else if constexpr (RQ_OK) {
    if (rq.on) {
      // this pass's rows landed (and the previous pass's stores drained: one wait per pass), then the
      // next pass's rows start while this pass computes and stores
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (pass + 1 < NPASS) res_dma(pass + 1);
      rq_cur = rq.buf + ((pass & 1) * 8 + wid_q) * RQ_BYTES;
    }
  }
  if (i0 == 0) STAMP(4);
  // phase 2
  const int rows = ni * 16;
#pragma unroll
  for (int it = 0; it < ITS; ++it) {
    const int r0 = it * RPP;
    const int r = r0 + rr;
    // TN = 96: 12 lanes per row, 5 rows per pass (60 lanes), and 48 rows are not a multiple of 5
    if (LPR * RPP < 64 && (rr >= RPP || r >= rows)) continue;
    int m = mrow0 + i0 * 16 + r;
    if constexpr (SPAT) {   // mrow0: the wave's first local row of the spatial tile
      const int py = m / sp.tw, px = m - py * sp.tw;
      m = (sp.ty0 + py < sp.oh && sp.tx0 + px < sp.ow) ? sp.base + (sp.ty0 + py) * sp.ow + sp.tx0 + px : p.M;
    }
    const int u0 = (2 * c8) ^ (r & SW), u1 = (2 * c8 + 1) ^ (r & SW);
    const float4 a = *reinterpret_cast<const float4*>(lds + r * TN + u0 * 4);
    const float4 b = *reinterpret_cast<const float4*>(lds + r * TN + u1 * 4);
    if (m >= p.M) continue;
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const int n = ncol0 + c8 * 8;
    int64_t off;
    int orow = 0;
    if (NO_EXTRA) {
      orow = m;
      off = (int64_t)m * p.ldc + n;
    } else if (p.ct_s > 0) {
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
    if (RQP || p.res) {
      const int64_t roff = (!NO_EXTRA && p.ct_s > 0) ? off : (int64_t)orow * p.ldr + n;
      if (F32_ONLY || (!NO_EXTRA && p.res_f32)) {
        const float4 x0 = *reinterpret_cast<const float4*>(static_cast<const float*>(p.res) + roff);
        const float4 x1 = *reinterpret_cast<const float4*>(static_cast<const float*>(p.res) + roff + 4);
        v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
        v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
      } else {
        const uint4 x = (RQP || rq_cur) ? *reinterpret_cast<const uint4*>(rq_cur + (r * LPR + c8) * 16)
                               : *reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(p.res) + roff);
        const uint32_t* q = reinterpret_cast<const uint32_t*>(&x);
        if (SIMPLE == 0 && p.rsh) {   // shifted bf16 residual stream: value = stored + its row's shift
          const float rs = RQP ? reinterpret_cast<const float*>(rq.rsl)[i0 * 16 + r]
                           : PRE_SH && pre ? pre_rs[PRE_SH ? it : 0]
                                           : __hip_atomic_load(p.rsh + orow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            v[2 * t] += __uint_as_float(q[t] << 16) + rs;
            v[2 * t + 1] += __uint_as_float(q[t] & 0xffff0000u) + rs;
          }
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) { v[2 * t] += __uint_as_float(q[t] << 16); v[2 * t + 1] += __uint_as_float(q[t] & 0xffff0000u); }
        }
      }
    }
    if ((!NO_EXTRA || SIMPLE == 1 || SIMPLE == 2) && p.res2) {
      const int64_t roff = (!NO_EXTRA && p.ct_s > 0) ? off : (int64_t)orow * p.ldr2 + n;
      const uint4 x = *reinterpret_cast<const uint4*>(p.res2 + roff);
      const uint32_t* q = reinterpret_cast<const uint32_t*>(&x);
#pragma unroll
      for (int t = 0; t < 4; ++t) { v[2 * t] += __uint_as_float(q[t] << 16); v[2 * t + 1] += __uint_as_float(q[t] & 0xffff0000u); }
    }
    if (F32_ONLY || (!NO_EXTRA && p.c_f32) || (!NO_LNP && p.lnp)) {
      if (F32_ONLY || (!NO_EXTRA && p.c_f32)) {
        float* c = static_cast<float*>(p.C) + off;
        *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
      if constexpr (LPR % 4 == 0 && !NO_LNP) {
        if (p.lnp) {
          // LayerNorm producer: the bf16 copy of out - shift[m], and (mean, M2) of each 64-column
          // chunk (= 8 lanes) of it, or of each 32-column chunk (4 lanes; lnc = 32)
          const float shf = p.lnsh ? (RQP ? reinterpret_cast<const float*>(rq.rsl)[TMW + i0 * 16 + r]
                                      : PRE_SH && pre ? pre_sh[PRE_SH ? it : 0]
                                                      : __hip_atomic_load(p.lnsh + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                                    : 0.f;
          float u[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) u[t] = v[t] - shf;
          uint4 o;
          o.x = pk2bf(u[0], u[1]);
          o.y = pk2bf(u[2], u[3]);
          o.z = pk2bf(u[4], u[5]);
          o.w = pk2bf(u[6], u[7]);
          *reinterpret_cast<uint4*>(p.cbf + (int64_t)m * p.ldcb + n) = o;
          // chunk sums across the row's lanes by DPP (one VALU each) instead of ds_bpermute round trips:
          // lane ^ 1, lane ^ 2 inside a quad, then the mirrored lane of the 8-lane group (7 - lane: the
          // other quad, whose lanes all hold that quad's sum by then) -- the same operands as xor 4
          float sm = ((u[0] + u[1]) + (u[2] + u[3])) + ((u[4] + u[5]) + (u[6] + u[7]));
          sm += dpp_f<0xB1>(sm);
          sm += dpp_f<0x4E>(sm);
          const bool c64 = LPR % 8 == 0 && p.lnc == 64;   // the host allows 64 only where LPR % 8 == 0
          if (c64) sm += dpp_f<0x141>(sm);
          const float mean = sm * (c64 ? 1.0f / 64.0f : 1.0f / 32.0f);
          float q = 0.f;
#pragma unroll
          for (int t = 0; t < 8; ++t) q = __builtin_fmaf(u[t] - mean, u[t] - mean, q);
          q += dpp_f<0xB1>(q);
          q += dpp_f<0x4E>(q);
          if (c64) q += dpp_f<0x141>(q);
          if ((c8 & (c64 ? 7 : 3)) == 0) {
            const int cs = c64 ? 6 : 5;
            *reinterpret_cast<float2*>(p.lnp + ((int64_t)m * (p.N >> cs) + (n >> cs)) * 2) = make_float2(mean, q);
          }
        }
      }
    } else {
      uint4 o;
      o.x = pk2bf(v[0], v[1]);
      o.y = pk2bf(v[2], v[3]);
      o.z = pk2bf(v[4], v[5]);
      o.w = pk2bf(v[6], v[7]);
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
  } else if (p.act == 3) {
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = gelu_tanh(v[t]);
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
    o.x = pk2bf(v[0], v[1]);
    o.y = pk2bf(v[2], v[3]);
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
  // split-K: slice blockIdx.y covers K-steps [kt0, kt0 + nk) and writes its raw fp32 partial
  // sums to slab blockIdx.y of the workspace (the host passes a plain fp32 epilogue)
  int nk = p.K / KB, kt0 = 0;
  if (p.kspan > 0) {
    kt0 = blockIdx.y * p.kspan;
    nk = min(nk - kt0, p.kspan);
    p.C = static_cast<float*>(p.C) + (int64_t)blockIdx.y * p.M * p.N;
  }
  stage(0, kt0 * KB);
  __syncthreads();   // waits vmcnt(0): tile 0 landed
  STAMP(1);

  const int frow = lane & 15;
  const int fq = lane >> 4;
  // 8 waves: the second half (the SIMD partners of waves 0-3) issue the next stage half-way through
  // the step, so one wave's MFMAs cover the other's LDS-DMA issue (the persistent engine's stagger)
  const bool late = NW == 8 && SUB == 2 && p.stagger && wid >= 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk && !late) stage(cur ^ 1, (kt0 + kt + 1) * KB);
    const uint8_t* sA = smem + cur * STAGE;
    const uint8_t* sW = sA + A_BYTES;
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
      if (s == 1 && late && kt + 1 < nk) {
        __builtin_amdgcn_sched_barrier(0);
        stage(cur ^ 1, (kt0 + kt + 1) * KB);
        __builtin_amdgcn_sched_barrier(0);
      }
      bf16x8 wf[RN];
      const int lchunk = 4 * s + fq;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = wn * TN + j * 16 + frow;
        wf[j] = *reinterpret_cast<const bf16x8*>(sW + row * ROWB + ((lchunk ^ swz(row)) << 4));
      }
#if I2PC_GEMM_APF_TILE > 0
      // A fragments I2PC_GEMM_APF_TILE m-subtiles ahead of their MFMAs (as the persistent engine)
      constexpr int APF = I2PC_GEMM_APF_TILE < RM ? I2PC_GEMM_APF_TILE : RM;
      bf16x8 afr[RM];
      auto a_read = [&](int i) {
        const int row = wm * TM + i * 16 + frow;
        afr[i] = *reinterpret_cast<const bf16x8*>(sA + row * ROWB + ((lchunk ^ swz(row)) << 4));
      };
#pragma unroll
      for (int i = 0; i < APF; ++i) a_read(i);
      __builtin_amdgcn_sched_group_barrier(0x100, RN + APF, 0);
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        if (i + APF < RM) {
          a_read(i + APF);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        bf16x8 af = afr[i];
        if (RELU_A) af = relu8(af);
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af, acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, RN, 0);
      }
#else
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = wm * TM + i * 16 + frow;
        bf16x8 af = *reinterpret_cast<const bf16x8*>(sA + row * ROWB + ((lchunk ^ swz(row)) << 4));
        if (RELU_A) af = relu8(af);
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af, acc[i][j], 0, 0, 0);
      }
#endif
    }
    __syncthreads();
  }
  STAMP(2);

  // ---- epilogue through this wave's LDS region (the K loop ended with a barrier)
  constexpr int EP_RM0 = (2 * STAGE) / (NW * TN * 4 * 16);   // m-tiles per pass that fit
  constexpr int EP_RM1 = EP_RM0 < RM ? EP_RM0 : RM;
  constexpr int EP_RM = RM % EP_RM1 == 0 ? EP_RM1 : RM % (EP_RM1 - 1) == 0 ? EP_RM1 - 1
                      : RM % (EP_RM1 - 2) == 0 ? EP_RM1 - 2 : 1;   // largest divisor of RM that fits
  static_assert(EP_RM >= 1 && RM % EP_RM == 0, "epilogue LDS");
  // the passes as a compile-time sequence (a `#pragma unroll` loop over them can exceed the
  // unroller's size limit, and a rolled loop puts acc[][] in scratch)
  // residual rows through LDS (ResQ): the passes' m-subtiles (EP_RQ, a divisor of RM) sized so the
  // phase-1 staging and two passes of bf16 residual rows fit the K-loop's LDS
  constexpr int EP_RQ0 = (2 * STAGE) / (NW * 16 * TN * 8);
  constexpr int EP_RQ = EP_RQ0 >= 1 ? (RM % EP_RQ0 == 0 ? EP_RQ0 : (EP_RQ0 >= 2 && RM % (EP_RQ0 - 1) == 0) ? EP_RQ0 - 1 : 1) : 0;
  ResQ rq{};
  constexpr int RQ_STAGING = NW * EP_RQ * 16 * TN * 4, RQ_ROWS = 2 * NW * EP_RQ * 16 * TN * 2;
  constexpr bool RQ_SHIFTS = RQ_STAGING + RQ_ROWS + NW * TM * 8 <= 2 * STAGE;   // room for the row shifts
  if constexpr (NW == 8 && (TN == 64 || TN == 96) && EP_RQ >= 1) {
    if (g_resq_dev(p) && p.res && !p.res_f32 && p.ct_s == 0 && p.o_g == 0 && p.o_o == 0 && p.kspan == 0) {
      rq.on = 1;
      rq.buf = smem + RQ_STAGING;
    }
  }
  if constexpr (EP_RQ >= 1 && RQ_SHIFTS && NW == 8 && (TN == 64 || TN == 96)) {
    // the RQ path's epilogue is compiled for exactly these calls (tile_epilogue<..., RQP>: no row bias,
    // table, activation, second residual or fp32 output)
    if (rq.on && g_resq_dev(p) >= 2 && p.act == 0 && !p.rbias && !p.tbl && !p.res2 && !p.c_f32) {
      float4 b4[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j)
        b4[j] = p.bias ? *reinterpret_cast<const float4*>(p.bias + n0 + wn * TN + j * 16 + ((threadIdx.x & 63) >> 4) * 4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      rq.rsl = smem + RQ_STAGING + RQ_ROWS + wid * TM * 8;
      rq.b4 = b4;
      rq.full = m0 + wm * TM + TM <= p.M;
      epi_passes<RM / EP_RQ>([&](int pass) {
        tile_epilogue<RM, RN, EP_RQ, false, true>(p, acc, pass * EP_RQ, m0 + wm * TM, n0 + wn * TN,
                                                  reinterpret_cast<float*>(smem) + wid * EP_RQ * 16 * TN, SpTile{}, rq);
        __builtin_amdgcn_wave_barrier();
      });
      STAMP(3);
      return;
    }
  }
  if constexpr (EP_RQ >= 1) {
    if (rq.on) {
      epi_passes<RM / EP_RQ>([&](int pass) {
        tile_epilogue<RM, RN, EP_RQ>(p, acc, pass * EP_RQ, m0 + wm * TM, n0 + wn * TN,
                                     reinterpret_cast<float*>(smem) + wid * EP_RQ * 16 * TN, SpTile{}, rq);
        __builtin_amdgcn_wave_barrier();
      });
      STAMP(3);
      return;
    }
  }
  const int sk = simple_kind(p);
  if (sk == 1) {
    epi_passes<RM / EP_RM>([&](int pass) {
      tile_epilogue<RM, RN, EP_RM, false, false, 1>(p, acc, pass * EP_RM, m0 + wm * TM, n0 + wn * TN,
                                                    reinterpret_cast<float*>(smem) + wid * EP_RM * 16 * TN);
      __builtin_amdgcn_wave_barrier();
    });
  } else if (sk == 3) {
    epi_passes<RM / EP_RM>([&](int pass) {
      tile_epilogue<RM, RN, EP_RM, false, false, 3>(p, acc, pass * EP_RM, m0 + wm * TM, n0 + wn * TN,
                                                    reinterpret_cast<float*>(smem) + wid * EP_RM * 16 * TN);
      __builtin_amdgcn_wave_barrier();
    });
  } else if (sk == 2) {
    epi_passes<RM / EP_RM>([&](int pass) {
      tile_epilogue<RM, RN, EP_RM, false, false, 2>(p, acc, pass * EP_RM, m0 + wm * TM, n0 + wn * TN,
                                                    reinterpret_cast<float*>(smem) + wid * EP_RM * 16 * TN);
      __builtin_amdgcn_wave_barrier();
    });
  } else {
    epi_passes<RM / EP_RM>([&](int pass) {
      tile_epilogue<RM, RN, EP_RM>(p, acc, pass * EP_RM, m0 + wm * TM, n0 + wn * TN,
                                   reinterpret_cast<float*>(smem) + wid * EP_RM * 16 * TN);
      __builtin_amdgcn_wave_barrier();
    });
  }
  STAMP(3);
}

// 8-wave GEMM kernels (tile and persistent): waves 4-7 issue each next K-stage half-way through the
// step (I2PC_GEMM_STAGGER / "gemm_stagger"; bit-identical either way)
static thread_local int g_stagger = [] { const char* e = getenv("I2PC_GEMM_STAGGER"); return e ? atoi(e) : 1; }();
// tile epilogue: a bf16 residual's rows staged in LDS one pass ahead (ResQ; I2PC_GEMM_RESQ / "gemm_resq");
// 2 = the RQ path (struct ResQ; its epilogue compiled without the generic one's runtime-skipped features):
// measured r06 in one process (tools/ab_pipeline.py), C2 18.675 -> 18.347 ms per step, DA-v2 7.074 ->
// 6.815 ms, bit-identical.  Per call (tools/stamps_tile.py): DPT-Large O 64.8 -> 53.4 us (epilogue phase 2
// 47 K -> 19 K stamp cycles), FC2 172.5 -> 164.7 us; DA-v2 FC2 87.0 -> 71.7 us, O 46.8 -> 33.5 us
static thread_local int g_resq = [] { const char* e = getenv("I2PC_GEMM_RESQ"); return e ? atoi(e) : 2; }();
// tile / halo kernel epilogues compiled without the generic one's features for calls that use none of them
// (bias, activation, bf16 residual, bf16 out; I2PC_GEMM_SIMPLE_EPI / "gemm_simple_epi"; bit-identical)
static thread_local int g_simple = [] { const char* e = getenv("I2PC_GEMM_SIMPLE_EPI"); return e ? atoi(e) : 1; }();

template <int BM, int BN, int WM, int WN, int KB, bool CONV, bool RELU_A>
static void launch(const Args& p, hipStream_t s, int splits = 1) {
  Args q = p;
  q.tiles_m = (p.M + BM - 1) / BM;
  q.tiles_n = p.N / BN;
  q.group_m = group_m_for(q.tiles_m);
  q.stagger = g_stagger;
  q.resq = g_resq;
  q.simple = g_simple;
  const int smem = 2 * (BM + BN) * KB * 2;
  auto kern = k_gemm<BM, BN, WM, WN, KB, CONV, RELU_A>;
  static bool attr = false;
  if (!attr && smem > 64 * 1024) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(q.tiles_m * q.tiles_n, splits), dim3(64 * WM * WN), smem, s, q);
}

// Split-K reduction: out = epilogue(sum over slabs z = 0..splits-1 of ws[z][m][n], in that
// order), 4 columns per thread (epilogue4: the tile kernel's epilogue arithmetic).  M * N / 4
// < 2^31 (plan).
__global__ __launch_bounds__(256) void k_splitk_reduce(Args p, const float* __restrict__ ws, int splits) {
  const uint32_t n4 = (uint32_t)p.N >> 2;
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= (uint32_t)p.M * n4) return;
  const uint32_t m = i / n4;
  const uint32_t n = (i - m * n4) * 4u;
  const int64_t slab = (int64_t)p.M * p.N;
  const float* src = ws + (int64_t)m * p.N + n;
  float4 a = *reinterpret_cast<const float4*>(src);
#pragma unroll 4
  for (int z = 1; z < splits; ++z) {
    const float4 b = *reinterpret_cast<const float4*>(src + z * slab);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  float v[4] = {a.x, a.y, a.z, a.w};
  epilogue4(p, (int)m, (int)n, v);
}

// ---------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 convolution of a 64-channel NHWC bf16 map with an LDS input halo
// (k_conv3_halo; the 64-channel fusion / head convs of Depth-Anything-V2-Small,
// modeling_depth_anything.py DepthAnythingPreActResidualLayer / DepthAnythingDepthEstimationHead).
// The implicit-GEMM tile kernel stages every tap's A rows by LDS-DMA -- nine 128-B rows per output
// pixel per 64 channels -- and with N = 64 its K-step is bound by that DMA issue (24 wave-instructions
// for 8 MFMAs per wave, measured 0.56 PF at M = 701 K).  Here a workgroup owns TH x TW output pixels
// of one image: their (TH + 2) x (TW + 2) input pixels (64 channels = one 128-B row each, zero
// outside the image) land in LDS once, and the nine taps read their A fragments from that halo at
// row (py + ky) * (TW + 2) + px + kx; only the tap's BN x 64 weight tile is double-buffered per
// K-step.  K order = tap-major, as the implicit GEMM's (k = tap * 64 + ci, two 32-k MFMA sub-steps
// per tap), so the result is bit-identical to it.  Epilogue: the tile kernel's (bias, act,
// residuals, bf16 / fp32 out) through a spatial row map.
template <int TH, int TW, int BN, int WM, int WN, bool RELU_A>
__global__ __launch_bounds__(64 * WM * WN) void k_conv3_halo(Args p) {
  constexpr int NW = WM * WN, BM = TH * TW, TM = BM / WM, TN = BN / WN, RM = TM / 16, RN = TN / 16;
  constexpr int HW_ = TW + 2, HR = (TH + 2) * HW_;
  constexpr int HR8 = (HR + 7) / 8;                 // halo DMA wave-instructions (8 rows of 128 B each)
  constexpr int HALO_BYTES = HR8 * 8 * 128;
  constexpr int WBYTES = BN * 128;                  // one tap's weight tile
  constexpr int W_LOADS = BN / (8 * NW);
  static_assert(RM >= 1 && RN >= 1 && W_LOADS >= 1 && W_LOADS * 8 * NW == BN, "tile");
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* sH = smem;
  uint8_t* sWb = smem + HALO_BYTES;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_x = (p.cow + TW - 1) / TW, tiles_y = (p.coh + TH - 1) / TH;
  int t = blockIdx.x;
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int b = t / tiles_y;
  const int y0 = ty * TH, x0 = tx * TW;
  const int n0 = blockIdx.y * BN;

  const __amdgpu_buffer_rsrc_t a_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.A), 0, (uint32_t)((int64_t)p.cb * p.ch * p.cw * 128), 0x00020000);
  const __amdgpu_buffer_rsrc_t w_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.W), 0, (uint32_t)((int64_t)p.N * p.ldw * 2), 0x00020000);
  const int lrow = lane >> 3, pchunk = lane & 7;

  // the halo: row R = hy * HW_ + hx <- input pixel (y0 - 1 + hy, x0 - 1 + hx); 16-B chunk pchunk of
  // the LDS row holds logical chunk pchunk ^ (R & 7) (the source-address swizzle of the engines)
  for (int j = wid; j < HR8; j += NW) {
    const int R = j * 8 + lrow;
    const int hy = R / HW_, hx = R - hy * HW_;
    const int yi = y0 - 1 + hy, xi = x0 - 1 + hx;
    const bool ok = R < HR && (unsigned)yi < (unsigned)p.ch && (unsigned)xi < (unsigned)p.cw;
    const int off = ok ? ((b * p.ch + yi) * p.cw + xi) * 128 + ((pchunk ^ (R & 7)) << 4) : 0x7FFFFFF0;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rs, (lds_ptr_t)(sH + j * 1024), 16, off, 0, 0, 0);
  }
  // tap t's weights: rows n0 .. n0 + BN of W [N][9 * 64], columns t * 64 .. + 64
  const int w_voff = (n0 + wid * W_LOADS * 8 + lrow) * (int)p.ldw * 2 + ((pchunk ^ lrow) << 4);
  auto stage_w = [&](int buf, int tap) {
#pragma unroll
    for (int j = 0; j < W_LOADS; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(w_rs, (lds_ptr_t)(sWb + buf * WBYTES + (wid * W_LOADS + j) * 1024), 16,
                                                w_voff + j * 8 * (int)p.ldw * 2, tap * 128, 0, 0);
  };
  stage_w(0, 0);

  const int frow = lane & 15, fq = lane >> 4;
  int hb[RM];                         // halo row of tap (0, 0) for each m-subtile of this lane
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int r = wm * TM + i * 16 + frow;
    const int py = r / TW, px = r - py * TW;
    hb[i] = py * HW_ + px;
  }
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();   // (vmcnt(0)) the halo and tap 0's weights landed

  for (int tap = 0; tap < 9; ++tap) {
    const int cur = tap & 1;
    if (tap + 1 < 9) stage_w(cur ^ 1, tap + 1);
    const uint8_t* sW = sWb + cur * WBYTES;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int hoff = ky * HW_ + kx;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int lchunk = 4 * s + fq;
      bf16x8 wf[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = wn * TN + j * 16 + frow;
        wf[j] = *reinterpret_cast<const bf16x8*>(sW + row * 128 + ((lchunk ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int R = hb[i] + hoff;
        bf16x8 af = *reinterpret_cast<const bf16x8*>(sH + R * 128 + ((lchunk ^ (R & 7)) << 4));
        if (RELU_A) af = relu8(af);
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af, acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();   // (vmcnt(0)) the next tap's weights landed; this tap's buffer may be refilled
  }

  // epilogue through this wave's LDS region (the halo and weight buffers are dead)
  constexpr int LDS_ALL = HALO_BYTES + 2 * WBYTES;
  constexpr int EP_RM0 = LDS_ALL / (NW * TN * 4 * 16);
  constexpr int EP_RM1 = EP_RM0 < RM ? EP_RM0 : RM;
  constexpr int EP_RM = RM % EP_RM1 == 0 ? EP_RM1 : RM % (EP_RM1 - 1) == 0 ? EP_RM1 - 1 : 1;
  static_assert(EP_RM >= 1 && RM % EP_RM == 0, "epilogue LDS");
  const SpTile sp{b * p.coh * p.cow, y0, x0, TW, p.coh, p.cow};
  const int sk = simple_kind(p);
  if (sk == 1) {
    epi_passes<RM / EP_RM>([&](int pass) {
      tile_epilogue<RM, RN, EP_RM, true, false, 1>(p, acc, pass * EP_RM, wm * TM, n0 + wn * TN,
                                                   reinterpret_cast<float*>(smem) + wid * EP_RM * 16 * TN, sp);
      __builtin_amdgcn_wave_barrier();
    });
  } else if (sk == 2) {
    epi_passes<RM / EP_RM>([&](int pass) {
      tile_epilogue<RM, RN, EP_RM, true, false, 2>(p, acc, pass * EP_RM, wm * TM, n0 + wn * TN,
                                                   reinterpret_cast<float*>(smem) + wid * EP_RM * 16 * TN, sp);
      __builtin_amdgcn_wave_barrier();
    });
  } else {
    epi_passes<RM / EP_RM>([&](int pass) {
      tile_epilogue<RM, RN, EP_RM, true>(p, acc, pass * EP_RM, wm * TM, n0 + wn * TN,
                                         reinterpret_cast<float*>(smem) + wid * EP_RM * 16 * TN, sp);
      __builtin_amdgcn_wave_barrier();
    });
  }
}

template <int TH, int TW, int BN, int WM, int WN, bool RELU_A>
static void launch_halo(const Args& p, hipStream_t s) {
  constexpr int HR8 = ((TH + 2) * (TW + 2) + 7) / 8;
  const int smem = HR8 * 8 * 128 + 2 * BN * 128;
  auto kern = k_conv3_halo<TH, TW, BN, WM, WN, RELU_A>;
  static bool attr = false;
  if (!attr && smem > 64 * 1024) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int tiles = p.cb * ((p.coh + TH - 1) / TH) * ((p.cow + TW - 1) / TW);
  Args q = p;
  q.simple = g_simple;
  hipLaunchKernelGGL(kern, dim3(tiles, p.N / BN), dim3(64 * WM * WN), smem, s, q);
}

// ---------------------------------------------------------------------------
// Persistent 256-column GEMM (BM x 256 x 64 tiles, BM = 256 or 320, 8 waves as
// 2 M x 4 N, wave tile (BM/2) x 64).  One workgroup per CU walks a strided list
// of tiles (XCD-contiguous slots, GROUP_M order inside a round).  What it hides
// that the one-tile-per-workgroup kernel cannot:
//  * the next tile's first K-stage (and its bias row) is issued by
//    global_load_lds during the current tile's last K-step, so no tile starts
//    cold;
//  * the epilogue is register-direct (no LDS round trip; bf16 pairs widened to
//    16-B stores with v_permlane16_swap) through buffer stores whose count per
//    wave is fixed, so the next tile's first wait is a counted vmcnt that lets
//    those stores drain behind the next tile's MFMAs instead of stalling on them;
//  * residual operands are read by inline-asm buffer loads one m-subtile ahead
//    with counted waits, so they never wait for the stores issued before them.
// Every epilogue memory operation is unconditional (rows past M go to an
// out-of-range buffer offset: loads read 0, stores are dropped), which is what
// makes the counted waits exact.
namespace pers {

using namespace ::i2pc::mx;

enum { EPI_PLAIN = 0, EPI_RESF32 = 1, EPI_RESBF16 = 2, EPI_RES2 = 3, EPI_CT = 4, EPI_Q8 = 5, EPI_LNF = 6, EPI_LNP = 7,
       EPI_LNPB = 8 };
constexpr int OOB = 0x7FFFFFF0;   // buffer range; offsets >= OOB are dropped / read as 0

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

__device__ __forceinline__ rsrc_t make_rsrc(const void* ptr) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), 0, OOB, 0x00020000);
}

__device__ __forceinline__ void grouped(const Args& p, int tile, int& tm, int& tn) {
  const int gsz = p.group_m * p.tiles_n;
  const int g = tile / gsz;
  const int first = g * p.group_m;
  const int gm = min(p.tiles_m - first, p.group_m);
  const int in = tile - g * gsz;
  tm = first + in % gm;
  tn = in / gm;
}

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  return pk2bf(a, b);
}

template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if constexpr (ACT == 1) return gelu_erf(x);
  else if constexpr (ACT == 3) return gelu_tanh(x);
  else if constexpr (ACT == 2) return fmaxf(x, 0.f);
  else return x;
}

// Byte offset of output element (m, n) (row remap or ConvTranspose pixel shuffle).
__device__ __forceinline__ int out_elem(const Args& p, int m, int n, int64_t ld, bool ct) {
  if (ct) {
    const int hw = p.ct_h * p.ct_w;
    const int bi = m / hw;
    const int rem = m - bi * hw;
    const int iy = rem / p.ct_w;
    const int ix = rem - iy * p.ct_w;
    const int tap = n / p.ct_c;
    const int co = n - tap * p.ct_c;
    const int dy = tap / p.ct_s, dx = tap - dy * p.ct_s;
    const int W2 = p.ct_w * p.ct_s;
    return (((bi * p.ct_h + iy) * p.ct_s + dy) * W2 + ix * p.ct_s + dx) * p.ct_c + co;
  }
  return remap(m, p.o_g, p.o_gs, p.o_o) * (int)ld + n;
}

#define I2PC_WAIT_VM(n)                                      \
  do {                                                       \
    __builtin_amdgcn_sched_barrier(0);                       \
    asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory");    \
  } while (0)
#define I2PC_LDS_BARRIER()                                   \
  do {                                                       \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       \
    __builtin_amdgcn_s_barrier();                            \
    __builtin_amdgcn_sched_barrier(0);                       \
  } while (0)

template <int EPI> struct EpiCount {
  static constexpr int loads = EPI == EPI_RESF32 || EPI == EPI_RESBF16 || EPI == EPI_LNP || EPI == EPI_LNPB ? 4
                               : EPI == EPI_RES2 ? 8 : 0;
  // EPI_LNP: 4 fp32 rows + 2 bf16 (shifted copy) + 1 chunk-partials store per m-subtile;
  // EPI_LNPB (bf16 residual stream): 2 bf16 (the stream, in place) + 1 chunk-partials store
  static constexpr int stores = EPI == EPI_RESF32 ? 4 : EPI == EPI_Q8 ? 5 : EPI == EPI_LNP ? 7 : EPI == EPI_LNPB ? 3 : 2;
};

// Register-direct tile epilogue of the persistent engines for one wave: rows mw0 + i*16 + (lane & 15),
// columns ncol + j*16 + (lane >> 4)*4 (the swapped 16x16 MFMA layout), j < RN.  Issues exactly
// RM * (loads + stores) vector-memory instructions (EpiCount), all unconditional -- plus, only in
// the fp8 engine, plain row-bias / table loads the counted waits tolerate (extra, older-first).
// EPI_LNF (LayerNorm fold, i2pc.h): t = rs.x * acc + rs.y * col_sum + bias with the wave's row
// scales rs (float2, from LDS at rows_lds[local row]) and column sums (LDS, like the bias).
// EPI_LNPB (LayerNorm-fold producer on the shifted bf16 residual stream, i2pc.h res_shift): the
// tile kernel's bf16-output producer -- v = act(acc + bias) + (res + res_shift[row]), the stream
// written back in place as bf16(v - ln_shift[row]) with the chunk partials of v - ln_shift
// (rows_lds: the ln shifts, rsh_lds: the res shifts, both staged in LDS with the tile's bias).
template <int RM, int RN, int EPI, bool F8>
__device__ __forceinline__ void epilogue_p(const Args& p, f32x4 (&acc)[RM][RN], int mw0, int ncol, const float* bias_lds,
                                           rsrc_t c_rs, rsrc_t r_rs, rsrc_t r2_rs, rsrc_t cs_rs,
                                           const float* csum_lds = nullptr, const float* rows_lds = nullptr,
                                           const float* rsh_lds = nullptr) {
    static_assert((EPI != EPI_LNP && EPI != EPI_LNPB) || RN == 4,
                  "EPI_LNP / EPI_LNPB: a wave's 64 columns are one LayerNorm chunk (or two of 32)");
    constexpr int NRL = EpiCount<EPI>::loads, NS = EpiCount<EPI>::stores;
    static_assert(RN == 2 || RN == 4, "RN");
    const int lane = threadIdx.x & 63;
    const int frow = lane & 15, fq = lane >> 4;
    float4 bias4[RN], csum4[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) bias4[j] = *reinterpret_cast<const float4*>(bias_lds + fq * 4 + j * 16);
    if constexpr (EPI == EPI_LNF) {
#pragma unroll
      for (int j = 0; j < RN; ++j) csum4[j] = *reinterpret_cast<const float4*>(csum_lds + fq * 4 + j * 16);
    }
    const int mrow = mw0 + frow;       // + i * 16
    const int act = p.act;
    constexpr bool CT = EPI == EPI_CT;
    constexpr bool OUTF = EPI == EPI_RESF32;
    // residual loads of m-subtile i into slot i & 1 (acc layout: 4 columns per lane)
    f32x4 rf[2][RN];
    u32x2 rb[2][RN], rb2[2][RN];
    auto load_res = [&](int i, int slot) {
      const int m = mrow + i * 16;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = ncol + j * 16 + fq * 4;
        if constexpr (EPI == EPI_RESF32 || EPI == EPI_LNP) {
          const int off = m < p.M ? (remap(m, p.o_g, p.o_gs, p.o_o) * (int)p.ldr + n) * 4 : OOB;
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(rf[slot][j]) : "v"(off), "s"(r_rs) : "memory");
        }
        if constexpr (EPI == EPI_RESBF16 || EPI == EPI_RES2 || EPI == EPI_LNPB) {
          const int off = m < p.M ? (remap(m, p.o_g, p.o_gs, p.o_o) * (int)p.ldr + n) * 2 : OOB;
          asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(rb[slot][j]) : "v"(off), "s"(r_rs) : "memory");
        }
        if constexpr (EPI == EPI_RES2) {
          const int off = m < p.M ? (remap(m, p.o_g, p.o_gs, p.o_o) * (int)p.ldr2 + n) * 2 : OOB;
          asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(rb2[slot][j]) : "v"(off), "s"(r2_rs) : "memory");
        }
      }
    };
    // one straight-line copy of the epilogue per activation
    auto epilogue = [&](auto actc) {
    constexpr int ACT = decltype(actc)::value;
    if constexpr (NRL > 0) load_res(0, 0);
    static_for<0, RM>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int slot = i & 1;
      if constexpr (NRL > 0) {
        if constexpr (i + 1 < RM) load_res(i + 1, slot ^ 1);
        constexpr int after = (i + 1 < RM ? NRL * RN / 4 : 0) + (i > 0 ? NS : 0);
        if constexpr (EPI == EPI_RESF32 || EPI == EPI_LNP) {
          if constexpr (RN == 4)
            asm volatile("s_waitcnt vmcnt(%c4)" : "+v"(rf[slot][0]), "+v"(rf[slot][1]), "+v"(rf[slot][2]), "+v"(rf[slot][3])
                         : "i"(after) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%c2)" : "+v"(rf[slot][0]), "+v"(rf[slot][1]) : "i"(after) : "memory");
        } else if constexpr (EPI == EPI_RESBF16 || EPI == EPI_LNPB) {
          if constexpr (RN == 4)
            asm volatile("s_waitcnt vmcnt(%c4)" : "+v"(rb[slot][0]), "+v"(rb[slot][1]), "+v"(rb[slot][2]), "+v"(rb[slot][3])
                         : "i"(after) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%c2)" : "+v"(rb[slot][0]), "+v"(rb[slot][1]) : "i"(after) : "memory");
        } else {
          if constexpr (RN == 4)
            asm volatile("s_waitcnt vmcnt(%c8)"
                         : "+v"(rb[slot][0]), "+v"(rb[slot][1]), "+v"(rb[slot][2]), "+v"(rb[slot][3]),
                           "+v"(rb2[slot][0]), "+v"(rb2[slot][1]), "+v"(rb2[slot][2]), "+v"(rb2[slot][3])
                         : "i"(after) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%c4)" : "+v"(rb[slot][0]), "+v"(rb[slot][1]), "+v"(rb2[slot][0]), "+v"(rb2[slot][1])
                         : "i"(after) : "memory");
        }
      }
      const int m = mrow + i * 16;
      const bool ok = m < p.M;
      const int mc = ok ? m : p.M - 1;
      float v[RN][4];
      float2 rs = make_float2(1.f, 0.f);
      if constexpr (EPI == EPI_LNF) rs = *reinterpret_cast<const float2*>(rows_lds + (i * 16 + frow) * 2);
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        float t[4];
        if constexpr (EPI == EPI_LNF) {
          t[0] = __builtin_fmaf(acc[i][j][0], rs.x, __builtin_fmaf(csum4[j].x, rs.y, bias4[j].x));
          t[1] = __builtin_fmaf(acc[i][j][1], rs.x, __builtin_fmaf(csum4[j].y, rs.y, bias4[j].y));
          t[2] = __builtin_fmaf(acc[i][j][2], rs.x, __builtin_fmaf(csum4[j].z, rs.y, bias4[j].z));
          t[3] = __builtin_fmaf(acc[i][j][3], rs.x, __builtin_fmaf(csum4[j].w, rs.y, bias4[j].w));
        } else {
          t[0] = acc[i][j][0] + bias4[j].x; t[1] = acc[i][j][1] + bias4[j].y;
          t[2] = acc[i][j][2] + bias4[j].z; t[3] = acc[i][j][3] + bias4[j].w;
        }
        if constexpr (F8 && (EPI == EPI_PLAIN || EPI == EPI_Q8)) {   // per-image row bias (DPT readout CLS half), position table
          const int n = ncol + j * 16 + fq * 4;
          if (p.rbias) {
            const float4 bb = *reinterpret_cast<const float4*>(p.rbias + (int64_t)(mc / p.rb_g) * p.N + n);
            t[0] += bb.x; t[1] += bb.y; t[2] += bb.z; t[3] += bb.w;
          }
          if (p.tbl) {
            const float4 bb = *reinterpret_cast<const float4*>(p.tbl + (int64_t)(mc % p.tbl_rows) * p.N + n);
            t[0] += bb.x; t[1] += bb.y; t[2] += bb.z; t[3] += bb.w;
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] = act_f<ACT>(t[e]);
        if constexpr (EPI == EPI_RESF32 || EPI == EPI_LNP) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[j][e] += rf[slot][j][e];
        }
        if constexpr (EPI == EPI_RESBF16 || EPI == EPI_RES2) {
          v[j][0] += __uint_as_float(rb[slot][j].x << 16); v[j][1] += __uint_as_float(rb[slot][j].x & 0xffff0000u);
          v[j][2] += __uint_as_float(rb[slot][j].y << 16); v[j][3] += __uint_as_float(rb[slot][j].y & 0xffff0000u);
        }
        if constexpr (EPI == EPI_LNPB) {   // the tile kernel's order: v + (stored + shift)
          const float rsv = rsh_lds[i * 16 + frow];
          v[j][0] += __uint_as_float(rb[slot][j].x << 16) + rsv; v[j][1] += __uint_as_float(rb[slot][j].x & 0xffff0000u) + rsv;
          v[j][2] += __uint_as_float(rb[slot][j].y << 16) + rsv; v[j][3] += __uint_as_float(rb[slot][j].y & 0xffff0000u) + rsv;
        }
        if constexpr (EPI == EPI_RES2) {
          v[j][0] += __uint_as_float(rb2[slot][j].x << 16); v[j][1] += __uint_as_float(rb2[slot][j].x & 0xffff0000u);
          v[j][2] += __uint_as_float(rb2[slot][j].y << 16); v[j][3] += __uint_as_float(rb2[slot][j].y & 0xffff0000u);
        }
      }
      if constexpr (EPI == EPI_Q8) {
        // MX fp8 output: blocks of 32 columns = j pair (2q, 2q+1) x the 4 lanes fq of one row
        constexpr int NB = RN / 2;
        uint32_t sbytes = 0;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          float am = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) am = fmaxf(am, fmaxf(fabsf(v[2 * q][e]), fabsf(v[2 * q + 1][e])));
          am = fmaxf(am, __shfl_xor(am, 16));
          am = fmaxf(am, __shfl_xor(am, 32));
          const int ex = mx_exponent(am);
          const float mul = exp2i(-ex);
          sbytes |= (uint32_t)(ex + 127) << (8 * q);
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * q + jj;
            const uint32_t d = pack_e4m3(v[j][0] * mul, v[j][1] * mul, v[j][2] * mul, v[j][3] * mul);
            const int off = ok ? remap(m, p.o_g, p.o_gs, p.o_o) * (int)p.ldc + ncol + j * 16 + fq * 4 : OOB;
            __builtin_amdgcn_raw_buffer_store_b32(d, c_rs, off, 0, 0);
          }
        }
        if constexpr (RN == 2) {   // keep the per-i store count at 5 (RN / 2 = 1 data pair -> pad)
          __builtin_amdgcn_raw_buffer_store_b32(0u, c_rs, OOB, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(0u, c_rs, OOB, 0, 0);
        }
        // scale bytes of the row's blocks ncol/32 .. + NB - 1, by the fq == 0 lane
        const int soff = (ok && fq == 0) ? remap(m, p.o_g, p.o_gs, p.o_o) * (int)p.ldcs * 4 + ncol / 32 : OOB;
        if constexpr (NB == 2) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)sbytes, cs_rs, soff, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b8((uint8_t)sbytes, cs_rs, soff, 0, 0);
      } else if constexpr (EPI == EPI_LNP || EPI == EPI_LNPB) {
        // LayerNorm-fold producer (the tile kernel's tile_epilogue, same values bit for bit): the fp32
        // output (EPI_LNP; the bf16 stream has none), a bf16 copy of u = out - shift[m], and per 64 (or
        // 32) columns (mean, M2) of u summed in the tile kernel's order -- there a lane holds 8
        // consecutive columns of a row and the chunk is reduced over lane groups by xor 1, 2, 4; here a
        // lane holds 4 columns of each 16-column group j, so 8-column group g = 2 j + (fq >> 1) is split
        // over lanes fq = 2 h, 2 h + 1 (lane xor 16), g ^ 1 is lane xor 32, g ^ 2 is j ^ 1 and g ^ 4 is
        // j ^ 2 (fp32 addition commutes).
        if constexpr (EPI == EPI_LNP) {
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            const int off = ok ? out_elem(p, m, ncol + j * 16 + fq * 4, p.ldc, false) * 4 : OOB;
            const u32x4 d = {__float_as_uint(v[j][0]), __float_as_uint(v[j][1]), __float_as_uint(v[j][2]),
                             __float_as_uint(v[j][3])};
            __builtin_amdgcn_raw_buffer_store_b128(d, c_rs, off, 0, 0);
          }
        }
        const float sh = rows_lds[i * 16 + frow];
        float u[RN][4];
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) u[j][e] = v[j][e] - sh;
#pragma unroll
        for (int pp = 0; pp < RN / 2; ++pp) {
          uint32_t x0 = pack_bf16(u[2 * pp][0], u[2 * pp][1]), x1 = pack_bf16(u[2 * pp][2], u[2 * pp][3]);
          uint32_t y0 = pack_bf16(u[2 * pp + 1][0], u[2 * pp + 1][1]), y1 = pack_bf16(u[2 * pp + 1][2], u[2 * pp + 1][3]);
          const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
          const int n = ncol + 32 * pp + (fq & 1) * 16 + (fq >> 1) * 8;
          const int off = ok ? (m * (int)p.ldcb + n) * 2 : OOB;
          const u32x4 d = {s0[0], s1[0], s0[1], s1[1]};
          __builtin_amdgcn_raw_buffer_store_b128(d, r2_rs, off, 0, 0);
        }
        const bool c64 = p.lnc == 64;
        float sm[RN], mean[RN], q[RN];
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const float a = (u[j][0] + u[j][1]) + (u[j][2] + u[j][3]);
          sm[j] = a + __shfl_xor(a, 16);             // the 8-column group
          sm[j] += __shfl_xor(sm[j], 32);            // + group g ^ 1
        }
        {
          float t2[RN];
#pragma unroll
          for (int j = 0; j < RN; ++j) t2[j] = sm[j] + sm[j ^ 1];               // + g ^ 2
#pragma unroll
          for (int j = 0; j < RN; ++j) mean[j] = c64 ? (t2[j] + t2[j ^ 2]) * (1.0f / 64.0f) : t2[j] * (1.0f / 32.0f);
        }
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          // the tile kernel's sequential fma chain over the group's 8 columns: the low 4 (lane fq even)
          // first, continued by the high 4 (lane fq odd) from the low lane's partial
          float x = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) x = __builtin_fmaf(u[j][e] - mean[j], u[j][e] - mean[j], x);
          float y = __shfl_xor(x, 16);
#pragma unroll
          for (int e = 0; e < 4; ++e) y = __builtin_fmaf(u[j][e] - mean[j], u[j][e] - mean[j], y);
          const float w = __shfl_xor(y, 16);
          q[j] = (fq & 1) ? y : w;
          q[j] += __shfl_xor(q[j], 32);
        }
        {
          float t2[RN];
#pragma unroll
          for (int j = 0; j < RN; ++j) t2[j] = q[j] + q[j ^ 1];
#pragma unroll
          for (int j = 0; j < RN; ++j) q[j] = c64 ? t2[j] + t2[j ^ 2] : t2[j];
        }
        if (c64) {
          const int off = (ok && fq == 0) ? (m * (p.N >> 6) + (ncol >> 6)) * 8 : OOB;
          const u32x2 d = {__float_as_uint(mean[0]), __float_as_uint(q[0])};
          __builtin_amdgcn_raw_buffer_store_b64(d, cs_rs, off, 0, 0);
        } else {
          const int off = (ok && fq == 0) ? (m * (p.N >> 5) + (ncol >> 5)) * 8 : OOB;
          const u32x4 d = {__float_as_uint(mean[0]), __float_as_uint(q[0]), __float_as_uint(mean[2]), __float_as_uint(q[2])};
          __builtin_amdgcn_raw_buffer_store_b128(d, cs_rs, off, 0, 0);
        }
      } else if constexpr (OUTF) {
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const int off = ok ? out_elem(p, m, ncol + j * 16 + fq * 4, p.ldc, false) * 4 : OOB;
          const u32x4 d = {__float_as_uint(v[j][0]), __float_as_uint(v[j][1]), __float_as_uint(v[j][2]),
                           __float_as_uint(v[j][3])};
          __builtin_amdgcn_raw_buffer_store_b128(d, c_rs, off, 0, 0);
        }
        if constexpr (RN == 2) {   // 4 stores per i whatever RN (EpiCount)
          __builtin_amdgcn_raw_buffer_store_b32(0u, c_rs, OOB, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(0u, c_rs, OOB, 0, 0);
        }
      } else {
        // pairs (2p, 2p+1): after the swap lane fq holds 8 consecutive columns at
        // 32p + (fq & 1) * 16 + (fq >> 1) * 8
#pragma unroll
        for (int pp = 0; pp < RN / 2; ++pp) {
          uint32_t x0 = pack_bf16(v[2 * pp][0], v[2 * pp][1]), x1 = pack_bf16(v[2 * pp][2], v[2 * pp][3]);
          uint32_t y0 = pack_bf16(v[2 * pp + 1][0], v[2 * pp + 1][1]), y1 = pack_bf16(v[2 * pp + 1][2], v[2 * pp + 1][3]);
          const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
          const int n = ncol + 32 * pp + (fq & 1) * 16 + (fq >> 1) * 8;
          const int off = ok ? out_elem(p, m, n, p.ldc, CT) * 2 : OOB;
          const u32x4 d = {s0[0], s1[0], s0[1], s1[1]};
          __builtin_amdgcn_raw_buffer_store_b128(d, c_rs, off, 0, 0);
        }
        if constexpr (RN == 2) __builtin_amdgcn_raw_buffer_store_b32(0u, c_rs, OOB, 0, 0);
      }
    });
    };
    if (act == 1) epilogue(std::integral_constant<int, 1>{});
    else if (act == 3) epilogue(std::integral_constant<int, 3>{});
    else if (act == 2) epilogue(std::integral_constant<int, 2>{});
    else epilogue(std::integral_constant<int, 0>{});
}

// F8: MX fp8 operands (e4m3fn data + one E8M0 scale per 32 k) on
// v_mfma_scale_f32_16x16x128_f8f6f4: a K-step is 128 fp8 = the same 128-B LDS row as 64 bf16,
// so the tile geometry, swizzle and pipeline are the bf16 engine's; per stage each row also
// brings one scale dword (its four 32-k blocks) into LDS (waves 0-3: A rows, 4-7: W rows).
// The MFMA's k order inside a lane is (bytes 0-15: k = 16 g + j, bytes 16-31: k = 64 + 16 g + j)
// for lane group g = lane >> 4, and the scale a lane passes covers k in [32 g, 32 g + 32)
// (tools/probes/probe_mx.hip), so lane group g reads 16-B chunks g and 4 + g of the row and
// passes byte g of the row's scale dword.
template <int BM, bool CONV, bool RELU_A, int EPI, int BN = 256, bool F8 = false>
__global__ __launch_bounds__(512) void k_gemm_p(Args p) {
  constexpr int TM = BM / 2, RM = TM / 16, RN = BN / 64;
  constexpr int ROWB = 128, RPI = 8;
  constexpr int ESZ = F8 ? 1 : 2;          // operand bytes
  constexpr int KSTEP = ROWB / ESZ;        // k per LDS stage
  // A: BM / 8 slabs of 8 rows (one glds wave-instruction each), slab w + 8 j to wave w (BM = 160:
  // waves 0-3 load three, waves 4-7 two); W: BN / 64 slabs per wave
  constexpr int A_SLABS = BM / RPI;
  constexpr int A_LOADS = (A_SLABS + 7) / 8, W_LOADS = BN / 64;
  constexpr int A_BYTES = BM * ROWB, W_BYTES = BN * ROWB;
  constexpr int SC_BYTES = F8 ? (BM + BN) * 4 : 0;
  constexpr int STAGE = A_BYTES + W_BYTES + SC_BYTES;
  constexpr int BIAS_OFF = 2 * STAGE;
  constexpr int CSUM_OFF = BIAS_OFF + 2048;          // EPI_LNF: column sums [2][1 KB], row scales [2][BM * 8]
  constexpr int ROWS_OFF = CSUM_OFF + 2048;
  constexpr int SHIFT_OFF = BIAS_OFF + 2048;         // EPI_LNP(B): row shifts [2][1 KB] (BM <= 256 floats)
  constexpr int RSH_OFF = SHIFT_OFF + 2048;          // EPI_LNPB: the stream's row shifts (res_shift) [2][1 KB]
  constexpr int NRL = EpiCount<EPI>::loads * RN / 4, NS = EpiCount<EPI>::stores;
  constexpr int E_ALL = RM * (NRL + NS);
  static_assert(BM == 256 || BM == 320 || BM == 160, "BM");
  static_assert(BM % 64 == 0 || (!F8 && !CONV), "BM = 160: dense bf16 A");
  static_assert(EPI != EPI_LNF || ((BM == 256 || BM == 160) && !F8 && !CONV), "EPI_LNF: dense bf16 A, BM 256 or 160");
  static_assert((EPI != EPI_LNP && EPI != EPI_LNPB) || (BN == 256 && BM <= 256 && !F8 && !CONV),
                "EPI_LNP / EPI_LNPB: dense bf16 A, BN 256");
  static_assert(BN == 256 || BN == 128, "BN");
  static_assert(!F8 || BM == 256, "fp8 engine: BM 256 (scale loads: one wave per 64 rows)");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int frow = lane & 15, fq = lane >> 4;
  const int lrow = lane >> 3, pchunk = lane & 7;

  const int T = p.tiles_m * p.tiles_n;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, xl = blockIdx.x >> 3, q = G >> 3, rr = G & 7;
  int t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + xl;
  if (t >= T) return;

  // operands through buffer descriptors: rows past M and conv taps outside the image
  // read as zero (offset >= range), so no per-row clamping and one VGPR offset per operand
  const rsrc_t a_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.A), 0, p.a_bytes, 0x00020000);
  const rsrc_t w_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.W), 0, p.w_bytes, 0x00020000);
  const rsrc_t b_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias), 0, p.bias ? p.N * 4 : 0, 0x00020000);
  const rsrc_t as_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(p.As), 0, F8 ? p.as_bytes : 0, 0x00020000);
  const rsrc_t ws_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(p.Ws), 0, F8 ? p.ws_bytes : 0, 0x00020000);
  const int chunk16 = (pchunk ^ lrow) << 4;           // swizzled 16-B chunk (row & 7 == lrow)
  const int a_row0 = wid * RPI + lrow;                // + j * 64 (slab wid + 8 j)
  const int w_row0 = wid * W_LOADS * RPI + lrow;
  const int a_sstep = 64 * (int)p.lda * ESZ, w_sstep = RPI * (int)p.ldw * ESZ;
  // fp8 scale rows: waves 0..BM/64-1 load A rows 64 w + lane, waves 4..4+BN/64-1 W rows
  const bool sc_a = F8 && wid < BM / 64;
  const bool sc_w = F8 && wid >= 4 && wid < 4 + BN / 64;
  const int sc_row = (wid & 3) * 64 + lane;

  uint32_t a_off;                 // dense A: byte offset of this lane's slab-0 row
  uint32_t w_off;
  uint32_t s_off;                 // dense A / W scale: byte offset of this lane's scale row
  int cpix[CONV ? A_LOADS : 1], cyx[CONV ? A_LOADS : 1];
  int spix = 0, syx = 0;          // conv: pixel of this lane's scale row
  int nm0, nn0;   // coordinates of the tile the offsets point at
  auto conv_row = [&](int m, int& pix, int& yx) {
    const int hw = p.coh * p.cow;
    const int b = m / hw;
    const int rem = m - b * hw;
    const int oy = rem / p.cow;
    const int ox = rem - oy * p.cow;
    // rows past M: an out-of-image y so every tap reads zero
    pix = b * p.ch * p.cw;
    yx = m < p.M ? ((oy * p.cs - p.cp) << 16) | ((ox * p.cs - p.cp) & 0xffff) : (int)(0x4000u << 16);
  };
  auto setup = [&](int tile) {
    int tm, tn;
    grouped(p, tile, tm, tn);
#ifdef I2PC_STAMPS
    if (p.dbg_drop & 2) tm = tn = 0;   // diagnostic: every tile computes tile (0, 0) (all loads L2 hits)
#endif
    nm0 = tm * BM;
    nn0 = tn * BN;
    if constexpr (!CONV) {
      a_off = (uint32_t)(nm0 + a_row0) * (uint32_t)(p.lda * ESZ) + chunk16;
    } else {
#pragma unroll
      for (int j = 0; j < A_LOADS; ++j) conv_row(nm0 + a_row0 + j * 64, cpix[j], cyx[j]);
    }
    w_off = (uint32_t)(nn0 + w_row0) * (uint32_t)(p.ldw * ESZ) + chunk16;
    if constexpr (F8) {
      if (sc_a) {
        if constexpr (CONV) conv_row(nm0 + sc_row, spix, syx);
        else s_off = (uint32_t)(nm0 + sc_row) * (uint32_t)(p.ldas * 4);
      } else {
        s_off = (uint32_t)(nn0 + sc_row) * (uint32_t)(p.ldws * 4);
      }
    }
  };
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  // cache policy of the LDS-DMA loads of the per-call row statistics / row shifts (written by the
  // k_ln_rowstats launch or the producer GEMM right before this one): sc1 = agent scope, past any
  // non-coherent line another XCD's L2 may hold (the bias and column sums are weights)
  constexpr int kAgentScope = 16;
  // one K-stage (A BM x KSTEP, W BN x KSTEP [+ their scale dwords]) into LDS buffer `buf`;
  // with `bias_par` >= 0 wave 0 first stages the tile's BN bias values into bias slot bias_par
  const rsrc_t cs_rs_ln = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.csum), 0, EPI == EPI_LNF ? p.N * 4 : 0,
                                                            0x00020000);
  const rsrc_t lr_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.lnr), 0, EPI == EPI_LNF ? p.M * 8 : 0,
                                                         0x00020000);
  const rsrc_t sh_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.lnsh), 0,
                                                         (EPI == EPI_LNP || EPI == EPI_LNPB) && p.lnsh ? p.M * 4 : 0,
                                                         0x00020000);
  const rsrc_t rsh_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.rsh), 0,
                                                          EPI == EPI_LNPB && p.rsh ? p.M * 4 : 0, 0x00020000);
  auto stage = [&](int buf, int k0, int bias_par) {
    uint8_t* sA = smem + buf * STAGE;
    uint8_t* sW = sA + A_BYTES;
    if (bias_par >= 0 && wid == 0 && lane < BN / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rs, (lds_ptr_t)(smem + BIAS_OFF + bias_par * 1024), 16,
                                                (nn0 + lane * 4) * 4, 0, 0, 0);
    if constexpr (EPI == EPI_LNF) {
      // the tile's column sums (wave 1) and its BM rows' (rstd, -rstd * mean) (waves 2, 3; rows past
      // M read as zero), landing with the stage
      if (bias_par >= 0 && wid == 1 && lane < BN / 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(cs_rs_ln, (lds_ptr_t)(smem + CSUM_OFF + bias_par * 1024), 16,
                                                  (nn0 + lane * 4) * 4, 0, 0, 0);
      if (bias_par >= 0 && (wid == 2 || (wid == 3 && lane < (BM - 128) / 2)))
        __builtin_amdgcn_raw_ptr_buffer_load_lds(lr_rs, (lds_ptr_t)(smem + ROWS_OFF + bias_par * BM * 8 + (wid - 2) * 1024),
                                                  16, (nm0 + (wid - 2) * 128 + lane * 2) * 8, 0, 0, kAgentScope);
    }
    if constexpr (EPI == EPI_LNP || EPI == EPI_LNPB) {
      // the tile's BM row shifts (wave 1; rows past M and a NULL shift read as zero)
      if (bias_par >= 0 && wid == 1 && lane < BM / 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(sh_rs, (lds_ptr_t)(smem + SHIFT_OFF + bias_par * 1024), 16,
                                                  (nm0 + lane * 4) * 4, 0, 0, kAgentScope);
    }
    if constexpr (EPI == EPI_LNPB) {
      // ... and the shifts the stream rows are stored relative to (wave 2)
      if (bias_par >= 0 && wid == 2 && lane < BM / 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsh_rs, (lds_ptr_t)(smem + RSH_OFF + bias_par * 1024), 16,
                                                  (nm0 + lane * 4) * 4, 0, 0, kAgentScope);
    }
    int kk = 0, ky = 0, kx = 0, ci0 = 0;
    if constexpr (CONV) {
      kk = k0 / p.cc;
      ky = kk / p.ck;
      kx = kk - ky * p.ck;
      ci0 = k0 - kk * p.cc;
    }
#ifdef I2PC_STAMPS
    if (p.dbg_drop & 4) return;   // diagnostic: no operand loads (MFMA + LDS reads on stale LDS)
#endif
    if constexpr (!CONV) {
#pragma unroll
      for (int j = 0; j < A_LOADS; ++j)
        if (A_SLABS % 8 == 0 || wid + 8 * j < A_SLABS)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rs, (lds_ptr_t)(sA + (wid + 8 * j) * RPI * ROWB), 16,
                                                    a_off + j * a_sstep, k0 * ESZ, 0, 0);   // row part in voffset: range-checked
    } else {
#pragma unroll
      for (int j = 0; j < A_LOADS; ++j) {
        const int yi = (cyx[j] >> 16) + ky, xi = ((int)(short)(cyx[j] & 0xffff)) + kx;
        const bool ok = (unsigned)yi < (unsigned)p.ch && (unsigned)xi < (unsigned)p.cw;
        const int off = ok ? ((cpix[j] + yi * p.cw + xi) * p.cc + ci0) * ESZ + chunk16 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rs, (lds_ptr_t)(sA + (wid + 8 * j) * RPI * ROWB), 16, off, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < W_LOADS; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(w_rs, (lds_ptr_t)(sW + (wid * W_LOADS + j) * RPI * ROWB), 16, w_off,
                                                j * w_sstep + k0 * ESZ, 0, 0);
    if constexpr (F8) {
      uint8_t* sS = sW + W_BYTES;                    // [BM] A scale dwords | [BN] W scale dwords
      if (sc_a) {
        if constexpr (!CONV) {
          __builtin_amdgcn_raw_ptr_buffer_load_lds(as_rs, (lds_ptr_t)(sS + (wid & 3) * 256), 4, s_off, (k0 / 128) * 4, 0, 0);
        } else {
          const int yi = (syx >> 16) + ky, xi = ((int)(short)(syx & 0xffff)) + kx;
          const bool ok = (unsigned)yi < (unsigned)p.ch && (unsigned)xi < (unsigned)p.cw;
          const int off = ok ? ((spix + yi * p.cw + xi) * (p.cc / 128) + ci0 / 128) * 4 : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(as_rs, (lds_ptr_t)(sS + (wid & 3) * 256), 4, off, 0, 0, 0);
        }
      } else if (sc_w) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ws_rs, (lds_ptr_t)(sS + BM * 4 + (wid & 3) * 256), 4, s_off,
                                                  (k0 / 128) * 4, 0, 0);
      }
    }
  };

  const rsrc_t c_rs = p.dbg_drop ? __builtin_amdgcn_make_buffer_rsrc(p.C, 0, 0, 0x00020000) : make_rsrc(p.C);
  const rsrc_t r_rs = make_rsrc(p.res);
  // EPI_LNP(B): the bf16 copy and the chunk partials take the second-residual / fp8-scale slots
  constexpr bool LNPX = EPI == EPI_LNP || EPI == EPI_LNPB;
  const rsrc_t r2_rs = make_rsrc(LNPX ? static_cast<const void*>(p.cbf) : static_cast<const void*>(p.res2));
  const rsrc_t cs_rs = make_rsrc(LNPX ? static_cast<const void*>(p.lnp) : static_cast<const void*>(p.Cs));
  const int nk = p.K / KSTEP;

  setup(t);
  int m0 = nm0, n0 = nn0;
  stage(0, 0, 0);
  int g = 0, tpar = 0, tord = 0;
  bool after_epi = false;
  for (;;) {
    const int t_next = t + G;
    const bool has_next = t_next < T;
    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    PSTAMP(tord, 0);
#ifdef I2PC_STAMPS
    unsigned long long st_wait = 0, st_a = 0, st_b = 0;
#endif
    for (int kt = 0; kt < nk; ++kt) {
#ifdef I2PC_STAMPS
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_a)::"memory");
#endif
      // stage g landed: everything issued after it (the previous epilogue) may stay in flight
      if (kt == 0 && after_epi && !(EPI == EPI_LNF && BN == 128)) {
        // any count <= E_ALL is safe (in-order completion); use the largest available
        // (not on the LN-fold consumer's 256 x 128 tiles: its column sums read back wrong at one
        // within-wave column of some tiles, run to run, with the counted wait -- r06, tools/probes/det_lnf2.py)
        if constexpr (E_ALL >= 63) I2PC_WAIT_VM(63);
        else if constexpr (E_ALL >= 48) I2PC_WAIT_VM(48);
        else if constexpr (E_ALL >= 40) I2PC_WAIT_VM(40);
        else if constexpr (E_ALL >= 32) I2PC_WAIT_VM(32);
        else if constexpr (E_ALL >= 20) I2PC_WAIT_VM(20);
        else if constexpr (E_ALL >= 16) I2PC_WAIT_VM(16);
        else I2PC_WAIT_VM(0);
      } else {
        I2PC_WAIT_VM(0);
      }
      I2PC_LDS_BARRIER();
#ifdef I2PC_STAMPS
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_b)::"memory");
      st_wait += st_b - st_a;
#endif
      if (kt == 0) PSTAMP(tord, 1);
      // the next K-stage's LDS-DMA issue (8 buffer_load ... lds per wave, ~60-185 cycles of issue each):
      // with the stagger, waves 4-7 issue theirs half-way through the step, so each SIMD's MFMA pipe
      // runs one wave's MFMAs while its partner (wave w +- 4) issues loads, instead of both issuing
      // at the top of the step (buffer (g + 1) & 1 was last read in step g - 1: any point is legal)
      // (bf16 only: in the fp8 engine the mid-step issue pushed the register allocation into scratch,
      // whose VMEM operations would break the counted vmcnt waits)
      const bool late = !F8 && p.stagger && wid >= 4;
      auto issue_next = [&]() {
        if (kt + 1 < nk) {
          stage((g + 1) & 1, (kt + 1) * KSTEP, -1);
        } else if (has_next) {
          setup(t_next);
          stage((g + 1) & 1, 0, tpar ^ 1);
        }
      };
      if (!late) issue_next();
      const uint8_t* sA = smem + (g & 1) * STAGE;
      const uint8_t* sW = sA + A_BYTES;
      if constexpr (!F8) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (s == 1 && late) {
            __builtin_amdgcn_sched_barrier(0);
            issue_next();
            __builtin_amdgcn_sched_barrier(0);
          }
          bf16x8 wf[RN];
          const int lchunk = 4 * s + fq;
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            const int row = wn * (BN / 4) + j * 16 + frow;
            wf[j] = *reinterpret_cast<const bf16x8*>(sW + row * ROWB + ((lchunk ^ (row & 7)) << 4));
          }
#if I2PC_GEMM_APF > 0
          // A fragments read APF m-subtiles ahead of their MFMAs, the order pinned by scheduling groups
          // (left to itself the compiler reused one fragment register: read -> lgkmcnt(0) -> 4 MFMAs per
          // m-subtile, each LDS latency exposed to the matrix pipe)
          constexpr int APF = I2PC_GEMM_APF < RM ? I2PC_GEMM_APF : RM;
          bf16x8 afr[RM];
          auto a_read = [&](int i) {
            const int row = wm * TM + i * 16 + frow;
            afr[i] = *reinterpret_cast<const bf16x8*>(sA + row * ROWB + ((lchunk ^ (row & 7)) << 4));
          };
#pragma unroll
          for (int i = 0; i < APF; ++i) a_read(i);
          __builtin_amdgcn_sched_group_barrier(0x100, RN + APF, 0);
#pragma unroll
          for (int i = 0; i < RM; ++i) {
            if (i + APF < RM) {
              a_read(i + APF);
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            bf16x8 af = afr[i];
            if (RELU_A) af = relu8(af);
#pragma unroll
            for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af, acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, RN, 0);
          }
#else
#pragma unroll
          for (int i = 0; i < RM; ++i) {
            const int row = wm * TM + i * 16 + frow;
            bf16x8 af = *reinterpret_cast<const bf16x8*>(sA + row * ROWB + ((lchunk ^ (row & 7)) << 4));
            if (RELU_A) af = relu8(af);
#pragma unroll
            for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af, acc[i][j], 0, 0, 0);
          }
#endif
        }
      } else {
        const uint32_t* sS = reinterpret_cast<const uint32_t*>(sW + W_BYTES);
        i32x8 wf[RN];
        int wsc[RN];
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const int row = wn * (BN / 4) + j * 16 + frow;
          const uint8_t* r = sW + row * ROWB;
          const i32x4 lo = *reinterpret_cast<const i32x4*>(r + ((fq ^ (row & 7)) << 4));
          const i32x4 hi = *reinterpret_cast<const i32x4*>(r + (((4 + fq) ^ (row & 7)) << 4));
          wf[j] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          wsc[j] = (int)(sS[BM + row] >> (8 * fq));
        }
#pragma unroll
        for (int i = 0; i < RM; ++i) {
          const int row = wm * TM + i * 16 + frow;
          const uint8_t* r = sA + row * ROWB;
          const i32x4 lo = *reinterpret_cast<const i32x4*>(r + ((fq ^ (row & 7)) << 4));
          const i32x4 hi = *reinterpret_cast<const i32x4*>(r + (((4 + fq) ^ (row & 7)) << 4));
          i32x8 af = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          if (RELU_A) {          // ReLU on e4m3 bytes: negative values (sign bit) -> +0
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t u = (uint32_t)af[e];
              af[e] = (int)(u & ~(((u >> 7) & 0x01010101u) * 0xffu));
            }
          }
          const int asc = (int)(sS[row] >> (8 * fq));
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[j], af, acc[i][j], 0, 0, 0, wsc[j], 0, asc);
        }
      }
      ++g;
    }

    PSTAMP(tord, 2);
#ifdef I2PC_STAMPS
    if (threadIdx.x == 0 && tord < 8) g_stamps[(blockIdx.x * 8 + tord) * 8 + 4] = st_wait;
#endif
    // ---- epilogue of tile (m0, n0): register-direct, counted
    epilogue_p<RM, RN, EPI, F8>(p, acc, m0 + wm * TM, n0 + wn * (BN / 4),
                                reinterpret_cast<const float*>(smem + BIAS_OFF + tpar * 1024) + wn * (BN / 4), c_rs, r_rs,
                                r2_rs, cs_rs, reinterpret_cast<const float*>(smem + CSUM_OFF + tpar * 1024) + wn * (BN / 4),
                                LNPX ? reinterpret_cast<const float*>(smem + SHIFT_OFF + tpar * 1024) + wm * TM
                                     : reinterpret_cast<const float*>(smem + ROWS_OFF + tpar * BM * 8) + wm * TM * 2,
                                reinterpret_cast<const float*>(smem + RSH_OFF + tpar * 1024) + wm * TM);
    PSTAMP(tord, 3);
    ++tord;
    if (!has_next) break;
    t = t_next;
    m0 = nm0;
    n0 = nn0;
    tpar ^= 1;
    after_epi = true;
  }
}
// Counted vmcnt wait (k_gemm_8p): sched barrier, then wait until at most N vector-memory operations remain.
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N < 63 ? N : 63) : "memory");
}

// ---------------------------------------------------------------------------
// Ping-pong persistent 256 x 256 x 64 bf16 engine (k_gemm_8p), dense A.
//
// LDS: two K-tile buffers of four 16-KB quarters (A-q0, A-q1, B-q0, B-q1 as in k_gemm_q:
// the 64-row halves mp of both 128-row wave halves, the 32-column halves np of every wave's
// 64 columns) + per-(parity, wave-row) 1-KB bias copies.  A K-tile is four phases, one
// (mp, np) quadrant of every wave's 128 x 64 output each, in the order (0,0) (0,1) (1,1) (1,0):
// phase 1 reads A-q0 + B-q0, phase 2 B-q1, phase 3 A-q1, phase 4 nothing new (A-q1 and the
// B-q0 fragments from phase 1 stay in registers).  Each phase is two barrier intervals,
//   R: ds_read the phase's fragments | issue one quarter (2 LDS-DMA per wave) | vmcnt(8) | s_barrier
//   M: lgkmcnt(0) | 16 MFMAs at priority 1 | s_barrier
// and wave-row 1 (waves 4-7) runs one interval behind wave-row 0 (one extra barrier at the
// start; wave-row 0 takes one at the end), so on every SIMD one wave's MFMAs overlap the
// other's LDS reads and DMA issue.
// The quarter stream: element e = quarter [A-q0, B-q0, B-q1, A-q1][e & 3] of K-tile e >> 2
// (counted over the CU's whole tile sequence, buffer = K-tile & 1); global phase k issues
// element k + 5 (the prologue issues 0..5).  A phase's vmcnt(8) leaves the four youngest
// elements in flight, i.e. it retires element k + 1, which is first read in phase k + 2 at
// the earliest (RAW: DMA data is ordered for a ds_read by the issuer's vmcnt and a barrier
// both wave-rows pass afterwards; with the one-interval stagger a wait in phase k's R
// interval precedes every read in phases > k).  Refills land at least two phases after the
// last read of the quarter they overwrite (WAR: the lagging wave-row retires a phase-p read
// before the barrier that ends interval 2p + 1; the earliest refill is issued in interval
// 2p + 3).  An epilogue (register-direct, E_ALL memory operations incl. the next tile's
// bias load) sits between two phases; the four phases after it wait vmcnt(8 + E_ALL).
// Phases whose element does not exist (the last tile's tail) wait vmcnt(0).
// The accumulation order of every acc[i][j] is k_gemm_p's (k ascending, s = 0 then 1 per
// K-tile), so both engines are bit-identical.
// per-tile operand descriptors: A from the tile's first row (rows past M read as zero), W panel
struct TileRs { rsrc_t a, w; int m0, n0; };
__device__ __forceinline__ TileRs tile_rs_8p(const Args& p, int tile) {
  int tm, tn;
  grouped(p, tile, tm, tn);
  TileRs r;
  r.m0 = tm * 256;
  r.n0 = tn * 256;
  r.a = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(p.A) + (int64_t)r.m0 * p.lda * 2), 0,
      (uint32_t)((int64_t)(p.M - r.m0) * p.lda * 2), 0x00020000);
  r.w = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(p.W) + (int64_t)r.n0 * p.ldw * 2), 0,
      (uint32_t)(256 * p.ldw * 2), 0x00020000);
  return r;
}

template <int EPI>
__global__ __launch_bounds__(512) void k_gemm_8p(Args p) {
  constexpr int RM = 8, RN = 4, ROWB = 128, QB = 128 * ROWB;
  constexpr int NRL = EpiCount<EPI>::loads * RN / 4, NS = EpiCount<EPI>::stores;
  constexpr int E_ALL = RM * (NRL + NS) + 1;
  constexpr int W_POST = 8 + E_ALL > 63 ? 63 : 8 + E_ALL;
  constexpr int BIAS_OFF = 8 * QB;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int frow = lane & 15, fq = lane >> 4;
  const int lrow = lane >> 3, pchunk = lane & 7;

  const int T = p.tiles_m * p.tiles_n;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, xl = blockIdx.x >> 3, xq = G >> 3, xr = G & 7;
  int t = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + xl;
  if (t >= T) return;

  // lane parts of this wave's quarter rows (r = wid * 16 + j * 8 + lrow), XOR swizzle on the source
  const int chunk16 = (pchunk ^ lrow) << 4;
  uint32_t a_lane[2][2], w_lane[2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = wid * 16 + j * 8 + lrow;
      a_lane[q][j] = (uint32_t)((r >> 6) * 128 + q * 64 + (r & 63)) * (uint32_t)(p.lda * 2) + chunk16;
      w_lane[q][j] = (uint32_t)((r >> 5) * 64 + q * 32 + (r & 31)) * (uint32_t)(p.ldw * 2) + chunk16;
    }
  const rsrc_t b_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias), 0, p.bias ? p.N * 4 : 0, 0x00020000);
  auto tile_rs = [&](int tile) { return tile_rs_8p(p, tile); };
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  // quarter (0 A-q0, 1 A-q1, 2 B-q0, 3 B-q1) of the K-tile at k0 into buffer buf
  auto issue = [&](int buf, int quarter, const TileRs& tr, int k0) {
    uint8_t* dst = smem + (buf * 4 + quarter) * QB + wid * 16 * ROWB;
    if (quarter < 2) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(tr.a, (lds_ptr_t)(dst + j * 8 * ROWB), 16, a_lane[quarter][j], k0 * 2, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(tr.w, (lds_ptr_t)(dst + j * 8 * ROWB), 16, w_lane[quarter - 2][j], k0 * 2, 0, 0);
    }
  };
  // the tile's 256 bias values, one copy per wave-row: wave (wm, wn) loads columns wn * 64 + lane
  auto load_bias = [&](int par, int n0) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rs, (lds_ptr_t)(smem + BIAS_OFF + (par * 2 + wm) * 1024 + wn * 256), 4,
                                              (n0 + wn * 64 + lane) * 4, 0, 0, 0);
  };
  auto frag = [&](int buf, int quarter, int row, int s) {
    const uint8_t* base = smem + (buf * 4 + quarter) * QB + row * ROWB;
    return *reinterpret_cast<const bf16x8*>(base + (((4 * s + fq) ^ (row & 7)) << 4));
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  const rsrc_t c_rs = p.dbg_drop ? __builtin_amdgcn_make_buffer_rsrc(p.C, 0, 0, 0x00020000) : make_rsrc(p.C);
  const rsrc_t r_rs = make_rsrc(p.res);
  const rsrc_t r2_rs = make_rsrc(p.res2);
  const int nk = p.K / BK;   // >= 2 (plan)

  TileRs cur = tile_rs(t);
  // prologue: bias, elements 0..5 (K-tile 0 whole, K-tile 1's A-q0 and B-q0)
  load_bias(0, cur.n0);
  issue(0, 0, cur, 0); issue(0, 2, cur, 0); issue(0, 3, cur, 0); issue(0, 1, cur, 0);
  issue(1, 0, cur, BK); issue(1, 2, cur, BK);
  I2PC_WAIT_VM(8);
  barrier();
  if (wm == 1) barrier();

  int g = 0, tpar = 0, post = 0;
  for (;;) {
    const int t_next = t + G;
    const bool has_next = t_next < T;
    const TileRs nxt = tile_rs(has_next ? t_next : t);
    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < nk; ++kt) {
      const int buf = g & 1;
      // K-tiles kt + 1 (phases 1, 2) and kt + 2 (phases 3, 4): this tile's, the next tile's, or none
      const bool e1_here = kt + 1 < nk, e2_here = kt + 2 < nk;
      const bool e1 = e1_here || has_next, e2 = e2_here || has_next;
      const TileRs& tr1 = e1_here ? cur : nxt;
      const TileRs& tr2 = e2_here ? cur : nxt;
      const int k1 = (e1_here ? kt + 1 : kt + 1 - nk) * BK;
      const int k2 = (e2_here ? kt + 2 : kt + 2 - nk) * BK;
      bf16x8 af[4][2], b0[2][2], b1[2][2];
      // a phase's R-interval tail: the wait for element k + 1, then the barrier
      auto r_wait = [&](bool issued) {
        if (!issued) I2PC_WAIT_VM(0);
        else if (post > 0) wait_vm<W_POST>();
        else I2PC_WAIT_VM(8);
        if (post > 0) --post;
        barrier();
      };
      auto mfma_quad = [&](auto mpc, auto npc, bf16x8 (&bq)[2][2]) {
        constexpr int MP = decltype(mpc)::value, NP = decltype(npc)::value;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[MP * 4 + i][NP * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][s], af[i][s], acc[MP * 4 + i][NP * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        barrier();
      };
      // ---- phase 1: (0, 0)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) af[i][s] = frag(buf, 0, wm * 64 + i * 16 + frow, s);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) b0[j][s] = frag(buf, 2, wn * 32 + j * 16 + frow, s);
      if (e1) issue(buf ^ 1, 3, tr1, k1);
      r_wait(e1);
      mfma_quad(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, b0);
      // ---- phase 2: (0, 1)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) b1[j][s] = frag(buf, 3, wn * 32 + j * 16 + frow, s);
      if (e1) issue(buf ^ 1, 1, tr1, k1);
      r_wait(e1);
      mfma_quad(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}, b1);
      // ---- phase 3: (1, 1)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) af[i][s] = frag(buf, 1, wm * 64 + i * 16 + frow, s);
      if (e2) issue(buf, 0, tr2, k2);
      r_wait(e2);
      mfma_quad(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}, b1);
      // ---- phase 4: (1, 0)
      if (e2) issue(buf, 2, tr2, k2);
      r_wait(e2);
      mfma_quad(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{}, b0);
      ++g;
    }
    // ---- epilogue of tile (cur.m0, cur.n0): register-direct, counted
    epilogue_p<RM, RN, EPI, false>(p, acc, cur.m0 + wm * 128, cur.n0 + wn * 64,
                                   reinterpret_cast<const float*>(smem + BIAS_OFF + (tpar * 2 + wm) * 1024) + wn * 64, c_rs,
                                   r_rs, r2_rs, c_rs);
    if (!has_next) break;
    load_bias(tpar ^ 1, nxt.n0);
    t = t_next;
    cur = nxt;
    tpar ^= 1;
    post = 4;
  }
  if (wm == 0) barrier();   // wave-row 0 is one barrier short of wave-row 1
}

#undef I2PC_WAIT_VM
#undef I2PC_LDS_BARRIER

}  // namespace pers

static int group_m_for(int tiles_m) {
  static const int env = [] { const char* e = getenv("I2PC_GEMM_GM"); return e ? atoi(e) : 0; }();
  const int g = env > 0 ? env : 8;
  return std::max(1, std::min(g, tiles_m));
}

static int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <int BM, bool CONV, bool RELU_A, int EPI, int BN = 256, bool F8 = false>
static void launch_p(const Args& p, hipStream_t s) {
  constexpr int ESZ = F8 ? 1 : 2;
  Args q = p;
  if (!CONV) {                        // dense rows: fold the row offset into the base
    q.A = reinterpret_cast<const bf16_t*>(reinterpret_cast<const uint8_t*>(p.A) + (int64_t)p.a_o * p.lda * ESZ);
    if (F8) q.As = p.As + (int64_t)p.a_o * p.ldas;
    q.a_o = 0;
    q.a_bytes = (uint32_t)((int64_t)p.M * p.lda * ESZ);
    q.as_bytes = (uint32_t)((int64_t)p.M * p.ldas * 4);
  } else {
    q.a_bytes = (uint32_t)((int64_t)p.cb * p.ch * p.cw * p.cc * ESZ);
    q.as_bytes = (uint32_t)((int64_t)p.cb * p.ch * p.cw * (p.cc / 128) * 4);
  }
  q.w_bytes = (uint32_t)((int64_t)p.N * p.ldw * ESZ);
  q.ws_bytes = (uint32_t)((int64_t)p.N * p.ldws * 4);
  q.tiles_m = (p.M + BM - 1) / BM;
  q.tiles_n = p.N / BN;
  q.group_m = group_m_for(q.tiles_m);
  const int smem = 2 * ((BM + BN) * 128 + (F8 ? (BM + BN) * 4 : 0)) + 2048 + (EPI == pers::EPI_LNF ? 2048 + 2 * BM * 8 : 0) +
                   (EPI == pers::EPI_LNP ? 2048 : 0) + (EPI == pers::EPI_LNPB ? 4096 : 0);
  auto kern = pers::k_gemm_p<BM, CONV, RELU_A, EPI, BN, F8>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  static const int drop = [] { const char* e = getenv("I2PC_GEMM_DROP_STORES"); return e ? atoi(e) : 0; }();
  q.dbg_drop = drop;
  // (the LN-fold consumer on 256 x 128 tiles -- DA-v2's QKV, N = 1152 -- returned run-to-run different
  // values with the stagger at one within-wave column (12: j 0, fq 3, e 0) of some tiles: r06,
  // tools/probes/det_lnf.py; the stagger off there made every call identical; root cause not found)
  q.stagger = g_stagger && !(EPI == pers::EPI_LNF && BN == 128);
  const int tiles = q.tiles_m * q.tiles_n;
  // (the 256 x 128 LN-fold instance: one tile per workgroup, see run_persistent)
  const int grid = EPI == pers::EPI_LNF && BN == 128 ? tiles : std::min(tiles, num_cus());
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), smem, s, q);
}

template <int EPI>
static void launch_8p(const Args& p, hipStream_t s) {
  Args q = p;
  q.A = p.A + (int64_t)p.a_o * p.lda;
  q.a_o = 0;
  q.tiles_m = (p.M + 255) / 256;
  q.tiles_n = p.N / 256;
  q.group_m = group_m_for(q.tiles_m);
  const int smem = 8 * 128 * 128 + 4 * 1024;
  auto kern = pers::k_gemm_8p<EPI>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int grid = std::min(q.tiles_m * q.tiles_n, num_cus());
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), smem, s, q);
}

// Which kernel a call runs: the persistent 256-column engine when the epilogue is one it
// implements and every byte offset fits its 31-bit buffer range; else the tile kernel.
struct Plan {
  int kind;      // 0 tile kernel, 1 persistent engine, 2 ping-pong persistent engine, 3 halo 3x3 conv
  int bm, bn, epi;
};

// 0 auto, 1 tile kernel only, 2 persistent engine wherever its epilogue applies;
// initial value from I2PC_GEMM_P (0 -> 1, 2 -> 2)
// 3 = automatic with the ping-pong engine where the persistent engine would run, 4 = ping-pong
// engine wherever it applies (else the persistent engine wherever its epilogue applies)
static thread_local int g_engine = [] {
  const char* e = getenv("I2PC_GEMM_P");
  if (!e) return 0;
  const int v = atoi(e);
  return v == 0 ? 1 : (v >= 2 && v <= 4) ? v : 0;
}();

static thread_local int g_tail = [] { const char* e = getenv("I2PC_GEMM_TAIL"); return e ? atoi(e) : 1; }();
// the persistent engine for N % 256 != 0, N % 128 == 0 (256 x 128 tiles; I2PC_GEMM_BN128 / "gemm_bn128")
static thread_local int g_bn128 = [] { const char* e = getenv("I2PC_GEMM_BN128"); return e ? atoi(e) : 1; }();

// split-K for calls the tile kernel would run with few tiles and a long K (I2PC_GEMM_SPLITK /
// "gemm_splitk"; needs the caller's workspace, i2pc_gemm_ws)
static thread_local int g_splitk = [] { const char* e = getenv("I2PC_GEMM_SPLITK"); return e ? atoi(e) : 1; }();
// split-K tile: 0 = 256 x 256 x 64 (one block per CU), 1 = 128 x 128 x 32 (32 KB of LDS: ~4 blocks
// per CU cover each other's load latency)
// 384 x 192 tiles for N % 192 == 0 calls that fit one round (I2PC_GEMM_TILE192 / "gemm_tile192")
static thread_local int g_tile192 = [] { const char* e = getenv("I2PC_GEMM_TILE192"); return e ? atoi(e) : 1; }();
static thread_local int g_split_tile = [] { const char* e = getenv("I2PC_GEMM_SPLIT_TILE"); return e ? atoi(e) : 0; }();
// LayerNorm-fold producers (attention-out / FC2 with an fp32 residual) on the persistent engine's EPI_LNP
// with 160 x 256 tiles where they fit (I2PC_GEMM_LNP_P / "gemm_lnp_p"; 0 = the tile kernel's epilogue)
// (measured r04, tools/epi_cost.py: O 70.6 vs 66.6 us, FC2 195.9 vs 173.3 us against the tile kernel's one round of
// 320 x 256 -- a 160-row K-step costs 0.79 of a 256-row one for 0.625 of its MFMAs, and the register-direct
// producer epilogue's shuffle tree is slower than the tile kernel's LDS-staged one; off by default)
static thread_local int g_lnp_p = [] { const char* e = getenv("I2PC_GEMM_LNP_P"); return e ? atoi(e) : 0; }();
// LayerNorm-fold producers on the shifted bf16 residual stream (attention-out / FC2 with a bf16 res and
// output, i2pc.h res_shift) on the persistent engine's EPI_LNPB: full rounds of 256 x 256 tiles plus
// the remaining rows as one round of 160 x 256 tiles (tail_split), so one tile's producer epilogue
// overlaps the next tile's K-loop instead of a single round's epilogues all running exposed together
// (I2PC_GEMM_LNP_STREAM / "gemm_lnp_stream": 0 = the tile kernel, 1 = where K <= 2048 (DPT-Large's
// attention-out; FC2's K = 4096 keeps the tile kernel's one round of 320 x 256), 2 = every such call)
// 3x3 stride-1 convs of 64-channel maps on k_conv3_halo (I2PC_CONV_HALO / "conv_halo"; 0 = the implicit GEMM)
// variants 1-4 (launch in run_plan); measured r06 on DA-v2's shapes (tools/bench_conv_halo.py, batch 32):
// 148^2 + res 106 / 87 / 85 / 104 us, 296^2 295 / 274 / 282 / 302 us against the implicit GEMM's 123 / 422 us
static thread_local int g_halo = [] { const char* e = getenv("I2PC_CONV_HALO"); return e ? atoi(e) : 3; }();
// Measured r06 in one process (tools/ab_pipeline.py, C2): tile kernel 20.68 ms per step, attention-out on
// EPI_LNPB 20.81, attention-out and FC2 21.22 -- the producer epilogue's register-direct shuffle tree and
// the 1 + 0.6-round schedule do not beat the tile kernel's single round, so the default is 0 (bit-identical).
// GELU in the tanh form (activation 3) for the calls that ask for GELU (I2PC_GELU_TANH / "gelu_tanh").
// Measured r06 in one process (tools/ab_pipeline.py): C2 20.91 -> 20.46 ms per step (+2.2 %), DA-v2
// 7.97 -> 7.78 ms (+2.5 %); the networks stay inside their transformers-fp32 bounds.
static thread_local int g_gelu_tanh = [] { const char* e = getenv("I2PC_GELU_TANH"); return e ? atoi(e) : 1; }();
static thread_local int g_lnp_stream = [] { const char* e = getenv("I2PC_GEMM_LNP_STREAM"); return e ? atoi(e) : 0; }();

static int64_t max_row(const Args& p) {
  const int64_t m = p.M - 1;
  return p.o_g > 0 ? (m / p.o_g) * p.o_gs + (p.o_g - 1) + p.o_o : m + p.o_o;
}

static Plan plan_for(const Args& p, bool conv, bool relu) {
  static const int force = [] { const char* e = getenv("I2PC_GEMM_TILE"); return e ? atoi(e) : 0; }();
  const int pforce = g_engine;
  Plan pl{0, 0, 0, -1};
  // persistent engine
  int epi = -1;
  // N a multiple of 128 only (e.g. the DPT head's first conv, 256 -> 128): 256 x 128 tiles
  const int pbn = p.N % 256 == 0 ? 256 : (p.N % 128 == 0 && g_bn128) ? 128 : 0;
  if (conv && g_halo && force == 0 && pforce != 1 && p.cc == 64 && p.ck == 3 && p.cs == 1 && p.cp == 1 &&
      p.coh == p.ch && p.cow == p.cw && p.N % 64 == 0 && !p.rbias && !p.tbl && !p.lnp && !p.lnr && p.ct_s == 0 &&
      p.o_g == 0 && p.o_o == 0 && (int64_t)p.cb * p.ch * p.cw * 128 < pers::OOB && (int64_t)p.N * p.ldw * 2 < pers::OOB &&
      p.ldw >= 9 * 64)
    return Plan{3, 256, 64, g_halo};
  if (p.lnr) {
    // LayerNorm-fold consumer: the persistent engine's EPI_LNF only (dense A, bf16 out, no extras)
    const bool ok = pbn && !conv && !relu && !p.rbias && !p.tbl && !p.res && !p.res2 && !p.c_f32 && p.ct_s == 0 &&
                    p.a_g == 0 && (int64_t)(p.M + 320) * p.lda * 2 < pers::OOB && (int64_t)p.N * p.ldw * 2 < pers::OOB &&
                    (max_row(p) * p.ldc + p.N) * 2 < pers::OOB;
    return ok ? Plan{1, 256, pbn, pers::EPI_LNF} : Plan{-2, 0, 0, 0};
  }
  if (p.lnp && !p.c_f32 && g_lnp_stream && force == 0 && pforce != 1) {
    const bool ok = p.N % 256 == 0 && !conv && !relu && !p.rbias && !p.tbl && p.res && !p.res_f32 && !p.res2 &&
                    p.ct_s == 0 && p.a_g == 0 && p.o_g == 0 && p.o_o == 0 && (g_lnp_stream >= 2 || p.K <= 2048) &&
                    (int64_t)(p.M + 320) * p.lda * 2 < pers::OOB && (int64_t)p.N * p.ldw * 2 < pers::OOB &&
                    ((int64_t)p.M * p.ldc + p.N) * 2 < pers::OOB && ((int64_t)p.M * p.ldr + p.N) * 2 < pers::OOB &&
                    ((int64_t)p.M * p.ldcb + p.N) * 2 < pers::OOB && (int64_t)p.M * (p.N / p.lnc) * 8 < pers::OOB;
    if (ok) return Plan{1, 256, 256, pers::EPI_LNPB};
  }
  if (p.lnp && g_lnp_p && force == 0 && pforce != 1) {
    // LayerNorm-fold producer on the persistent engine (EPI_LNP): a wave's 64 columns are one chunk
    // (or two of 32), fp32 output with the fp32 residual, linear rows.  160-row tiles where they
    // take fewer row-rounds than 256 (DPT-Large O / FC2, M 18464, N 1024: 464 tiles = 2 per CU of
    // 160 rows, the tile kernel's one round of 320 rows, but with the first tile's epilogue and the
    // second's first stage overlapped)
    const bool ok = p.N % 256 == 0 && !conv && !relu && !p.rbias && !p.tbl && p.res && p.res_f32 && p.c_f32 && !p.res2 &&
                    p.ct_s == 0 && p.a_g == 0 && p.o_g == 0 && p.o_o == 0 &&
                    (int64_t)(p.M + 320) * p.lda * 2 < pers::OOB && (int64_t)p.N * p.ldw * 2 < pers::OOB &&
                    (max_row(p) * p.ldc + p.N) * 4 < pers::OOB && (max_row(p) * p.ldr + p.N) * 4 < pers::OOB &&
                    ((int64_t)p.M * p.ldcb + p.N) * 2 < pers::OOB && (int64_t)p.M * (p.N / p.lnc) * 8 < pers::OOB;
    if (ok) {
      const int64_t ncu = num_cus();
      int best = 160;
      int64_t best_cost = -1;
      for (int bm : {160, 256}) {
        const int64_t tiles = (int64_t)((p.M + bm - 1) / bm) * (p.N / 256);
        const int64_t cost = (tiles + ncu - 1) / ncu * bm;
        if (best_cost < 0 || cost < best_cost) { best_cost = cost; best = bm; }
      }
      return Plan{1, best, 256, pers::EPI_LNP};
    }
  }
  if (pbn && !p.rbias && !p.tbl && !p.lnp && force == 0 && pforce != 1) {
    const bool ct = p.ct_s > 0;
    if (ct) epi = (!p.res && !p.res2 && !p.c_f32 && p.ct_c % 8 == 0) ? pers::EPI_CT : -1;
    else if (!p.res && !p.res2 && !p.c_f32) epi = pers::EPI_PLAIN;
    else if (p.res && p.res_f32 && p.c_f32 && !p.res2) epi = pers::EPI_RESF32;
    else if (p.res && !p.res_f32 && !p.c_f32 && !p.res2) epi = pers::EPI_RESBF16;
    else if (p.res && !p.res_f32 && !p.c_f32 && p.res2) epi = pers::EPI_RES2;
    // instantiated combinations
    if (!conv && relu) epi = -1;
    if (!conv && (epi == pers::EPI_RESBF16 || epi == pers::EPI_RES2)) epi = -1;
    if (conv && (epi == pers::EPI_RESF32 || epi == pers::EPI_CT)) epi = -1;
    if (conv && relu && epi != pers::EPI_PLAIN) epi = -1;
    if (!conv && p.a_g != 0) epi = -1;
    if (pbn == 128 && (epi != pers::EPI_PLAIN || relu)) epi = -1;   // instantiated BN = 128 variants
    if (epi >= 0) {
      const int64_t esz = p.c_f32 ? 4 : 2;
      const int64_t abytes = conv ? (int64_t)p.cb * p.ch * p.cw * p.cc * 2 : (int64_t)(p.M + 320) * p.lda * 2;
      if (abytes >= pers::OOB || (int64_t)p.N * p.ldw * 2 >= pers::OOB) epi = -1;
      const int64_t cbytes = ct ? (int64_t)p.M * p.N * 2 : (max_row(p) * p.ldc + p.N) * esz;
      int64_t rbytes = 0;
      if (p.res) rbytes = std::max(rbytes, (max_row(p) * p.ldr + p.N) * (p.res_f32 ? 4 : 2));
      if (p.res2) rbytes = std::max(rbytes, (max_row(p) * p.ldr2 + p.N) * 2);
      if (cbytes >= pers::OOB || rbytes >= pers::OOB) epi = -1;
    }
  }
  if (epi >= 0) {
    static const int bm_force = [] { const char* e = getenv("I2PC_GEMM_PBM"); return e ? atoi(e) : 0; }();
    const int64_t ncu = num_cus();
    int best = 256;
    int64_t best_cost = -1;
    for (int bm : {256}) {   // 320 spills registers (scratch would break the counted waits)
      const int64_t tiles = (int64_t)((p.M + bm - 1) / bm) * (p.N / pbn);
      const int64_t cost = (tiles + ncu - 1) / ncu * bm;
      if (best_cost < 0 || cost < best_cost) { best_cost = cost; best = bm; }
    }
    if (bm_force == 256) best = bm_force;
    // The persistent engine pays where a CU runs several tiles (it hides each tile's first
    // stage and epilogue behind the neighbouring tiles); at one or two tiles per CU the
    // tile kernel's 128 x 128 configurations quantise better (profiles/r01_gemm_engines.txt).
    const int64_t tiles = (int64_t)((p.M + best - 1) / best) * (p.N / pbn);
    if (pbn == 128) {
      if (pforce == 2 || pforce == 4 || tiles >= 3 * ncu) return Plan{1, best, 128, epi};
      epi = -1;
    }
  }
  if (epi >= 0) {
    const int64_t ncu = num_cus();
    const int best = 256;
    const int64_t tiles = (int64_t)((p.M + best - 1) / best) * (p.N / 256);
    // the ping-pong engine (k_gemm_8p): dense A, plain / fp32-residual epilogues, K >= 128
    const bool can8 = !conv && !relu && (epi == pers::EPI_PLAIN || epi == pers::EPI_RESF32) && p.K >= 128;
    if (pforce == 4 && can8) return Plan{2, 256, 256, epi};
    // one to three rounds: persistent when its last round is at least 80 % full (DPT-Hybrid's
    // bf16 FC2 / O, M = 36928, N = 768: 435 tiles = 0.85 of 2 rounds; 180 vs 203 us and 56 vs
    // 68 us against the 128 x 128 tile kernel, tools/gpu.sh ab-hyb); DPT-Large's N = 1024 calls
    // (292 tiles = 0.57 of 2 rounds) keep the one-round 320 x 256 tile kernel
    const int64_t rounds = (tiles + ncu - 1) / ncu;
    const bool full_rounds = tiles >= ncu && tiles * 10 >= rounds * ncu * 8;
    if (pforce == 2 || pforce == 4 || tiles >= 3 * ncu || full_rounds) {
      // the single-stage engine by default: in the DPT-Large step the ping-pong engine measured
      // 1.6 % slower end to end (tools/ab_pipeline.py), though equal or faster in isolation
      pl = Plan{pforce == 3 && can8 ? 2 : 1, best, 256, epi};
      return pl;
    }
  }
  const int64_t t256 = (int64_t)((p.M + 255) / 256) * (p.N / 256);
  const int64_t t128 = (int64_t)((p.M + 127) / 128) * (p.N / 128);
  if (force == 256 && p.N % 256 == 0) pl = Plan{0, 256, 256, 64};
  else if (force == 25632 && p.N % 256 == 0) pl = Plan{0, 256, 256, 32};
  else if (force == 320 && p.N % 256 == 0) pl = Plan{0, 320, 256, 64};
  else if (force == 192 && p.N % 256 == 0) pl = Plan{0, 192, 256, 64};
  else if (force == 128 && p.N % 128 == 0) pl = Plan{0, 128, 128, 64};
  else if (force == 12832 && p.N % 128 == 0) pl = Plan{0, 128, 128, 32};
  // one round of 320 x 256 tiles (e.g. M = 18464, N = 1024: 232 tiles) beats two rounds of
  // 256^2 or 2.3 rounds of 128^2 once K is long enough to amortise the bigger epilogue
  // (fc2: 156 vs 192 us, O: 53 vs 57 us, 48x48 neck conv: 102 vs 131 us; profiles/r01_gemm_engines.txt)
  else if (p.N % 256 == 0 && p.K >= 1024 && (int64_t)((p.M + 319) / 320) * (p.N / 256) <= num_cus() &&
           t256 > num_cus()) pl = Plan{0, 320, 256, 64};
  else if (p.N % 256 == 0 && t256 >= 512) pl = Plan{0, 256, 256, 64};
  // N = 384 (Depth-Anything-V2-Small's FC2 / attention-out, M = 43840): one round of 384 x 192
  // tiles (230) instead of four-plus rounds of 128 x 128
  else if (p.N % 256 != 0 && p.N % 192 == 0 && (int64_t)((p.M + 383) / 384) * (p.N / 192) <= num_cus() &&
           t128 > num_cus() && g_tile192) pl = Plan{0, 384, 192, 64};
  else if (p.N % 128 == 0 && t128 >= 512) pl = Plan{0, 128, 128, 64};
  else if (p.N % 64 == 0) pl = Plan{0, 128, 64, 64};
  else if (p.N % 32 == 0) pl = Plan{0, 128, 32, 64};
  else pl = Plan{-1, 0, 0, 0};
  if (p.lnp && pl.kind == 0) {
    // LayerNorm-fold producer: the tile epilogue's row layout must give whole 64-column chunks
    // to 8-lane groups (wave tile a multiple of 64 columns)
    const int wn = pl.bn == 256 ? 4 : pl.bn == 32 || pl.bn == 192 ? (pl.bn == 192 ? 2 : 1) : 2;
    if ((pl.bn / wn) % p.lnc != 0) pl = p.N % 128 == 0 ? Plan{0, 128, 128, 64} : Plan{-2, 0, 0, 0};
  }
  return pl;
}

// Split-K plan: when the tile kernel was chosen, K >= 4096 and even 256 x 256 (N % 256 == 0, else
// 128 x 128) tiles fill at most half the CUs, split K into `splits` slices of `kspan` K-steps (at least 4)
// so tiles x splits <= CUs: one round of shorter K-loops, then k_splitk_reduce sums the fp32
// slabs in slice order and applies the epilogue.  E.g. the 12 x 12 neck conv of DPT-Large
// (M 4608, N 256, K 9216): 18 tiles of 144 K-steps -> 14 slices of 11.
struct SplitPlan {
  int splits = 0, kspan = 0, bm = 0, bn = 0, kb = 64;
  int64_t bytes = 0;
};

static SplitPlan split_for(const Args& p, const Plan& pl) {
  SplitPlan sp;
  if (!g_splitk || pl.kind != 0 || (g_engine != 0 && g_engine != 3) || p.lnp) return sp;   // automatic modes only
  int bm, bn, kb = 64, slots = 1;
  if (g_split_tile == 1 && p.N % 128 == 0) { bm = bn = 128; kb = 32; slots = 4; }
  else if (p.N % 256 == 0) bm = bn = 256;
  else if (p.N % 128 == 0) bm = bn = 128;
  else return sp;
  const int64_t ncu = num_cus() * slots;
  const int64_t tiles = (int64_t)((p.M + bm - 1) / bm) * (p.N / bn);
  if (tiles * 2 > ncu || (int64_t)p.M * (p.N / 4) >= (int64_t)1 << 31) return sp;
  if (p.K < (g_splitk > 1 ? g_splitk * 64 : 4096)) return sp;
  const int nk = p.K / kb;
  // K >= 4096 only: at K = 1024-2304 the slab traffic and the second launch ate the gain
  // (DPT-Large neck, tools/gemm_census.py: K 2304 47 -> 59 us, the CLS readout 21 -> 25 us)
  const int s0 = (int)std::min<int64_t>(ncu / tiles, nk / (256 / kb));   // slices of >= 256 K
  if (s0 < 2) return sp;
  sp.kspan = (nk + s0 - 1) / s0;
  sp.splits = (nk + sp.kspan - 1) / sp.kspan;
  if (sp.splits < 2) return SplitPlan{};
  sp.bm = bm;
  sp.bn = bn;
  sp.kb = kb;
  sp.bytes = (int64_t)sp.splits * p.M * p.N * 4;
  return sp;
}

template <bool CONV, bool RELU_A>
static int run_split(const SplitPlan& sp, const Args& p, float* ws, hipStream_t s) {
  Args q = p;   // raw partial sums: no bias / act / residuals, dense fp32 rows of N
  q.bias = nullptr;
  q.rbias = nullptr;
  q.tbl = nullptr;
  q.act = 0;
  q.res = nullptr;
  q.res2 = nullptr;
  q.C = ws;
  q.c_f32 = 1;
  q.ldc = p.N;
  q.o_g = q.o_gs = q.o_o = 0;
  q.ct_s = 0;
  q.kspan = sp.kspan;
  if (sp.bm == 256) launch<256, 256, 2, 4, 64, CONV, RELU_A>(q, s, sp.splits);
  else if (sp.kb == 32) launch<128, 128, 2, 2, 32, CONV, RELU_A>(q, s, sp.splits);
  else launch<128, 128, 2, 2, 64, CONV, RELU_A>(q, s, sp.splits);
  const int64_t n = (int64_t)p.M * (p.N / 4);
  hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, ws, sp.splits);
  return check_launch("gemm (split-K)");
}

template <bool CONV, bool RELU_A>
static int run_persistent(const Plan& pl, const Args& p, hipStream_t s) {
  using namespace pers;
  if (pl.bn == 128) {   // plan: EPI_PLAIN (or EPI_LNF), no ReLU on A
    if constexpr (!RELU_A) {
      if constexpr (!CONV) {
        if (pl.epi == EPI_LNF) {
          // N = 256 k + 128 (DA-v2's QKV, 1152): the 256-multiple part on 256 x 256 tiles, the last 128
          // columns on 256 x 128 tiles, one tile per workgroup (launch_p).  r06: the 256 x 128 LN-fold
          // instance returned run-to-run different column-sum terms at one within-wave column of some
          // tiles once a workgroup walked more than one tile (tools/probes/det_lnf.py, det_lnf2.py);
          // with one tile per workgroup every call is identical.  Same per-output arithmetic either way.
          if (p.N > 128) {
            const int nb = p.N - 128;
            Args pa = p, pb = p;
            pa.N = nb;
            pb.N = 128;
            pb.W = p.W + (int64_t)nb * p.ldw;
            pb.C = static_cast<bf16_t*>(p.C) + nb;
            pb.bias = p.bias ? p.bias + nb : nullptr;
            pb.csum = p.csum + nb;
            launch_p<256, false, false, EPI_LNF>(pa, s);
            launch_p<256, false, false, EPI_LNF, 128>(pb, s);
            return check_launch("gemm (LN fold, N = 256 k + 128)");
          }
          launch_p<256, false, false, EPI_LNF, 128>(p, s);
          return check_launch("gemm");
        }
      }
      launch_p<256, CONV, false, EPI_PLAIN, 128>(p, s);
      return check_launch("gemm");
    }
    return set_error(I2PC_EUNSUPPORTED, "gemm: no persistent BN=128 variant with ReLU on A");
  }
  if constexpr (!CONV && !RELU_A) {
    if (pl.epi == EPI_LNPB) {
      launch_p<256, false, false, EPI_LNPB>(p, s);
      return check_launch("gemm (LN producer, bf16 stream)");
    }
    if (pl.epi == EPI_LNP) {
      if (pl.bm == 160) launch_p<160, false, false, EPI_LNP>(p, s);
      else launch_p<256, false, false, EPI_LNP>(p, s);
      return check_launch("gemm (LN producer)");
    }
    if (pl.epi == EPI_LNF) launch_p<256, false, false, EPI_LNF>(p, s);
    else if (pl.epi == EPI_PLAIN) launch_p<256, false, false, EPI_PLAIN>(p, s);
    else if (pl.epi == EPI_RESF32) launch_p<256, false, false, EPI_RESF32>(p, s);
    else launch_p<256, false, false, EPI_CT>(p, s);
  } else if constexpr (CONV && !RELU_A) {
    if (pl.epi == EPI_PLAIN) launch_p<256, true, false, EPI_PLAIN>(p, s);
    else if (pl.epi == EPI_RESBF16) launch_p<256, true, false, EPI_RESBF16>(p, s);
    else launch_p<256, true, false, EPI_RES2>(p, s);
  } else if constexpr (CONV && RELU_A) {
    launch_p<256, true, true, EPI_PLAIN>(p, s);
  } else {
    return set_error(I2PC_EUNSUPPORTED, "gemm: no persistent variant");
  }
  return check_launch("gemm");
}

// Round quantisation of the persistent engines: T 256 x 256 tiles take ceil(T / CUs) rounds.
// When a whole number of rounds covers whole M-tile rows and the remaining rows fit one round
// of 256 x 128 tiles (half the work each), run those rows as a second, BN = 128 launch
// (e.g. M = 18464, N = 3072: 3 rounds + a half round instead of 4).  Plain dense epilogue
// with a linear output row map only; the two parts compute every output exactly as one launch
// would (same per-output accumulation order).  I2PC_GEMM_TAIL=0 disables it.
// (Measured and dropped: FC1's remainder, M = 18464, N = 4096, as one round of the tile kernel's
// 192 x 256 tiles instead of a fifth persistent round -- no gain end to end.)
// When 256 x 128 tiles do not fit one round, 160 x 256 tiles may: DPT-Large's FC1 (M 18464, N 4096,
// 4.56 rounds of 256^2) keeps 4 rounds and runs its last 2080 rows as 13 x 16 = 208 tiles of 160 rows
// (r04; a 160-row K-step costs ~0.79 of a 256-row one, tools/stamps_p.py) instead of a fifth round.
// Returns 0 (no split), 1 (BN = 128 persistent remainder) or 2 (BM = 160 remainder).
static thread_local int g_tail160 = [] { const char* e = getenv("I2PC_GEMM_TAIL160"); return e ? atoi(e) : 1; }();
static int tail_split(const Args& p, int& ma, bool bn128_ok = true) {
  if (!g_tail || p.o_g != 0 || p.a_g != 0 || p.ct_s > 0 || p.N % 256 != 0) return 0;
  const int64_t tn = p.N / 256, tm = (p.M + 255) / 256, T = tm * tn, G = num_cus();
  const int64_t rounds = T / G;
  if (T % G == 0 || rounds < 1) return 0;
  // whole M-tile rows in the full rounds (a few slots of the last one may idle: DA-v2's FC1,
  // N = 1536, 6 tiles per row, 1032 tiles: 170 rows in 4 rounds + 24 half tiles, not 5 rounds)
  const int64_t mt = rounds * G / tn;
  if (mt >= tm) return 0;
  ma = (int)(mt * 256);
  const int64_t half_tiles = (tm - mt) * 2 * tn;
  if (bn128_ok && half_tiles <= G) return 1;
  const int64_t t160 = (p.M - ma + 159) / 160 * tn;
  return g_tail160 && t160 <= G ? 2 : 0;
}

template <bool CONV, bool RELU_A>
static int run_plan(const Plan& pl, const Args& p, hipStream_t s) {
  if constexpr (!CONV && !RELU_A) {
    int ma = 0;
    const bool lnf = pl.epi == pers::EPI_LNF, lnpb = pl.epi == pers::EPI_LNPB;
    // (EPI_LNPB: a 64-column partial chunk is one wave's 64 columns, so its remainder takes 160-row tiles)
    const int ts = (pl.kind == 1 || pl.kind == 2) && (pl.epi == pers::EPI_PLAIN || lnf || lnpb) && pl.bn == 256
                       ? tail_split(p, ma, !lnpb) : 0;
    if (ts) {
      Args pa = p, pb = p;
      pa.M = ma;
      pb.M = p.M - ma;
      pb.a_o = p.a_o + ma;
      pb.o_o = p.o_o + ma;
      if (lnpb) {
        // every per-row operand of the producer follows the rows (its output row map stays linear)
        pb.o_o = p.o_o;
        pb.C = static_cast<bf16_t*>(p.C) + (int64_t)ma * p.ldc;
        pb.cbf = p.cbf + (int64_t)ma * p.ldcb;
        pb.res = static_cast<const bf16_t*>(p.res) + (int64_t)ma * p.ldr;
        pb.lnp = p.lnp + (int64_t)ma * (p.N / p.lnc) * 2;
        if (p.lnsh) pb.lnsh = p.lnsh + ma;
        if (p.rsh) pb.rsh = p.rsh + ma;
        launch_p<256, false, false, pers::EPI_LNPB>(pa, s);
        launch_p<160, false, false, pers::EPI_LNPB>(pb, s);
        return check_launch("gemm (LN producer, bf16 stream, tail split)");
      }
      if (lnf) {
        pb.lnr = p.lnr + (int64_t)ma * 2;      // row scales follow the rows
        launch_p<256, false, false, pers::EPI_LNF>(pa, s);
        if (ts == 2) launch_p<160, false, false, pers::EPI_LNF>(pb, s);
        else launch_p<256, false, false, pers::EPI_LNF, 128>(pb, s);
        return check_launch("gemm (tail split)");
      }
      if (pl.kind == 2) launch_8p<pers::EPI_PLAIN>(pa, s);
      else launch_p<256, false, false, pers::EPI_PLAIN>(pa, s);
      if (ts == 2) launch_p<160, false, false, pers::EPI_PLAIN>(pb, s);
      else launch_p<256, false, false, pers::EPI_PLAIN, 128>(pb, s);
      return check_launch("gemm (tail split)");
    }
  }
  if (pl.kind == 2) {
    if constexpr (!CONV && !RELU_A) {
      if (pl.epi == pers::EPI_PLAIN) launch_8p<pers::EPI_PLAIN>(p, s);
      else launch_8p<pers::EPI_RESF32>(p, s);
      return check_launch("gemm_8p");
    }
    return set_error(I2PC_EUNSUPPORTED, "gemm: no ping-pong variant");
  }
  if (pl.kind == 1) return run_persistent<CONV, RELU_A>(pl, p, s);
  if (pl.kind == 3) {
    if constexpr (CONV) {
      // variants (knob conv_halo): 1 = 16 x 16 pixels, 4 waves; 2 = 16 x 16, 8 waves; 3 = 8 x 16, 4 waves;
      // 4 = 8 x 32, 4 waves
      if (pl.epi == 2) launch_halo<16, 16, 64, 8, 1, RELU_A>(p, s);
      else if (pl.epi == 3) launch_halo<8, 16, 64, 4, 1, RELU_A>(p, s);
      else if (pl.epi == 4) launch_halo<8, 32, 64, 4, 1, RELU_A>(p, s);
      else launch_halo<16, 16, 64, 4, 1, RELU_A>(p, s);
      return check_launch("conv (halo)");
    }
    return set_error(I2PC_EUNSUPPORTED, "gemm: halo plan without a conv");
  }
  if (pl.kind == -2) return set_error(I2PC_EUNSUPPORTED, "gemm: LayerNorm fold not available for this call");
  if (pl.kind < 0) return set_error(I2PC_EUNSUPPORTED, "gemm: N=%d must be a multiple of 32", p.N);
  if (pl.bm == 256 && pl.epi == 64) launch<256, 256, 2, 4, 64, CONV, RELU_A>(p, s);
  else if (pl.bm == 256) launch<256, 256, 2, 4, 32, CONV, RELU_A>(p, s);
  else if (pl.bm == 320) launch<320, 256, 2, 4, 64, CONV, RELU_A>(p, s);
  else if (pl.bm == 192) launch<192, 256, 2, 4, 64, CONV, RELU_A>(p, s);
  else if (pl.bm == 384) launch<384, 192, 4, 2, 64, CONV, RELU_A>(p, s);
  else if (pl.bn == 128 && pl.epi == 64) launch<128, 128, 2, 2, 64, CONV, RELU_A>(p, s);
  else if (pl.bn == 128) launch<128, 128, 2, 2, 32, CONV, RELU_A>(p, s);
  else if (pl.bn == 64) launch<128, 64, 2, 2, 64, CONV, RELU_A>(p, s);
  else launch<128, 32, 4, 1, 64, CONV, RELU_A>(p, s);
  return check_launch("gemm");
}

static const char* plan_name(const Plan& pl, bool conv, bool relu, const SplitPlan& sp = SplitPlan{}) {
  static thread_local char buf[96];
  if (sp.splits > 1) {
    const int wm = 2, wn = sp.bn == 256 ? 4 : 2;
    snprintf(buf, sizeof buf, "k_gemm<%d, %d, %d, %d, %d, %s, %s> split-K %d", sp.bm, sp.bn, wm, wn, sp.kb,
             conv ? "true" : "false", relu ? "true" : "false", sp.splits);
    return buf;
  }
  const char* c = conv ? "true" : "false";
  const char* r = relu ? "true" : "false";
  if (pl.kind == 3) {
    static const int th[] = {16, 16, 16, 8, 8}, tw[] = {16, 16, 16, 16, 32}, wv[] = {4, 4, 8, 4, 4};
    const int v = pl.epi >= 1 && pl.epi <= 4 ? pl.epi : 1;
    snprintf(buf, sizeof buf, "k_conv3_halo<%d, %d, 64, %d, 1, %s>", th[v], tw[v], wv[v], r);
  } else if (pl.kind == 2) {
    snprintf(buf, sizeof buf, "k_gemm_8p<%s>", pl.epi == pers::EPI_PLAIN ? "plain" : "res_f32");
  } else if (pl.kind == 1) {
    static const char* epis[] = {"plain", "res_f32", "res_bf16", "res2", "convT", "q8", "ln_fold", "ln_prod", "ln_stream"};
    if (pl.bn == 128) snprintf(buf, sizeof buf, "k_gemm_p<%d, %s, %s, %s, 128>", pl.bm, c, r, epis[pl.epi]);
    else snprintf(buf, sizeof buf, "k_gemm_p<%d, %s, %s, %s>", pl.bm, c, r, epis[pl.epi]);
  } else if (pl.kind == 0) {
    const int wm = pl.bn == 32 || pl.bn == 192 ? 4 : 2, wn = pl.bn == 256 ? 4 : pl.bn == 32 ? 1 : 2;
    snprintf(buf, sizeof buf, "k_gemm<%d, %d, %d, %d, %d, %s, %s>", pl.bm, pl.bn, wm, wn, pl.epi, c, r);
  } else if (pl.kind == -2) {
    snprintf(buf, sizeof buf, "invalid");
  } else {
    snprintf(buf, sizeof buf, "unsupported");
  }
  return buf;
}

// ---------------------------------------------------------------------------
// MX fp8 GEMM (i2pc_gemm_fp8): always the persistent engine, BM 256, BN 256 (N % 256 == 0)
// or 128 (N % 128 == 0).  Epilogues: bf16 out (+ bf16 residual(s)), fp32 out + fp32
// residual, MX fp8 out (EPI_Q8); conv A (implicit im2col, Cin % 128 == 0) optionally with
// ReLU on load.
struct Plan8 { int bn, epi; };

static int plan8(const Args& p, bool conv, bool relu, bool q8, Plan8& pl) {
  pl.bn = p.N % 256 == 0 ? 256 : p.N % 128 == 0 ? 128 : 0;
  if (!pl.bn) return set_error(I2PC_EUNSUPPORTED, "gemm_fp8: N=%d must be a multiple of 128", p.N);
  if (p.ct_s > 0) return set_error(I2PC_EUNSUPPORTED, "gemm_fp8: no ConvTranspose store");
  int epi = -1;
  if ((p.rbias || p.tbl) && (p.res || p.res2 || p.c_f32))
    return set_error(I2PC_EUNSUPPORTED, "gemm_fp8: row bias / table only with a bf16 or fp8 output and no residual");
  if (q8) epi = (!p.res && !p.res2) ? pers::EPI_Q8 : -1;
  else if (!p.res && !p.res2 && !p.c_f32) epi = pers::EPI_PLAIN;
  else if (p.res && p.res_f32 && p.c_f32 && !p.res2) epi = pers::EPI_RESF32;
  else if (p.res && !p.res_f32 && !p.c_f32 && !p.res2) epi = pers::EPI_RESBF16;
  else if (p.res && !p.res_f32 && !p.c_f32 && p.res2) epi = pers::EPI_RES2;
  // instantiated combinations
  const bool ok = conv ? (pl.bn == 256 ? (epi == pers::EPI_PLAIN && !relu) || epi == pers::EPI_Q8 ||
                                             ((epi == pers::EPI_RESBF16 || epi == pers::EPI_RES2) && !relu)
                                       : epi == pers::EPI_PLAIN && !relu)
                       : !relu && pl.bn == 256 && (epi == pers::EPI_PLAIN || epi == pers::EPI_RESF32 || epi == pers::EPI_Q8);
  if (!ok) return set_error(I2PC_EUNSUPPORTED, "gemm_fp8: epilogue %d (conv %d relu %d bn %d) not instantiated", epi, conv, relu, pl.bn);
  if (!conv && p.a_g != 0) return set_error(I2PC_EUNSUPPORTED, "gemm_fp8: no A row groups");
  const int64_t esz = q8 ? 1 : p.c_f32 ? 4 : 2;
  const int64_t abytes = conv ? (int64_t)p.cb * p.ch * p.cw * p.cc : (int64_t)(p.M + 256) * p.lda;
  const int64_t cbytes = (max_row(p) * p.ldc + p.N) * esz;
  int64_t rbytes = 0;
  if (p.res) rbytes = std::max(rbytes, (max_row(p) * p.ldr + p.N) * (p.res_f32 ? 4 : 2));
  if (p.res2) rbytes = std::max(rbytes, (max_row(p) * p.ldr2 + p.N) * 2);
  if (abytes >= pers::OOB || (int64_t)p.N * p.ldw >= pers::OOB || cbytes >= pers::OOB || rbytes >= pers::OOB)
    return set_error(I2PC_EUNSUPPORTED, "gemm_fp8: operand beyond the 31-bit buffer range");
  pl.epi = epi;
  return I2PC_OK;
}

static int run8(const Plan8& pl, const Args& p, bool conv, bool relu, hipStream_t s) {
  using namespace pers;
  if (!conv) {
    if (pl.epi == EPI_PLAIN) launch_p<256, false, false, EPI_PLAIN, 256, true>(p, s);
    else if (pl.epi == EPI_RESF32) launch_p<256, false, false, EPI_RESF32, 256, true>(p, s);
    else launch_p<256, false, false, EPI_Q8, 256, true>(p, s);
  } else if (pl.bn == 128) {
    launch_p<256, true, false, EPI_PLAIN, 128, true>(p, s);
  } else if (pl.epi == EPI_Q8) {
    if (relu) launch_p<256, true, true, EPI_Q8, 256, true>(p, s);
    else launch_p<256, true, false, EPI_Q8, 256, true>(p, s);
  } else if (pl.epi == EPI_PLAIN) {
    launch_p<256, true, false, EPI_PLAIN, 256, true>(p, s);
  } else if (pl.epi == EPI_RESBF16) {
    launch_p<256, true, false, EPI_RESBF16, 256, true>(p, s);
  } else {
    launch_p<256, true, false, EPI_RES2, 256, true>(p, s);
  }
  return check_launch("gemm_fp8");
}

static const char* plan8_name(const Plan8& pl, bool conv, bool relu) {
  static thread_local char buf[96];
  static const char* epis[] = {"plain", "res_f32", "res_bf16", "res2", "convT", "q8"};
  snprintf(buf, sizeof buf, "k_gemm_f8<%d, %s, %s, %s>", pl.bn, conv ? "true" : "false", relu ? "true" : "false",
           epis[pl.epi]);
  return buf;
}

}  // namespace gemm
}  // namespace i2pc

using namespace i2pc;

#ifdef I2PC_STAMPS
extern "C" int i2pc_debug_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(i2pc::gemm::g_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif

static int make_args(const i2pc_gemm_desc* d, gemm::Args& p) {
  I2PC_REQUIRE(d != nullptr, "desc is NULL");
  I2PC_REQUIRE(d->a && d->w && d->c, "NULL operand");
  I2PC_REQUIRE(d->m > 0 && d->n > 0 && d->k > 0, "empty gemm");
  I2PC_REQUIRE(d->k % 64 == 0, "gemm: K=%d must be a multiple of 64", d->k);
  I2PC_REQUIRE(d->n % 4 == 0, "gemm: N must be a multiple of 4");
  p = gemm::Args{};
  p.A = static_cast<const gemm::bf16_t*>(d->a);
  p.lda = d->lda; p.M = d->m; p.N = d->n; p.K = d->k;
  p.a_g = d->a_group; p.a_gs = d->a_group_stride; p.a_o = d->a_offset;
  p.W = static_cast<const gemm::bf16_t*>(d->w); p.ldw = d->ldw;
  p.bias = d->bias;
  p.rbias = d->row_bias; p.rb_g = d->row_bias_group > 0 ? d->row_bias_group : 1;
  p.tbl = d->table; p.tbl_rows = d->table_rows > 0 ? d->table_rows : 1;
  p.act = d->act == 1 && gemm::g_gelu_tanh ? 3 : d->act;
  p.res = d->res; p.res_f32 = d->res_f32; p.ldr = d->ldr;
  p.res2 = static_cast<const gemm::bf16_t*>(d->res2); p.ldr2 = d->ldr2;
  p.C = d->c; p.c_f32 = d->c_f32; p.ldc = d->ldc;
  p.o_g = d->out_group; p.o_gs = d->out_group_stride; p.o_o = d->out_offset;
  p.ct_s = d->convt_s; p.ct_h = d->convt_h; p.ct_w = d->convt_w; p.ct_c = d->convt_c;
  p.lnr = d->ln_rows; p.csum = d->col_sum;
  p.lnp = d->ln_part; p.cbf = static_cast<gemm::bf16_t*>(d->c_bf16); p.ldcb = d->ldc_bf16;
  p.lnsh = d->ln_part ? d->ln_shift : nullptr;
  p.lnc = d->ln_chunk ? d->ln_chunk : 64;
  p.rsh = d->res_shift;
  if (d->ln_rows) I2PC_REQUIRE(d->col_sum, "gemm: ln_rows needs col_sum");
  if (d->res_shift) I2PC_REQUIRE(d->res && !d->res_f32 && d->ln_part, "gemm: res_shift needs a bf16 res in a producer call");
  if (d->ln_part && !d->c_f32) {
    // bf16 residual stream: C is the shifted bf16 copy itself
    I2PC_REQUIRE(!d->c_bf16 || d->c_bf16 == d->c, "gemm: a bf16-output producer writes its copy to c (c_bf16 NULL or c)");
    p.cbf = static_cast<gemm::bf16_t*>(d->c);
    p.ldcb = d->ldc;
  }
  if (d->ln_part) {
    I2PC_REQUIRE(p.lnc == 32 || p.lnc == 64, "gemm: ln_chunk=%d must be 0, 32 or 64", d->ln_chunk);
    I2PC_REQUIRE(p.cbf && d->n % p.lnc == 0 && p.ldcb % 8 == 0 && p.ldcb >= d->n,
                 "gemm: ln_part needs c_bf16 (ldc_bf16 %% 8, >= n) or a bf16 output, and n %% ln_chunk == 0");
    I2PC_REQUIRE(d->out_group == 0 && d->out_offset == 0 && d->convt_s == 0, "gemm: ln_part needs a linear output row map");
    I2PC_REQUIRE(!d->ln_rows, "gemm: ln_part and ln_rows in one call");
  }
  if (d->conv) {
    I2PC_REQUIRE(d->conv_c % 64 == 0, "conv: Cin=%d must be a multiple of 64", d->conv_c);
    I2PC_REQUIRE(d->k == d->conv_k * d->conv_k * d->conv_c, "conv: K != k*k*Cin");
    I2PC_REQUIRE(d->m == d->conv_batch * d->conv_oh * d->conv_ow, "conv: M != B*OH*OW");
    p.cb = d->conv_batch; p.ch = d->conv_h; p.cw = d->conv_w; p.cc = d->conv_c;
    p.coh = d->conv_oh; p.cow = d->conv_ow; p.ck = d->conv_k; p.cs = d->conv_stride; p.cp = d->conv_pad;
  }
  return I2PC_OK;
}

extern "C" int i2pc_gemm_ws(const i2pc_gemm_desc* d, void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  gemm::Args p;
  const int rc = make_args(d, p);
  if (rc != I2PC_OK) return rc;
  hipStream_t s = as_stream(stream);
  const bool conv = d->conv != 0, relu = d->conv_relu_in != 0;
  const gemm::Plan pl = gemm::plan_for(p, conv, relu);
  const gemm::SplitPlan sp = gemm::split_for(p, pl);
  if (sp.splits > 1 && workspace && (int64_t)workspace_bytes >= sp.bytes) {
    I2PC_REQUIRE(reinterpret_cast<uintptr_t>(workspace) % 16 == 0, "gemm workspace must be 16-byte aligned");
    float* ws = static_cast<float*>(workspace);
    if (conv) return relu ? gemm::run_split<true, true>(sp, p, ws, s) : gemm::run_split<true, false>(sp, p, ws, s);
    return relu ? gemm::run_split<false, true>(sp, p, ws, s) : gemm::run_split<false, false>(sp, p, ws, s);
  }
  if (conv) return relu ? gemm::run_plan<true, true>(pl, p, s) : gemm::run_plan<true, false>(pl, p, s);
  return relu ? gemm::run_plan<false, true>(pl, p, s) : gemm::run_plan<false, false>(pl, p, s);
}

extern "C" int i2pc_gemm(const i2pc_gemm_desc* d, void* stream) { return i2pc_gemm_ws(d, nullptr, 0, stream); }

// Planning pass of a caller that builds its descriptors ahead of the launches (model.cpp): the same
// validation and plan as i2pc_gemm_ws, without a launch; sets the thread's error like the launch would.
int i2pc_gemm_check(const i2pc_gemm_desc* d, size_t* workspace_bytes) {
  gemm::Args p;
  const int rc = make_args(d, p);
  if (rc != I2PC_OK) return rc;
  const gemm::Plan pl = gemm::plan_for(p, d->conv != 0, d->conv_relu_in != 0);
  if (pl.kind == -2) return set_error(I2PC_EUNSUPPORTED, "gemm: LayerNorm fold not available for this call");
  if (pl.kind == -1) return set_error(I2PC_EUNSUPPORTED, "gemm: N=%d must be a multiple of 32", p.N);
  const gemm::SplitPlan sp = gemm::split_for(p, pl);
  if (workspace_bytes) *workspace_bytes = sp.splits > 1 ? (size_t)sp.bytes : 0;
  return I2PC_OK;
}

extern "C" size_t i2pc_gemm_workspace_bytes(const i2pc_gemm_desc* d) {
  gemm::Args p;
  if (make_args(d, p) != I2PC_OK) return 0;
  const gemm::SplitPlan sp = gemm::split_for(p, gemm::plan_for(p, d->conv != 0, d->conv_relu_in != 0));
  return sp.splits > 1 ? (size_t)sp.bytes : 0;
}

static int make_args8(const i2pc_gemm_fp8_desc* d8, gemm::Args& p) {
  I2PC_REQUIRE(d8 != nullptr, "desc is NULL");
  const i2pc_gemm_desc* d = &d8->g;
  I2PC_REQUIRE(d->a && d->w && d->c && d8->a_scale && d8->w_scale, "NULL operand");
  I2PC_REQUIRE(d->m > 0 && d->n > 0 && d->k > 0, "empty gemm");
  I2PC_REQUIRE(d->k % 128 == 0, "gemm_fp8: K=%d must be a multiple of 128", d->k);
  I2PC_REQUIRE(!d8->c_fp8 || (d8->c_scale && d->ldc % 16 == 0 && d->n % 32 == 0), "gemm_fp8: fp8 output needs c_scale, ldc %% 16, n %% 32");
  I2PC_REQUIRE(d->lda % 16 == 0 && d->ldw % 16 == 0, "gemm_fp8: lda/ldw must be multiples of 16 bytes");
  if (d->conv) I2PC_REQUIRE(d->conv_c % 128 == 0, "gemm_fp8 conv: Cin=%d must be a multiple of 128", d->conv_c);
  gemm::Args q;
  i2pc_gemm_desc dd = *d;
  if (d->conv) dd.conv_c = d->conv_c;   // (make_args checks Cin % 64, implied)
  const int rc = make_args(&dd, q);
  if (rc != I2PC_OK) return rc;
  p = q;
  p.As = static_cast<const uint32_t*>(d8->a_scale); p.ldas = d8->lda_scale;
  p.Ws = static_cast<const uint32_t*>(d8->w_scale); p.ldws = d8->ldw_scale;
  p.Cs = static_cast<uint32_t*>(d8->c_scale); p.ldcs = d8->ldc_scale;
  I2PC_REQUIRE(d->conv || p.ldas >= d->k / 128, "gemm_fp8: lda_scale < K/128");
  I2PC_REQUIRE(p.ldws >= d->k / 128, "gemm_fp8: ldw_scale < K/128");
  return I2PC_OK;
}

extern "C" int i2pc_gemm_fp8(const i2pc_gemm_fp8_desc* d8, void* stream) {
  clear_error();
  gemm::Args p;
  int rc = make_args8(d8, p);
  if (rc != I2PC_OK) return rc;
  const i2pc_gemm_desc* d = &d8->g;
  gemm::Plan8 pl;
  rc = gemm::plan8(p, d->conv != 0, d->conv_relu_in != 0, d8->c_fp8 != 0, pl);
  if (rc != I2PC_OK) return rc;
  return gemm::run8(pl, p, d->conv != 0, d->conv_relu_in != 0, as_stream(stream));
}

extern "C" const char* i2pc_gemm_fp8_kernel_name(const i2pc_gemm_fp8_desc* d8) {
  gemm::Args p;
  if (make_args8(d8, p) != I2PC_OK) return "invalid";
  gemm::Plan8 pl;
  if (gemm::plan8(p, d8->g.conv != 0, d8->g.conv_relu_in != 0, d8->c_fp8 != 0, pl) != I2PC_OK) return "invalid";
  return gemm::plan8_name(pl, d8->g.conv != 0, d8->g.conv_relu_in != 0);
}

extern "C" const char* i2pc_gemm_kernel_name(const i2pc_gemm_desc* d) {
  gemm::Args p;
  if (make_args(d, p) != I2PC_OK) return "invalid";
  const gemm::Plan pl = gemm::plan_for(p, d->conv != 0, d->conv_relu_in != 0);
  return gemm::plan_name(pl, d->conv != 0, d->conv_relu_in != 0, gemm::split_for(p, pl));
}

extern "C" int i2pc_gemm_set_engine(int mode) {
  clear_error();
  I2PC_REQUIRE(mode >= 0 && mode <= 4,
               "gemm engine mode %d (0 auto, 1 tile kernel only, 2 persistent wherever it applies, 3 auto with the "
               "ping-pong engine, 4 ping-pong engine wherever it applies)", mode);
  gemm::g_engine = mode;
  return I2PC_OK;
}

// per-host-thread tuning knobs (i2pc_set_tuning; thread_local above): gemm_tail, gemm_bn128,
// gemm_splitk, gemm_split_tile, gemm_tile192, gemm_lnp_p, gemm_tail160, gemm_stagger
bool i2pc_gemm_tune(const char* name, int value) {
  if (std::strcmp(name, "gemm_tail") == 0) { i2pc::gemm::g_tail = value; return true; }
  if (std::strcmp(name, "gemm_bn128") == 0) { i2pc::gemm::g_bn128 = value; return true; }
  if (std::strcmp(name, "gemm_splitk") == 0) { i2pc::gemm::g_splitk = value; return true; }
  if (std::strcmp(name, "gemm_split_tile") == 0) { i2pc::gemm::g_split_tile = value; return true; }
  if (std::strcmp(name, "gemm_tile192") == 0) { i2pc::gemm::g_tile192 = value; return true; }
  if (std::strcmp(name, "gemm_lnp_p") == 0) { i2pc::gemm::g_lnp_p = value; return true; }
  if (std::strcmp(name, "gemm_lnp_stream") == 0) { i2pc::gemm::g_lnp_stream = value; return true; }
  if (std::strcmp(name, "conv_halo") == 0) { i2pc::gemm::g_halo = value; return true; }
  if (std::strcmp(name, "gelu_tanh") == 0) { i2pc::gemm::g_gelu_tanh = value; return true; }
  if (std::strcmp(name, "gemm_resq") == 0) { i2pc::gemm::g_resq = value; return true; }
  if (std::strcmp(name, "gemm_simple_epi") == 0) { i2pc::gemm::g_simple = value; return true; }
  if (std::strcmp(name, "gemm_tail160") == 0) { i2pc::gemm::g_tail160 = value; return true; }
  if (std::strcmp(name, "gemm_stagger") == 0) { i2pc::gemm::g_stagger = value; return true; }
  return false;
}

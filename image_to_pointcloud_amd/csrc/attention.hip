// Fused multi-head self-attention, head_dim 64, bf16 in/out, fp32 softmax (gfx950).
//
// Replaces the SDPA / eager attention of DPTSelfAttention
// (transformers modeling_dpt.py:123-154, eager_attention_forward :73-98):
//   O = softmax(Q K^T * scale) V, no mask, dropout off (inference).
//
// One workgroup = 4 waves = 128 query rows of one (image, head); each wave owns
// 32 query rows.  K/V tiles of 64 keys are double-buffered in LDS (K by
// global_load_lds with an XOR-swizzled image, V transposed through registers
// into a [d][key] image for the P.V operand).  "Swapped" products with
// v_mfma_f32_32x32x16_bf16 keep each query on one lane:
//   S^T[key][q] = K . Q^T      (A = K rows from LDS, B = Q fragments in VGPRs)
//   O^T[d][q]  += V^T . P^T    (A = V^T rows from LDS, B = P straight from the
//                               S accumulators, converted to bf16 in place)
// so the online-softmax max/sum are lane-local plus one cross-half exchange.
#include "common.h"
#include "mx.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace i2pc {
namespace attn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t bf16_t;

constexpr int kQ = 128;   // query rows per workgroup
constexpr int kKV = 64;   // keys per tile
constexpr int kTileBytes = kKV * 64 * 2;   // 8 KiB (K tile and V^T tile each)

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds_base), 16, 0, 0);
}

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  // one v_cvt_pk_bf16_f32 for the pair (RNE), no shift/or repacking
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}

// V^T image: row d (128 B = 64 keys), 8-byte units of 4 keys swizzled by (d >> 1) & 15.
__device__ __forceinline__ int vt_off(int d, int key) {
  const int unit = (key >> 2) ^ ((d >> 1) & 15);
  return d * 128 + unit * 8 + (key & 3) * 2;
}

__global__ __launch_bounds__(256, 2) void k_attention(const bf16_t* __restrict__ qkv, int B, int T, int NH, float scale_log2,
                                                      bf16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * 2 * kTileBytes];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int qtiles = (T + kQ - 1) / kQ;
  // XCD-aware order: workgroups b and b + 8 share an XCD, so give each XCD a contiguous range
  // of (image, head, q-tile) indices (bijective for any count): the q-tiles of one head then
  // read its K / V through one L2 instead of up to five
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, xq = nwg >> 3, xr = nwg & 7;
  int bid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (blockIdx.x >> 3);
  const int qt = bid % qtiles;
  bid /= qtiles;
  const int h = bid % NH;
  const int b = bid / NH;
  const int D = NH * 64;
  const int64_t ld = 3 * (int64_t)D;
  const bf16_t* Qg = qkv + (int64_t)b * T * ld + h * 64;
  const bf16_t* Kg = Qg + D;
  const bf16_t* Vg = Qg + 2 * D;

  const int hh = lane >> 5;     // lane half
  const int lq = lane & 31;
  const int q = qt * kQ + wid * 32 + lq;
  const int qc = min(q, T - 1);

  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(Qg + qc * ld + 16 * s + 8 * hh);

  // K glds: 8 wave-instructions per tile (8 keys x 128 B each), 2 per wave
  auto stage_k = [&](int buf, int kt) {
    uint8_t* sK = smem + buf * 2 * kTileBytes;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (wid * 2 + j) * 8 + (lane >> 3);
      const int pchunk = lane & 7;
      const int lchunk = pchunk ^ (row & 7);
      const int key = min(kt * kKV + row, T - 1);
      glds16(Kg + key * ld + lchunk * 8, sK + (wid * 2 + j) * 8 * 128);
    }
  };
  // V: each thread loads 2 x 16 B (8 d of one key), later scattered transposed
  uint4 vreg[2];
  auto load_v = [&](int kt) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = threadIdx.x + j * 256;
      const int key = piece >> 3, ch = piece & 7;
      const int gk = min(kt * kKV + key, T - 1);
      vreg[j] = *reinterpret_cast<const uint4*>(Vg + gk * ld + ch * 8);
    }
  };
  auto write_vt = [&](int buf) {
    uint8_t* sV = smem + buf * 2 * kTileBytes + kTileBytes;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = threadIdx.x + j * 256;
      const int key = piece >> 3, d0 = (piece & 7) * 8;
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&vreg[j]);
#pragma unroll
      for (int t = 0; t < 8; ++t) *reinterpret_cast<uint16_t*>(sV + vt_off(d0 + t, key)) = e[t];
    }
  };

  f32x16 o[2];
  for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }
  float m_run = -INFINITY, l_run = 0.f;

  const int nt = (T + kKV - 1) / kKV;
  stage_k(0, 0);
  load_v(0);
  write_vt(0);
  __syncthreads();

  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nt) {
      stage_k(cur ^ 1, kt + 1);
      load_v(kt + 1);
    }
    const uint8_t* sK = smem + cur * 2 * kTileBytes;
    const uint8_t* sV = sK + kTileBytes;
    // S^T = K Q^T for two 32-key halves
    f32x16 st[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      for (int i = 0; i < 16; ++i) st[k2][i] = 0.f;
      const int key = 32 * k2 + lq;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int lchunk = 2 * s + hh;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(sK + key * 128 + ((lchunk ^ (key & 7)) << 4));
        st[k2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], st[k2], 0, 0, 0);
      }
    }
    // mask keys beyond T, scale into log2 domain, row max
    const int kbase = kt * kKV;
    float mx = -INFINITY;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + 32 * k2 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        float v = st[k2][r] * scale_log2;
        if (key >= T) v = -INFINITY;
        st[k2][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float ls = 0.f;
    uint32_t pk[2][8];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float p0 = exp2f(st[k2][r] - m_new);
        const float p1 = exp2f(st[k2][r + 1] - m_new);
        ls += p0 + p1;
        pk[k2][r >> 1] = pack_bf16(p0, p1);
      }
    l_run = l_run * alpha + ls;
#pragma unroll
    for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; }
    // O^T += V^T P^T : 4 key steps of 16 keys
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pf;
        {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          u32x4 u = {pk[k2][4 * s + 0], pk[k2][4 * s + 1], pk[k2][4 * s + 2], pk[k2][4 * s + 3]};
          pf = __builtin_bit_cast(bf16x8, u);
        }
        const int kb = 32 * k2 + 16 * s + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int d = 32 * dt + lq;
          const uint2 lo = *reinterpret_cast<const uint2*>(sV + vt_off(d, kb));
          const uint2 hi = *reinterpret_cast<const uint2*>(sV + vt_off(d, kb + 8));
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          u32x4 u = {lo.x, lo.y, hi.x, hi.y};
          const bf16x8 vf = __builtin_bit_cast(bf16x8, u);
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[dt], 0, 0, 0);
        }
      }
    if (kt + 1 < nt) write_vt(cur ^ 1);
    __syncthreads();
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  const float inv = 1.0f / l_tot;
  if (q < T) {
    bf16_t* orow = out + ((int64_t)b * T + q) * D + h * 64;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * hh;
        uint2 w;
        w.x = pack_bf16(o[dt][4 * g + 0] * inv, o[dt][4 * g + 1] * inv);
        w.y = pack_bf16(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d) = w;
      }
  }
}


// ---------------------------------------------------------------------------
// k_attention_tr: same decomposition, with
//  * V staged like K (global_load_lds, row-major [key][d] image, 128-B rows) and read
//    with ds_read_b64_tr_b16 (gfx950's transposing LDS read) straight into the
//    V^T A-operand -- no register round trip, no 16 ds_write_b16 per thread per tile;
//    chunk swizzle ((row >> 1) & 1) << 2 keeps the transposed reads conflict-free;
//  * the 1/sqrt(d) * log2(e) scale folded into the exponent (one FMA per score:
//    p = exp2(s*c - m*c), max taken on the raw scores since c > 0);
//  * key masking only on the last tile, and a last tile of <= 32 keys computes one
//    32-key half (T = 577 = 9*64 + 1: the tail was a whole wasted 64-key tile);
//  * waves whose 32 query rows are all beyond T skip the MFMA/softmax work.
__device__ __forceinline__ int v_swz(int row) { return ((row >> 1) & 1) << 2; }
// K image: 16-B chunk c of key row r at c ^ ((r >> 1) & 7).  A ds_read_b128 serves 16 lanes per LDS
// cycle (lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} and their +32 twins); a group's 16 keys
// fall into 8 even and 8 odd rows, the parity picks the 128-B half of the 256-B bank row, and
// (r >> 1) & 7 is a bijection on each parity class of a group -- conflict-free.  The r & 7 swizzle of
// r04 mapped keys 20-27 onto the chunks of keys 0-3 / 12-15: every K read was 2-way conflicted.
__device__ __forceinline__ int k_swz(int row) { return (row >> 1) & 7; }

typedef short v4s __attribute__((ext_vector_type(4)));

// 16 B per lane global -> LDS at lds_base + 16 * lane (buffer_load ... lds), issued by inline asm.
// Through __builtin_amdgcn_raw_ptr_buffer_load_lds the compiler sees an LDS write it cannot prove
// disjoint from the current tile's ds_reads, so it put s_waitcnt vmcnt(3..0) in front of this tile's
// QK^T MFMAs -- each tile waited for the NEXT tile's K / V to land and the prefetch hid nothing.  The
// kernel orders the DMA itself: vmcnt(0) + barrier before a buffer is read.  M0 carries the LDS base
// and is declared clobbered, so the compiler saves / restores any M0 value of its own around it.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t lds_base, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs), "s"(soff)
               : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__device__ __forceinline__ v4s tr_read(const uint8_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// lazy != 0: skip the alpha exponential and the O / l rescale of a tile when no query row of the
// wave raised its running max -- alpha would be exp2(0) = 1 exactly, so the skip is bit-exact
// (the usual case after the first tiles: the max of a row settles early)
// SC: the exponent arguments as single v_fma_f32 (inline asm, so the SLP vectorizer cannot pair
// them) instead of one v_pk_fma_f32 per pair -- packed FP32 ops cost extra issue cycles beside
// MFMAs (MI355X_MICROARCH.md, filler prices) -- and the row max across the two lane halves by
// v_permlane32_swap instead of ds_bpermute; the same operations, so bit-identical

// The normalised output rows of one wave: bf16 out[row][D] or (F8OUT) the MX fp8 operand.
template <bool F8OUT>
__device__ __forceinline__ void store_rows(const f32x16 (&o)[2], float inv, int q, int T, int b, int h, int D, int lane,
                                           bf16_t* __restrict__ out, uint8_t* __restrict__ out8,
                                           uint8_t* __restrict__ out8s, int lds8) {
  const int hh = lane >> 5;
  if constexpr (F8OUT) {
    // lane (lq, hh) holds d = 32 dt + 8 g + 4 hh + e of its query; the 32-d block dt is split over
    // the lane pair (lq, lq + 32), which trade amax and bytes by v_permlane32_swap (both lanes of a
    // pair share q, so both take this branch or neither)
    if (q < T) {
      const int64_t row = (int64_t)b * T + q;
      uint32_t sbytes = 0;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        float v[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t w0 = pack_bf16(o[dt][4 * g + 0] * inv, o[dt][4 * g + 1] * inv);
          const uint32_t w1 = pack_bf16(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
          v[4 * g + 0] = __uint_as_float(w0 << 16); v[4 * g + 1] = __uint_as_float(w0 & 0xffff0000u);
          v[4 * g + 2] = __uint_as_float(w1 << 16); v[4 * g + 3] = __uint_as_float(w1 & 0xffff0000u);
        }
        float am = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) am = fmaxf(am, fabsf(v[e]));
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(am), __float_as_uint(am), false, false);
        am = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
        const int ex = mx::mx_exponent(am);
        const float mul = mx::exp2i(-ex);
        uint32_t d[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) d[g] = mx::pack_e4m3(v[4 * g] * mul, v[4 * g + 1] * mul, v[4 * g + 2] * mul, v[4 * g + 3] * mul);
        // hh = 0 ends with bytes 0-15 of the block, hh = 1 with bytes 16-31
        const auto s0 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
        *reinterpret_cast<uint4*>(out8 + row * (int64_t)D + h * 64 + 32 * dt + 16 * hh) = make_uint4(s0[0], s0[1], s1[0], s1[1]);
        sbytes |= (uint32_t)(ex + 127) << (8 * dt);
      }
      if (hh == 0) *reinterpret_cast<uint16_t*>(out8s + row * (int64_t)lds8 + 2 * h) = (uint16_t)sbytes;
    }
  } else if (q < T) {
    bf16_t* orow = out + ((int64_t)b * T + q) * D + h * 64;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * hh;
        uint2 w;
        w.x = pack_bf16(o[dt][4 * g + 0] * inv, o[dt][4 * g + 1] * inv);
        w.y = pack_bf16(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d) = w;
      }
  }
}

// F8OUT: the output is written as the MX fp8 operand of the next GEMM (C5's attention-out) instead of
// bf16: e4m3 bytes out8[row][NH * 64] and one E8M0 scale byte per 32 d, out8s[row * lds8 + 2 h + dt],
// quantised from the bf16-rounded values exactly as i2pc_quant_fp8 quantises the bf16 output (so the
// bytes are those of attention -> quant_fp8, with no bf16 round trip through HBM).
template <int OCC, bool SC = false, bool F8OUT = false>
__global__ __launch_bounds__(256, OCC) void k_attention_tr(const bf16_t* __restrict__ qkv, int B, int T, int NH,
                                                           float scale_log2, bf16_t* __restrict__ out, int lazy,
                                                           uint8_t* __restrict__ out8 = nullptr,
                                                           uint8_t* __restrict__ out8s = nullptr, int lds8 = 0) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * 2 * kTileBytes];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: LDS-DMA addresses in SGPRs
  const int qtiles = (T + kQ - 1) / kQ;
  // XCD-aware order: workgroups b and b + 8 share an XCD, so give each XCD a contiguous range
  // of (image, head, q-tile) indices (bijective for any count): the q-tiles of one head then
  // read its K / V through one L2 instead of up to five
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, xq = nwg >> 3, xr = nwg & 7;
  int bid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (blockIdx.x >> 3);
  const int qt = bid % qtiles;
  bid /= qtiles;
  const int h = bid % NH;
  const int b = bid / NH;
  const int D = NH * 64;
  const int64_t ld = 3 * (int64_t)D;
  const bf16_t* Qg = qkv + (int64_t)b * T * ld + h * 64;
  const bf16_t* Kg = Qg + D;
  const bf16_t* Vg = Qg + 2 * D;

  const int hh = lane >> 5;
  const int lq = lane & 31;
  const int q = qt * kQ + wid * 32 + lq;
  const int qc = min(q, T - 1);
  const bool wave_active = qt * kQ + wid * 32 < T;      // wave-uniform

  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(Qg + qc * ld + 16 * s + 8 * hh);

  // K and V by LDS-DMA: 8 wave-instructions per tile each (8 keys x 128 B), 2 + 2 per wave.
  // Buffer descriptors over this (image, head)'s key rows: a lane's byte offset inside a tile is
  // fixed (row * ld + swizzled chunk), the tile adds a uniform kt * 64 rows, and keys past T read as
  // zero by the range check (the last tile masks them to -inf; zero V rows meet p = 0), so the
  // 64-bit clamped address arithmetic of every tile is gone.  (Bit-identical: the clamped rows were
  // copies of key T - 1 that met the same mask.)
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  const uint32_t span = (uint32_t)(((int64_t)(T - 1) * ld + 64) * 2);   // bytes through key T - 1's 64 d
  const __amdgpu_buffer_rsrc_t k_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Kg), 0, span, 0x00020000);
  const __amdgpu_buffer_rsrc_t v_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Vg), 0, span, 0x00020000);
  const uint32_t tile_bytes = (uint32_t)(kKV * ld * 2);
  uint32_t koff[2], voff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wid * 2 + j) * 8 + (lane >> 3);
    const int pchunk = lane & 7;
    koff[j] = (uint32_t)((row * ld + (pchunk ^ k_swz(row)) * 8) * 2);
    voff[j] = (uint32_t)((row * ld + (pchunk ^ v_swz(row)) * 8) * 2);
  }
  auto stage = [&](int buf, int kt) {
    uint8_t* sK = smem + buf * 2 * kTileBytes;
    uint8_t* sV = sK + kTileBytes;
    const uint32_t t0 = __builtin_amdgcn_readfirstlane((uint32_t)kt * tile_bytes);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      dma16(k_rs, __builtin_amdgcn_readfirstlane(lds_addr(sK + (wid * 2 + j) * 8 * 128)), koff[j], t0);
      dma16(v_rs, __builtin_amdgcn_readfirstlane(lds_addr(sV + (wid * 2 + j) * 8 * 128)), voff[j], t0);
    }
  };

  f32x16 o[2];
  for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }
  float m_run = -INFINITY, l_run = 0.f;          // m_run on the raw (unscaled) scores
  const float c = scale_log2;

  // transposed-read lane geometry: 16-lane group g, lane 4q'+p inside it
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  const int nt = (T + kKV - 1) / kKV;
  stage(0, 0);
  // vmcnt(0) by the builtin, which the compiler's wait-count pass sees: the Q fragments are then known
  // to have landed here.  (With no wait it knows of, it placed the Q waits at their first use INSIDE
  // the loop -- vmcnt(3..0) in front of the QK^T MFMAs of every tile, which in hardware waited for the
  // next tile's just-issued DMA.)
  __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
  __syncthreads();

  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nt) stage(cur ^ 1, kt + 1);
    const uint8_t* sK = smem + cur * 2 * kTileBytes;
    const uint8_t* sV = sK + kTileBytes;
    const int kbase = kt * kKV;
    const int nvalid = T - kbase;                  // keys of this tile that exist (>= 1)
    const bool half = nvalid <= 32;                // uniform: one 32-key half suffices
    if (wave_active) {
      f32x16 st[2];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        if (k2 == 1 && half) break;
        const int key = 32 * k2 + lq;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int lchunk = 2 * s + hh;
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(sK + key * 128 + ((lchunk ^ k_swz(key)) << 4));
          // s == 0 starts from an inline-constant zero accumulator (no 16 v_movs per chain)
          st[k2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], s == 0 ? f32x16{} : st[k2], 0, 0, 0);
        }
      }
      if (half) for (int i = 0; i < 16; ++i) st[1][i] = -INFINITY;
      if (nvalid < kKV) {                          // last tile only
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = 32 * k2 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (key >= nvalid) st[k2][r] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[k2][r]);
      if constexpr (SC) {   // the two 32-lane halves' maxima by v_permlane32_swap (VALU, no LDS round trip)
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      } else {
        mx = fmaxf(mx, __shfl_xor(mx, 32));
      }
      const float m_new = fmaxf(m_run, mx);
      // raw v_exp_f32 (ocml's exp2f adds 4 VALU ops per call for denormal results, which
      // only matter for probabilities < 2^-126 of a sum >= 1)
      const bool rescale = !lazy || __ballot(m_new != m_run) != 0;   // wave-uniform
      float alpha = 1.f;
      if (rescale) alpha = __builtin_amdgcn_exp2f((m_run - m_new) * c);
      const float mc = m_new * c;
      m_run = m_new;
      float ls = 0.f;
      uint32_t pk[2][8];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          typedef float f32x2 __attribute__((ext_vector_type(2)));
          f32x2 e;
          if constexpr (SC) {
            const float nmc = -mc;
            asm("v_fma_f32 %0, %1, %2, %3" : "=v"(e.x) : "v"(st[k2][r]), "v"(c), "v"(nmc));
            asm("v_fma_f32 %0, %1, %2, %3" : "=v"(e.y) : "v"(st[k2][r + 1]), "v"(c), "v"(nmc));
          } else {
            e = __builtin_elementwise_fma(f32x2{st[k2][r], st[k2][r + 1]}, f32x2{c, c},
                                          f32x2{-mc, -mc});     // one v_pk_fma_f32 per pair
          }
          const float p0 = __builtin_amdgcn_exp2f(e.x);
          const float p1 = __builtin_amdgcn_exp2f(e.y);
          ls += p0 + p1;
          pk[k2][r >> 1] = pack_bf16(p0, p1);
        }
      if (rescale) {
        l_run = l_run * alpha + ls;
#pragma unroll
        for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; }
      } else {
        l_run = l_run + ls;
      }
      // O^T += V^T P^T over 16-key steps; V^T fragments by transposed reads
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        if (k2 == 1 && half) break;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 pf;
          {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4 u = {pk[k2][4 * s + 0], pk[k2][4 * s + 1], pk[k2][4 * s + 2], pk[k2][4 * s + 3]};
            pf = __builtin_bit_cast(bf16x8, u);
          }
          // P's k order (swapped S^T layout): elements 0-3 = keys kb..kb+3, 4-7 = kb+8..kb+11
          const int kb = 32 * k2 + 16 * s + 4 * (tg >> 1);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const int d0 = 32 * dt + 16 * (tg & 1) + 4 * tp;      // logical column of this lane's address
            const int lch = d0 >> 3, within = (d0 & 7) * 2;
            const int r0 = kb + tq, r1 = kb + 8 + tq;
            const v4s lo = tr_read(sV + r0 * 128 + ((lch ^ v_swz(r0)) << 4) + within);
            const v4s hi = tr_read(sV + r1 * 128 + ((lch ^ v_swz(r1)) << 4) + within);
            const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[dt], 0, 0, 0);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next tile's K / V landed (this wave's part)
    __syncthreads();                                     // ... and every wave's
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  store_rows<F8OUT>(o, 1.0f / l_tot, q, T, b, h, D, lane, out, out8, out8s, lds8);
}


// ---------------------------------------------------------------------------
// k_attention_fast: k_attention_tr's tiling and staging with a shorter softmax per tile (r05).
// What bounds k_attention_tr is vector issue, not the matrix pipe (PMC, profiles/r05_attention_pmc.txt:
// ~190 VALU per 64-key tile per wave beside 16 MFMAs, MFMA busy ~29 %).  Per score it spent an FMA
// (scale and max subtraction), half a v_max3 (tile max), an exp, an add and half a cvt.  Here:
//  * Q arrives multiplied by scale * log2(e): the network folds that factor into the Q rows of its
//    QKV weights and bias (fp32, before their one bf16 rounding -- so no extra rounding anywhere), and
//    the scores come out of the MFMA in the exp2 domain (i2pc_attention_q2 / _q2_fp8);
//  * the QK^T accumulators start from -m (a 16-register block holding minus the row's running max,
//    rewritten only when the max moves), so the MFMA itself subtracts it: p = exp2(st), no FMA;
//  * the running max moves only when it must (threshold rescale): a tile's probabilities are taken
//    against the current m as long as none of them can grow large -- a lane's partial row sum below
//    2^8 bounds every p below 2^8, harmless for the bf16 P operand and the fp32 O / l accumulators.
//    Only when a lane's sum reaches 2^8 (a score above m + 3 at least) does the wave take the full
//    path: the tile max, m += max(0, tile max - m), the tile's p again and the O / l rescale.  The
//    first tile always takes it (m starts at that tile's max, so every row's l >= 1).
// The result is the same softmax (O / l is invariant to the reference point m); it differs from
// k_attention_tr by rounding only (P in bf16 against a different reference point).  (Scaling Q inside
// the kernel instead -- bf16(q * c) -- would add a rounding of Q whose error grows with the score: 6 %
// of the largest output on x4 scores against torch fp32, outside the 3 % bound; measured r05.)
template <int OCC, bool F8OUT = false, bool RB = false>
__global__ __launch_bounds__(256, OCC) void k_attention_fast(const bf16_t* __restrict__ qkv, int B, int T, int NH,
                                                             bf16_t* __restrict__ out,
                                                             uint8_t* __restrict__ out8 = nullptr,
                                                             uint8_t* __restrict__ out8s = nullptr, int lds8 = 0) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * 2 * kTileBytes];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int qtiles = (T + kQ - 1) / kQ;
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, xq = nwg >> 3, xr = nwg & 7;
  int bid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (blockIdx.x >> 3);
  const int qt = bid % qtiles;
  bid /= qtiles;
  const int h = bid % NH;
  const int b = bid / NH;
  const int D = NH * 64;
  const int64_t ld = 3 * (int64_t)D;
  const bf16_t* Qg = qkv + (int64_t)b * T * ld + h * 64;
  const bf16_t* Kg = Qg + D;
  const bf16_t* Vg = Qg + 2 * D;

  const int hh = lane >> 5;
  const int lq = lane & 31;
  const int q = qt * kQ + wid * 32 + lq;
  const int qc = min(q, T - 1);
  const bool wave_active = qt * kQ + wid * 32 < T;

  const uint32_t span = (uint32_t)(((int64_t)(T - 1) * ld + 64) * 2);
  const __amdgpu_buffer_rsrc_t k_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Kg), 0, span, 0x00020000);
  const __amdgpu_buffer_rsrc_t v_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Vg), 0, span, 0x00020000);
  const uint32_t tile_bytes = (uint32_t)(kKV * ld * 2);
  uint32_t koff[2], voff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wid * 2 + j) * 8 + (lane >> 3);
    const int pchunk = lane & 7;
    koff[j] = (uint32_t)((row * ld + (pchunk ^ k_swz(row)) * 8) * 2);
    voff[j] = (uint32_t)((row * ld + (pchunk ^ v_swz(row)) * 8) * 2);
  }
  auto stage = [&](int buf, int kt) {
    uint8_t* sK = smem + buf * 2 * kTileBytes;
    uint8_t* sV = sK + kTileBytes;
    const uint32_t t0 = __builtin_amdgcn_readfirstlane((uint32_t)kt * tile_bytes);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      dma16(k_rs, __builtin_amdgcn_readfirstlane(lds_addr(sK + (wid * 2 + j) * 8 * 128)), koff[j], t0);
      dma16(v_rs, __builtin_amdgcn_readfirstlane(lds_addr(sV + (wid * 2 + j) * 8 * 128)), voff[j], t0);
    }
  };
  const int nt = (T + kKV - 1) / kKV;
  // tile 0's DMA, the Q fragments (compiler-visible loads), then a compiler-visible vmcnt(0), so no
  // Q wait lands inside the loop (see k_attention_tr).  (A 3-slot ring prefetching two tiles ahead
  // measured equal, r05.)
  stage(0, 0);
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(Qg + qc * ld + 16 * s + 8 * hh);
  __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
  __syncthreads();

  f32x16 o[2];
  for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }
  f32x16 nm;                                     // -m of this lane's query, all 16 entries alike
  for (int i = 0; i < 16; ++i) nm[i] = 0.f;
  float l_run = 0.f;
  constexpr float kThresh = 256.f;               // 2^8

  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;

  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nt) stage(cur ^ 1, kt + 1);
    const uint8_t* sK = smem + cur * 2 * kTileBytes;
    const uint8_t* sV = sK + kTileBytes;
    const int nvalid = T - kt * kKV;
    const bool half = nvalid <= 32;
    if (wave_active) {
      // one 32-key half at a time: its QK^T, softmax and P.V before the next half's, so a half's
      // scores and probabilities are all that is live (<= 128 VGPRs: four waves per SIMD; both
      // halves' chains interleaved in one tile at 168 VGPRs and three waves measured 4 % slower on
      // C2's shape, equal on DA-v2's)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        if (k2 == 1 && half) break;
        const int key = 32 * k2 + lq;
        f32x16 st;
        if constexpr (RB) {
          // the four K fragment reads in flight together, then the four MFMAs (one LDS round trip per
          // half instead of four)
          bf16x8 kf[4];
#pragma unroll
          for (int s = 0; s < 4; ++s)
            kf[s] = *reinterpret_cast<const bf16x8*>(sK + key * 128 + (((2 * s + hh) ^ k_swz(key)) << 4));
#pragma unroll
          for (int s = 0; s < 4; ++s) st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[s], qf[s], s == 0 ? nm : st, 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int lchunk = 2 * s + hh;
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(sK + key * 128 + ((lchunk ^ k_swz(key)) << 4));
            st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], s == 0 ? nm : st, 0, 0, 0);
          }
        }
        if (nvalid < 32 * k2 + 32) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int kk = 32 * k2 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (kk >= nvalid) st[r] = -INFINITY;
          }
        }
        float ls = 0.f;
        uint32_t pk[8];
        auto probs = [&](float sub) {
          ls = 0.f;
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const float p0 = __builtin_amdgcn_exp2f(st[r] - sub);
            const float p1 = __builtin_amdgcn_exp2f(st[r + 1] - sub);
            ls += p0 + p1;
            pk[r >> 1] = pack_bf16(p0, p1);
          }
        };
        const bool first = kt == 0 && k2 == 0;                 // uniform
        bool full = first;
        if (!full) {
          probs(0.f);
          full = __ballot(ls >= kThresh) != 0;
        }
        if (full) {
          float mx = -INFINITY;
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[r]);
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
          mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
          const float delta = first ? mx : fmaxf(mx, 0.f);   // finite: the first half holds key 0
          probs(delta);
          if (!first) {
            const float alpha = __builtin_amdgcn_exp2f(-delta);
            l_run *= alpha;
#pragma unroll
            for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; }
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) nm[i] -= delta;
        }
        l_run += ls;
        bf16x8 vfs[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 pf;
          {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4 u = {pk[4 * s + 0], pk[4 * s + 1], pk[4 * s + 2], pk[4 * s + 3]};
            pf = __builtin_bit_cast(bf16x8, u);
          }
          const int kb = 32 * k2 + 16 * s + 4 * (tg >> 1);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const int d0 = 32 * dt + 16 * (tg & 1) + 4 * tp;
            const int lch = d0 >> 3, within = (d0 & 7) * 2;
            const int r0 = kb + tq, r1 = kb + 8 + tq;
            const v4s lo = tr_read(sV + r0 * 128 + ((lch ^ v_swz(r0)) << 4) + within);
            const v4s hi = tr_read(sV + r1 * 128 + ((lch ^ v_swz(r1)) << 4) + within);
            vfs[s][dt] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            if constexpr (!RB) o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfs[s][dt], pf, o[dt], 0, 0, 0);
          }
          if constexpr (RB) {
            if (s == 1) {
              // all eight V^T reads in flight, then the four MFMAs
              typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
              const bf16x8 p0 = __builtin_bit_cast(bf16x8, u32x4{pk[0], pk[1], pk[2], pk[3]});
#pragma unroll
              for (int dt = 0; dt < 2; ++dt) o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfs[0][dt], p0, o[dt], 0, 0, 0);
#pragma unroll
              for (int dt = 0; dt < 2; ++dt) o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfs[1][dt], pf, o[dt], 0, 0, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            }
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next tile's K / V landed (this wave's part)
    __syncthreads();                                     // ... and every wave's
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  store_rows<F8OUT>(o, 1.0f / l_tot, q, T, b, h, D, lane, out, out8, out8s, lds8);
}

}  // namespace attn
}  // namespace i2pc

using namespace i2pc;

// lazy rescale on by default (I2PC_ATTN_LAZY / i2pc_set_tuning "attn_lazy")
static thread_local int g_lazy = [] { const char* e = getenv("I2PC_ATTN_LAZY"); return e ? atoi(e) : 1; }();
// scalar exponent FMAs (I2PC_ATTN_SCALAR / "attn_scalar")
static thread_local int g_scalar = [] { const char* e = getenv("I2PC_ATTN_SCALAR"); return e ? atoi(e) : 1; }();
// the q2 kernel's LDS fragment reads batched per MFMA group (I2PC_ATTN_RB / "attn_rb"; bit-identical).
// Measured r06 in one process (tools/attn_ab.py, 5 rounds): C2 shape 64.4 -> 63.5 us, DA-v2
// 112.2 -> 109.1 us.  Also measured there and not kept: the next block's QK^T and the previous block's
// P.V issued beside each block's softmax (a software-pipelined form; ~140 VGPRs, so three waves per
// SIMD): C2 74.4 us, DA-v2 112.0 -- the four-wave form's cross-wave overlap was worth more.
static thread_local int g_rb = [] { const char* e = getenv("I2PC_ATTN_RB"); return e ? atoi(e) : 1; }();
bool i2pc_attention_tune(const char* name, int value) {
  if (std::strcmp(name, "attn_lazy") == 0) { g_lazy = value; return true; }
  if (std::strcmp(name, "attn_scalar") == 0) { g_scalar = value; return true; }
  if (std::strcmp(name, "attn_rb") == 0) { g_rb = value; return true; }
  return false;
}

extern "C" int i2pc_attention_fp8(const void* qkv, int batch, int tokens, int heads, float scale, void* out,
                                  int64_t ldo, void* out_scale, int64_t ldo_scale, void* stream) {
  clear_error();
  I2PC_REQUIRE(qkv && out && out_scale, "NULL pointer");
  I2PC_REQUIRE(batch > 0 && tokens > 0 && heads > 0, "attention_fp8: empty shape");
  I2PC_REQUIRE(ldo == (int64_t)heads * 64, "attention_fp8: the fp8 rows are dense (ldo = heads * 64)");
  I2PC_REQUIRE(ldo_scale * 128 >= (int64_t)heads * 64 && (reinterpret_cast<uintptr_t>(out) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(out_scale) % 4) == 0,
               "attention_fp8: scale rows of ldo_scale dwords cover heads * 2 blocks; 16-B aligned data");
  const int qtiles = (tokens + attn::kQ - 1) / attn::kQ;
  const float scale_log2 = scale * 1.4426950408889634f;
  // the same exponent form as i2pc_attention's default dispatch (occupancy 3; scalar or packed
  // exponent FMAs by the "attn_scalar" knob), so the bytes equal quant_fp8 of its bf16 output under
  // the same knobs (I2PC_ATTN_OCC / I2PC_ATTN_OLD select bf16-only variants and are not mirrored here)
  if (g_scalar)
    hipLaunchKernelGGL((attn::k_attention_tr<3, true, true>), dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, scale_log2, nullptr, g_lazy,
                       static_cast<uint8_t*>(out), static_cast<uint8_t*>(out_scale), (int)(ldo_scale * 4));
  else
    hipLaunchKernelGGL((attn::k_attention_tr<3, false, true>), dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, scale_log2, nullptr, g_lazy,
                       static_cast<uint8_t*>(out), static_cast<uint8_t*>(out_scale), (int)(ldo_scale * 4));
  return check_launch("attention_fp8");
}

extern "C" int i2pc_attention(const void* qkv, int batch, int tokens, int heads, float scale, void* out, void* stream) {
  clear_error();
  I2PC_REQUIRE(qkv && out, "NULL pointer");
  I2PC_REQUIRE(batch > 0 && tokens > 0 && heads > 0, "attention: empty shape");
  const int qtiles = (tokens + attn::kQ - 1) / attn::kQ;
  const float scale_log2 = scale * 1.4426950408889634f;
  static const int old_kernel = [] { const char* e = getenv("I2PC_ATTN_OLD"); return e ? atoi(e) : 0; }();
  // waves per SIMD the register budget targets (170 VGPRs at 2; <= 168 gives 3)
  static const int occ = [] { const char* e = getenv("I2PC_ATTN_OCC"); return e ? atoi(e) : 3; }();
  if (old_kernel)
    hipLaunchKernelGGL(attn::k_attention, dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, scale_log2, static_cast<uint16_t*>(out));
  else if (occ == 2)
    hipLaunchKernelGGL(attn::k_attention_tr<2>, dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, scale_log2, static_cast<uint16_t*>(out), g_lazy);
  else if (occ == 4)   // four waves per SIMD: the scalar-FMA form only (r05)
    hipLaunchKernelGGL((attn::k_attention_tr<4, true>), dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, scale_log2, static_cast<uint16_t*>(out), g_lazy);
  else if (g_scalar)
    hipLaunchKernelGGL((attn::k_attention_tr<3, true>), dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, scale_log2, static_cast<uint16_t*>(out), g_lazy);
  else
    hipLaunchKernelGGL(attn::k_attention_tr<3>, dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, scale_log2, static_cast<uint16_t*>(out), g_lazy);
  return check_launch("attention");
}

extern "C" int i2pc_attention_q2(const void* qkv, int batch, int tokens, int heads, void* out, void* stream) {
  clear_error();
  I2PC_REQUIRE(qkv && out, "NULL pointer");
  I2PC_REQUIRE(batch > 0 && tokens > 0 && heads > 0, "attention_q2: empty shape");
  const int qtiles = (tokens + attn::kQ - 1) / attn::kQ;
  if (g_rb)
    hipLaunchKernelGGL((attn::k_attention_fast<4, false, true>), dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, static_cast<uint16_t*>(out));
  else
    hipLaunchKernelGGL((attn::k_attention_fast<4>), dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, static_cast<uint16_t*>(out));
  return check_launch("attention_q2");
}

extern "C" int i2pc_attention_q2_fp8(const void* qkv, int batch, int tokens, int heads, void* out, int64_t ldo,
                                     void* out_scale, int64_t ldo_scale, void* stream) {
  clear_error();
  I2PC_REQUIRE(qkv && out && out_scale, "NULL pointer");
  I2PC_REQUIRE(batch > 0 && tokens > 0 && heads > 0, "attention_q2_fp8: empty shape");
  I2PC_REQUIRE(ldo == (int64_t)heads * 64, "attention_q2_fp8: the fp8 rows are dense (ldo = heads * 64)");
  I2PC_REQUIRE(ldo_scale * 128 >= (int64_t)heads * 64 && (reinterpret_cast<uintptr_t>(out) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(out_scale) % 4) == 0,
               "attention_q2_fp8: scale rows of ldo_scale dwords cover heads * 2 blocks; 16-B aligned data");
  const int qtiles = (tokens + attn::kQ - 1) / attn::kQ;
  if (g_rb)
    hipLaunchKernelGGL((attn::k_attention_fast<4, true, true>), dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, nullptr, static_cast<uint8_t*>(out),
                       static_cast<uint8_t*>(out_scale), (int)(ldo_scale * 4));
  else
    hipLaunchKernelGGL((attn::k_attention_fast<4, true>), dim3(batch * heads * qtiles), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t*>(qkv), batch, tokens, heads, nullptr, static_cast<uint8_t*>(out),
                       static_cast<uint8_t*>(out_scale), (int)(ldo_scale * 4));
  return check_launch("attention_q2_fp8");
}

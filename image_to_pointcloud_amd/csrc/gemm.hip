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

namespace i2pc {
namespace gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;

constexpr int BK = 64;
constexpr int kThreads = 256;

__device__ __attribute__((aligned(16))) uint8_t g_zero[512];   // conv zero padding source

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

template <int BM, int BN, bool CONV, bool RELU_A>
__global__ __launch_bounds__(kThreads, 2) void k_gemm(Args p) {
  constexpr int WAVES_N = BN >= 64 ? 2 : 1;
  constexpr int WAVES_M = 4 / WAVES_N;
  constexpr int TM = BM / WAVES_M;       // activation rows per wave
  constexpr int TN = BN / WAVES_N;       // output columns per wave
  constexpr int RM = TM / 16;
  constexpr int RN = TN / 16;
  constexpr int A_LOADS = BM / 32;       // glds wave-instructions per wave per tile (8 rows each)
  constexpr int W_LOADS = BN / 32;
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int W_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + W_BYTES;
  static_assert(RM >= 1 && RN >= 1, "tile too small");
  static_assert(BN % 32 == 0 && BM % 32 == 0, "tile");

  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / WAVES_N;
  const int wn = wid % WAVES_N;

  // XCD-aware tile order (bijective for any tile count).
  const int nwg = p.tiles_m * p.tiles_n;
  const int bid = blockIdx.x;
  int tile;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7, idx = bid >> 3;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  // ---- per-lane source rows for the A and W glds streams
  const int lrow = lane >> 3;          // row inside an 8-row glds slab
  const int pchunk = lane & 7;         // physical 16-B chunk this lane fills
  const bf16_t* a_src[A_LOADS];
  int cy[A_LOADS], cx[A_LOADS];
  bool cval[A_LOADS];
#pragma unroll
  for (int j = 0; j < A_LOADS; ++j) {
    const int row = (wid * A_LOADS + j) * 8 + lrow;
    const int lchunk = pchunk ^ (row & 7);
    int m = m0 + row;
    if (m > p.M - 1) m = p.M - 1;
    if (!CONV) {
      a_src[j] = p.A + (int64_t)remap(m, p.a_g, p.a_gs, p.a_o) * p.lda + lchunk * 8;
      cy[j] = cx[j] = 0;
      cval[j] = true;
    } else {
      const int hw = p.coh * p.cow;
      const int b = m / hw;
      const int rem = m - b * hw;
      const int oy = rem / p.cow;
      const int ox = rem - oy * p.cow;
      cy[j] = oy * p.cs - p.cp;
      cx[j] = ox * p.cs - p.cp;
      cval[j] = true;
      a_src[j] = p.A + (int64_t)b * p.ch * p.cw * p.cc + lchunk * 8;
    }
  }
  const bf16_t* w_src[W_LOADS];
#pragma unroll
  for (int j = 0; j < W_LOADS; ++j) {
    const int row = (wid * W_LOADS + j) * 8 + lrow;
    const int lchunk = pchunk ^ (row & 7);
    w_src[j] = p.W + (int64_t)(n0 + row) * p.ldw + lchunk * 8;
  }

  auto stage = [&](int buf, int k0) {
    uint8_t* sA = smem + buf * STAGE;
    uint8_t* sW = sA + A_BYTES;
    if (!CONV) {
#pragma unroll
      for (int j = 0; j < A_LOADS; ++j) glds16(a_src[j] + k0, sA + (wid * A_LOADS + j) * 8 * 128);
    } else {
      const int kk = k0 / p.cc;
      const int ky = kk / p.ck;
      const int kx = kk - ky * p.ck;
      const int ci0 = k0 - kk * p.cc;
#pragma unroll
      for (int j = 0; j < A_LOADS; ++j) {
        const int yi = cy[j] + ky, xi = cx[j] + kx;
        const bool ok = cval[j] && yi >= 0 && yi < p.ch && xi >= 0 && xi < p.cw;
        const void* src = ok ? (const void*)(a_src[j] + ((int64_t)yi * p.cw + xi) * p.cc + ci0)
                             : (const void*)(g_zero + pchunk * 16);
        glds16(src, sA + (wid * A_LOADS + j) * 8 * 128);
      }
    }
#pragma unroll
    for (int j = 0; j < W_LOADS; ++j) glds16(w_src[j] + k0, sW + (wid * W_LOADS + j) * 8 * 128);
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  stage(0, 0);
  __syncthreads();   // waits vmcnt(0): tile 0 landed

  const int frow = lane & 15;
  const int fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
    const uint8_t* sA = smem + cur * STAGE;
    const uint8_t* sW = sA + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[RM], wf[RN];
      const int lchunk = 4 * s + fq;
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = wm * TM + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8*>(sA + row * 128 + ((lchunk ^ (row & 7)) << 4));
        if (RELU_A) af[i] = relu8(af[i]);
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = wn * TN + j * 16 + frow;
        wf[j] = *reinterpret_cast<const bf16x8*>(sW + row * 128 + ((lchunk ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds out[m][n..n+3] for each (i, j)
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int m = m0 + wm * TM + i * 16 + frow;
    if (m >= p.M) continue;
    int orow = 0;
    int64_t obase;
    if (p.ct_s > 0) {
      const int hw = p.ct_h * p.ct_w;
      const int b = m / hw;
      const int rem = m - b * hw;
      const int iy = rem / p.ct_w;
      const int ix = rem - iy * p.ct_w;
      obase = ((int64_t)b * p.ct_h * p.ct_s + (int64_t)iy * p.ct_s) * (p.ct_w * p.ct_s) + (int64_t)ix * p.ct_s;
    } else {
      orow = remap(m, p.o_g, p.o_gs, p.o_o);
      obase = (int64_t)orow * p.ldc;
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = n0 + wn * TN + j * 16 + fq * 4;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
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
      int64_t off;
      if (p.ct_s > 0) {
        const int tap = n / p.ct_c;
        const int co = n - tap * p.ct_c;
        const int dy = tap / p.ct_s, dx = tap - dy * p.ct_s;
        off = (obase + (int64_t)dy * (p.ct_w * p.ct_s) + dx) * p.ct_c + co;
      } else {
        off = obase + n;
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
  }
}

template <int BM, int BN, bool CONV, bool RELU_A>
static void launch(const Args& p, hipStream_t s) {
  Args q = p;
  q.tiles_m = (p.M + BM - 1) / BM;
  q.tiles_n = p.N / BN;
  const int smem = 2 * (BM + BN) * BK * 2;
  hipLaunchKernelGGL((k_gemm<BM, BN, CONV, RELU_A>), dim3(q.tiles_m * q.tiles_n), dim3(kThreads), smem, s, q);
}

template <bool CONV, bool RELU_A>
static int dispatch(const Args& p, hipStream_t s) {
  // Prefer the 128x128 tile; narrow N and small grids take narrower tiles.
  const int64_t t128 = (int64_t)((p.M + 127) / 128) * (p.N / 128);
  if (p.N % 128 == 0 && t128 >= 512) launch<128, 128, CONV, RELU_A>(p, s);
  else if (p.N % 64 == 0) launch<128, 64, CONV, RELU_A>(p, s);
  else if (p.N % 32 == 0) launch<128, 32, CONV, RELU_A>(p, s);
  else return set_error(I2PC_EUNSUPPORTED, "gemm: N=%d must be a multiple of 32", p.N);
  return check_launch("gemm");
}

}  // namespace gemm
}  // namespace i2pc

using namespace i2pc;

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

// Batched depth -> (x, y, z, rgb) back-projection for gfx950 (MI355X).
//
// Replaces backend/app.py:174-250 (depth_to_point_cloud) and the bounds of
// generate_gis_metadata (app.py:393-400) for a whole batch of images.
//
// Pipeline per call (all stream-ordered, graph-capturable, fixed launch list):
//   k_init            per-image selection state + cv2 INTER_LINEAR tap tables
//   k_sel_hist/resolve x3 levels (pass 0)   exact order statistics of the
//                     full-resolution depth (recomputed on the fly from the
//                     model-resolution map, which stays L2-resident): the
//                     p2/p98 ranks of np.percentile (app.py:197) -- or, if the
//                     map holds NaN/Inf, the ranks of np.nanmedian (app.py:195)
//   k_sel_hist/resolve x3 levels (pass 1)   only when a nanmedian fill was
//                     needed: p2/p98 of the sanitised map (no-op launches otherwise)
//   [k_norm_field, k_blur<rows>, k_blur<cols>]  only when smooth=True (app.py:209-214), any odd k
//   k_unproject       normalise (fp64 / fp32 / constant branch exactly as
//                     numpy evaluates app.py:198-206), pinhole back-projection in
//                     Python-double semantics (app.py:219-238), RGB gather
//                     (app.py:239-244), per-image bbox via wave reductions
//   k_finalize        bbox / stats to float64
//
// Selection: 3-level radix select on order-preserving 32-bit float keys
// (11 + 11 + 10 bits) with LDS histograms and wave-aggregated LDS atomics
// (a smooth depth field puts most lanes of a wave in the same bin).
// Arithmetic is bit-faithful: no FMA contraction in this file.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <cmath>

#pragma clang fp contract(off)

namespace i2pc {
namespace unproj {

constexpr int kSlots = 4;
constexpr int kBins = 2048;
constexpr int kBlock = 256;
constexpr int kMaxRows = 4;   // unprojection rows per workgroup (register-prefetched RGB)

enum Phase : uint32_t { PH_INIT = 0, PH_PCT = 1, PH_MED = 2, PH_PCT2_INIT = 3, PH_PCT2 = 4, PH_DONE = 5 };

struct Tap {
  int i0, i1;     // i1 < 0: single tap (cv2 HResizeLinear right border copies S[sx])
  float w0, w1;
};

struct alignas(16) SelState {
  uint32_t phase;
  uint32_t n;            // pixels per image
  uint32_t nan_count;
  uint32_t nonfinite_count;
  uint32_t kmin, kmax;   // ordered keys of the non-NaN values of the current pass
  uint32_t ntgt, nslot;
  uint32_t rank[4];      // remaining rank of each target inside its prefix range
  uint32_t prefix[4];
  uint32_t slot[4];
  uint32_t slot_prefix[4];
  uint32_t med_ranks;    // 1 = odd count (one rank), 2 = even
  uint32_t has_med;
  float med;
  int32_t mode;          // 0: float64 branch, 1: float32 min/max branch, 2: constant
  uint32_t err;
  uint32_t pad0;
  double p2, p98, den64;
  float lo32, hi32, den32, pad1;
  uint32_t bbox_key[6];
  uint32_t pad2[2];
  double rden64;         // RN(1 / den64): quotient seed for div_rn
  double pad3;
};

// Correctly rounded a / b from r = RN(1 / b) (Markstein's correction: q0 = RN(a r),
// rem = a - q0 b exactly by FMA, q = RN(q0 + rem r)).  Three FP64 ops instead of the
// ~10-op scaled division sequence; bit-identical to IEEE a / b (brute-forced on 2e8
// random operand pairs incl. all-ones significands, tools/check_div_rn.c).
__device__ __forceinline__ double div_rn(double a, double b, double r) {
  const double q0 = a * r;
  const double rem = __builtin_fma(-q0, b, a);
  return __builtin_fma(rem, r, q0);
}

struct Geo {
  const float* depth;
  int dh, dw, H, W;
  const Tap* xt;
  const Tap* yt;
  int same;  // depth already at image resolution: app.py:187 skips cv2.resize
  double sx, sy;  // cv2 inverse scales 1 / (out / in) per axis (host-computed, IEEE-identical)
};

// cv2's inverse scale for one axis (resize.cpp: scale_x = 1. / inv_scale_x, inv_scale_x = dsize / ssize)
inline double cv_scale(int in, int out) { return 1.0 / ((double)out / (double)in); }

struct Layout {
  size_t state, hist, xtab, ytab, ex, field, tmp, total;
};

static Layout layout(int B, int H, int W, int smooth) {
  Layout L{};
  size_t off = 0;
  L.state = off; off = align_up(off + sizeof(SelState) * (size_t)B, 256);
  L.hist = off;  off = align_up(off + sizeof(uint32_t) * kSlots * kBins * (size_t)B, 256);
  L.xtab = off;  off = align_up(off + sizeof(Tap) * (size_t)W, 256);
  L.ytab = off;  off = align_up(off + sizeof(Tap) * (size_t)H, 256);
  L.ex = off;    off = align_up(off + sizeof(int64_t) * 4 * (size_t)B, 256);
  L.field = off;
  if (smooth) {
    off = align_up(off + sizeof(double) * (size_t)B * H * W, 256);
    L.tmp = off;
    off = align_up(off + sizeof(double) * (size_t)B * H * W, 256);
  } else {
    L.tmp = off;
  }
  L.total = off;
  return L;
}

// ---------------------------------------------------------------- device utils

__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// Blocks b and b+8 share an XCD (round-robin dispatch): when the batch is a
// multiple of 8, give every image's blocks to one XCD so its model-resolution
// depth map is read from one L2.
__device__ __forceinline__ void map_block(int bid, int B, int G, int& b, int& chunk) {
  if ((B & 7) == 0) {
    int xcd = bid & 7, slot = bid >> 3, per = B >> 3;
    b = xcd + 8 * (slot % per);
    chunk = slot / per;
  } else {
    b = bid % B;
    chunk = bid / B;
  }
}

__device__ __forceinline__ float sample(const Geo& g, int b, int v, int u) {
  const float* D = g.depth + (size_t)b * g.dh * g.dw;
  if (g.same) return D[(size_t)v * g.dw + u];
  const Tap ty = g.yt[v];
  const Tap tx = g.xt[u];
  const float* r0 = D + (size_t)ty.i0 * g.dw;
  const float* r1 = D + (size_t)ty.i1 * g.dw;
  float h0, h1;
  if (tx.i1 < 0) {
    h0 = r0[tx.i0];
    h1 = r1[tx.i0];
  } else {
    h0 = r0[tx.i0] * tx.w0 + r0[tx.i1] * tx.w1;
    h1 = r1[tx.i0] * tx.w0 + r1[tx.i1] * tx.w1;
  }
  return h0 * ty.w0 + h1 * ty.w1;
}

// Wave-aggregated LDS histogram add: lanes with equal bins are merged (up to 4
// distinct bins per wave-instruction), the rest fall back to per-lane atomics.
__device__ __forceinline__ void agg_add(uint32_t* h, int bin, bool active) {
  const int lane = threadIdx.x & 63;
  uint64_t pending = __ballot(active);
  for (int it = 0; it < 4 && pending; ++it) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const int lbin = __builtin_amdgcn_readlane(bin, leader);   // SALU broadcast, no LDS round trip
    const uint64_t same = __ballot(active && bin == lbin) & pending;
    if (lane == leader) atomicAdd(&h[lbin], (uint32_t)__popcll(same));
    pending &= ~same;
  }
  if ((pending >> lane) & 1ull) atomicAdd(&h[bin], 1u);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o));
  return x;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
  return x;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o);
  return x;
}

// cv2 resize.cpp INTER_LINEAR tap geometry (fx computed in double, cast to float).
__device__ Tap make_tap(int dx, int in, double scale) {
  float fx = (float)(((double)dx + 0.5) * scale - 0.5);
  int sx = (int)floorf(fx);
  fx = fx - (float)sx;
  Tap t;
  bool right = false;
  if (sx < 0) { fx = 0.f; sx = 0; }
  if (sx >= in - 1) { fx = 0.f; sx = in - 1; right = true; }
  t.i0 = sx;
  t.i1 = right ? -1 : sx + 1;
  t.w0 = 1.0f - fx;
  t.w1 = fx;
  return t;
}

// ---------------------------------------------------------------- kernels

__global__ void k_init(SelState* st, int B, int n, Tap* xt, Tap* yt, int dh, int dw, int H, int W, double sx,
                       double sy) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid < B) {
    SelState s{};
    s.phase = PH_INIT;
    s.n = (uint32_t)n;
    s.kmin = 0xffffffffu;
    s.kmax = 0u;
    for (int i = 0; i < 6; i += 2) { s.bbox_key[i] = 0xffffffffu; s.bbox_key[i + 1] = 0u; }
    s.med = __uint_as_float(0x7fc00000u);
    st[tid] = s;
  }
  if (tid < W) {
    Tap t = make_tap(tid, dw, sx);
    if (dw == 1) { t.i0 = 0; t.i1 = -1; t.w0 = 1.f; t.w1 = 0.f; }
    xt[tid] = t;
  }
  if (tid < H) {
    Tap t = make_tap(tid, dh, sy);
    // vertical pass always uses two rows: the second clamps to the last row
    if (t.i1 < 0) t.i1 = t.i0;
    yt[tid] = t;
  }
}

template <int PASS>
__device__ __forceinline__ bool hist_gate(uint32_t phase, int level) {
  if (PASS == 0) return level == 0 ? phase == PH_INIT : (phase == PH_PCT || phase == PH_MED);
  return level == 0 ? phase == PH_PCT2_INIT : phase == PH_PCT2;
}

// Row-blocked sweep geometry: a workgroup owns image b and output rows [v0, v1);
// the model-resolution rows feeding them are staged once into LDS, every thread
// owns 4 consecutive columns (+1024 per chunk), the row taps are wave-uniform.
struct Sweep {
  int R;         // output rows per workgroup
  int nrb;       // row blocks per image
  int lds_rows;  // capacity of the LDS row window (0: sample from global)
  int row0;      // first output row swept (a band of the image in tile-parallel mode)
  int row_end;   // one past the last output row swept
};

__device__ __forceinline__ void map_rows(int bid, int B, int nrb, int& b, int& rb) { map_block(bid, B, nrb, b, rb); }

// Stage model rows [yt[v0].i0, yt[v1-1].i1] of image b into LDS; returns the first row.
__device__ __forceinline__ int stage_rows(const Geo& g, int b, int v0, int v1, float* rows, int cap) {
  if (g.same || cap == 0) return 0;
  const int lo = g.yt[v0].i0;
  const int hi = g.yt[v1 - 1].i1;
  const int n = (hi - lo + 1) * g.dw;
  const float* src = g.depth + ((size_t)b * g.dh + lo) * g.dw;
  for (int i = threadIdx.x; i < n; i += blockDim.x) rows[i] = src[i];
  return lo;
}

__device__ __forceinline__ float sample_rows(const Geo& g, const float* rows, int lo, bool use_lds, int b,
                                             const Tap& ty, int v, int u) {
  if (g.same) return g.depth[((size_t)b * g.dh + v) * g.dw + u];
  if (!use_lds) return sample(g, b, v, u);
  const Tap tx = g.xt[u];
  const float* r0 = rows + (ty.i0 - lo) * g.dw;
  const float* r1 = rows + (ty.i1 - lo) * g.dw;
  float h0, h1;
  if (tx.i1 < 0) {
    h0 = r0[tx.i0];
    h1 = r1[tx.i0];
  } else {
    h0 = r0[tx.i0] * tx.w0 + r0[tx.i1] * tx.w1;
    h1 = r1[tx.i0] * tx.w0 + r1[tx.i1] * tx.w1;
  }
  return h0 * ty.w0 + h1 * ty.w1;
}

// (Materialising the keys in the first sweep and streaming them in the later ones
// was measured slower: the sweeps are bound by the histogram, not the resize.)
template <int LEVEL, int PASS>
__global__ __launch_bounds__(kBlock) void k_sel_hist(Geo g, SelState* st, uint32_t* hist, int B, Sweep sw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_u[];
  uint32_t* sh = smem_u;                                        // [slots * kBins]
  float* rows = reinterpret_cast<float*>(smem_u + (LEVEL == 0 ? 1 : kSlots) * kBins);
  __shared__ uint32_t red[4][4];
  int b, rb;
  map_rows(blockIdx.x, B, sw.nrb, b, rb);
  SelState* S = st + b;
  const uint32_t phase = S->phase;
  if (!hist_gate<PASS>(phase, LEVEL)) return;

  const int nslot = LEVEL == 0 ? 1 : (int)S->nslot;
  uint32_t sp[kSlots];
#pragma unroll
  for (int q = 0; q < kSlots; ++q) sp[q] = S->slot_prefix[q];
  const bool sanitize = PASS == 1;
  const float med = S->med;
  constexpr int match_shift = LEVEL == 1 ? 21 : 10;
  constexpr int bin_shift = LEVEL == 0 ? 21 : (LEVEL == 1 ? 10 : 0);
  constexpr uint32_t bin_mask = LEVEL == 2 ? 1023u : 2047u;

  const int v0 = sw.row0 + rb * sw.R;
  const int v1 = min(sw.row_end, v0 + sw.R);
  for (int i = threadIdx.x; i < nslot * kBins; i += kBlock) sh[i] = 0;
  const int lo = stage_rows(g, b, v0, v1, rows, sw.lds_rows);
  const bool use_lds = sw.lds_rows > 0;
  __syncthreads();

  uint32_t nan_c = 0, nonfin_c = 0, kmin = 0xffffffffu, kmax = 0u;
  // thread columns u = cb + j*256 + tid: neighbouring lanes read neighbouring LDS words
  for (int cb = 0; cb < g.W; cb += 4 * kBlock) {
    Tap tx[4];
    bool colok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int u = cb + j * kBlock + threadIdx.x;
      colok[j] = u < g.W;
      tx[j] = g.xt[min(u, g.W - 1)];      // unconditional (clamped) load: no divergent waits
    }
    for (int v = v0; v < v1; ++v) {
      const Tap ty = g.same ? Tap{0, 0, 1.f, 0.f} : g.yt[v];
      const float* r0 = use_lds ? rows + (ty.i0 - lo) * g.dw : g.depth + ((size_t)b * g.dh + ty.i0) * g.dw;
      const float* r1 = use_lds ? rows + (ty.i1 - lo) * g.dw : g.depth + ((size_t)b * g.dh + ty.i1) * g.dw;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int u = min(cb + j * kBlock + threadIdx.x, g.W - 1);
        bool active = colok[j];
        float val;
        if (g.same) {
          val = g.depth[((size_t)b * g.dh + v) * g.dw + u];
        } else {
          // single-tap columns (i1 < 0) use weights (1, 0) on a duplicated index: identical
          // value except for Inf/NaN neighbours, so keep the exact expression via select
          const int i1 = tx[j].i1 < 0 ? tx[j].i0 : tx[j].i1;
          const float a0 = r0[tx[j].i0], a1 = r0[i1], c0 = r1[tx[j].i0], c1 = r1[i1];
          const float h0 = tx[j].i1 < 0 ? a0 : a0 * tx[j].w0 + a1 * tx[j].w1;
          const float h1 = tx[j].i1 < 0 ? c0 : c0 * tx[j].w0 + c1 * tx[j].w1;
          val = h0 * ty.w0 + h1 * ty.w1;
        }
        if (sanitize && !isfinite(val)) val = med;
        if (LEVEL == 0 && active && !isfinite(val)) ++nonfin_c;   // NaN and +-Inf
        if (active && isnan(val)) { ++nan_c; active = false; }
        const uint32_t key = f2key(val);
        int bin = 0;
        if (LEVEL == 0) {
          if (active) { kmin = min(kmin, key); kmax = max(kmax, key); }
          bin = (int)((key >> bin_shift) & bin_mask);
        } else {
          bool hit = false;
#pragma unroll
          for (int q = 0; q < kSlots; ++q) {
            if (q < nslot && (key >> match_shift) == sp[q]) { hit = true; bin = q * kBins + (int)((key >> bin_shift) & bin_mask); }
          }
          active = active && hit;
        }
        agg_add(sh, bin, active);
      }
    }
  }
  if (LEVEL == 0) {
    const int wid = threadIdx.x >> 6;
    nan_c = wave_sum_u32(nan_c);
    nonfin_c = wave_sum_u32(nonfin_c);
    kmin = wave_min_u32(kmin);
    kmax = wave_max_u32(kmax);
    if ((threadIdx.x & 63) == 0) { red[0][wid] = nan_c; red[1][wid] = nonfin_c; red[2][wid] = kmin; red[3][wid] = kmax; }
  }
  __syncthreads();
  if (LEVEL == 0 && threadIdx.x == 0) {
    uint32_t a = 0, c = 0, mn = 0xffffffffu, mx = 0;
    for (int w = 0; w < kBlock / 64; ++w) { a += red[0][w]; c += red[1][w]; mn = min(mn, red[2][w]); mx = max(mx, red[3][w]); }
    if (a) atomicAdd(&S->nan_count, a);
    if (c) atomicAdd(&S->nonfinite_count, c);
    if (mn != 0xffffffffu) atomicMin(&S->kmin, mn);
    if (mx) atomicMax(&S->kmax, mx);
  }
  uint32_t* gh = hist + (size_t)b * kSlots * kBins;
  for (int i = threadIdx.x; i < nslot * kBins; i += kBlock) {
    const uint32_t c = sh[i];
    if (c) atomicAdd(&gh[i], c);
  }
}

// Find, for one histogram of `nb` bins, the bin holding 0-based `rank`
// (all threads call; result left in *out_bin / *out_rem by the owning thread).
__device__ void find_bin(const uint32_t* h, int nb, uint32_t rank, uint32_t* sc, uint32_t* out_bin, uint32_t* out_rem) {
  const int per = nb / kBlock;   // 8 or 4
  const int t = threadIdx.x;
  uint32_t local = 0;
  for (int i = 0; i < per; ++i) local += h[t * per + i];
  sc[t] = local;
  __syncthreads();
  // Hillis-Steele inclusive scan over 256 entries
  for (int o = 1; o < kBlock; o <<= 1) {
    uint32_t x = t >= o ? sc[t - o] : 0u;
    __syncthreads();
    sc[t] += x;
    __syncthreads();
  }
  const uint32_t incl = sc[t];
  const uint32_t excl = incl - local;
  if (rank >= excl && rank < incl) {
    uint32_t c = excl;
    for (int i = 0; i < per; ++i) {
      const uint32_t hv = h[t * per + i];
      if (rank < c + hv) { *out_bin = (uint32_t)(t * per + i); *out_rem = rank - c; break; }
      c += hv;
    }
  }
  __syncthreads();
}

__device__ void pct_targets(SelState& s) {
  const uint32_t n = s.n;
  int k = 0;
  const double qs[2] = {2.0 / 100.0, 98.0 / 100.0};   // q = [2,98] / float32(100) -> float64
  for (int j = 0; j < 2; ++j) {
    const double v = (double)(n - 1) * qs[j];
    uint32_t i0, i1;
    if (v >= (double)(n - 1)) { i0 = i1 = n - 1; }
    else { i0 = (uint32_t)floor(v); i1 = i0 + 1; }
    s.rank[k++] = i0;
    s.rank[k++] = i1;
  }
  s.ntgt = 4;
  for (int i = 0; i < 4; ++i) s.prefix[i] = 0;
}

__device__ void finalize_pct(SelState& s) {
  const uint32_t n = s.n;
  const double qs[2] = {2.0 / 100.0, 98.0 / 100.0};
  double r[2];
  for (int j = 0; j < 2; ++j) {
    const double v = (double)(n - 1) * qs[j];
    const double t = v - floor(v);
    const float a = key2f(s.prefix[2 * j]);
    const float bb = key2f(s.prefix[2 * j + 1]);
    const float diff = bb - a;
    r[j] = t >= 0.5 ? (double)bb - (double)diff * (1.0 - t) : (double)a + (double)diff * t;
  }
  double p2 = r[0], p98 = r[1];
  int branch = 0;
  if (p98 <= p2) {                       // app.py:198-199
    p2 = (double)key2f(s.kmin);
    p98 = (double)key2f(s.kmax);
    branch = 1;
  }
  if (p98 > p2) {
    s.mode = branch;
    s.den64 = (p98 - p2) + 1e-6;
    s.rden64 = 1.0 / s.den64;
    s.lo32 = (float)p2;
    s.hi32 = (float)p98;
    s.den32 = (float)((p98 - p2) + 1e-6);
  } else {
    s.mode = 2;
  }
  s.p2 = p2;
  s.p98 = p98;
  s.phase = PH_DONE;
}

template <int LEVEL, int PASS>
__global__ __launch_bounds__(kBlock) void k_sel_resolve(SelState* st, uint32_t* hist, int B) {
  __shared__ uint32_t sc[kBlock];
  __shared__ uint32_t res_bin[4], res_rem[4];
  __shared__ SelState s;
  const int b = blockIdx.x;
  if (b >= B) return;
  if (threadIdx.x == 0) s = st[b];
  __syncthreads();
  bool run;
  if (PASS == 0) run = LEVEL == 0 ? s.phase == PH_INIT : (s.phase == PH_PCT || s.phase == PH_MED);
  else run = LEVEL == 0 ? s.phase == PH_PCT2_INIT : s.phase == PH_PCT2;
  if (!run) return;
  __syncthreads();
  if (threadIdx.x == 0 && LEVEL == 0) {
    if (PASS == 0 && s.nonfinite_count != 0) {
      const uint32_t m = s.n - s.nan_count;
      if (m == 0) {                      // all-NaN: nanmedian is NaN, every value stays NaN
        s.has_med = 1;
        s.mode = 2;
        s.p2 = s.p98 = (double)__uint_as_float(0x7fc00000u);
        s.phase = PH_DONE;
      } else {
        const uint32_t h = m / 2;
        if (m & 1u) { s.rank[0] = s.rank[1] = h; s.med_ranks = 1; }
        else { s.rank[0] = h - 1; s.rank[1] = h; s.med_ranks = 2; }
        s.ntgt = 2;
        s.prefix[0] = s.prefix[1] = 0;
        s.phase = PH_MED;
      }
    } else {
      pct_targets(s);
      s.phase = PASS == 0 ? PH_PCT : PH_PCT2;
    }
    for (int i = 0; i < 4; ++i) s.slot[i] = 0;
    s.nslot = 1;
  }
  __syncthreads();
  if (s.phase == PH_DONE) {
    if (threadIdx.x == 0) st[b] = s;
    return;
  }
  uint32_t* gh = hist + (size_t)b * kSlots * kBins;
  const int nb = LEVEL == 2 ? 1024 : kBins;
  for (int t = 0; t < (int)s.ntgt; ++t) {
    if (threadIdx.x == 0) { res_bin[t] = 0; res_rem[t] = 0; }
    __syncthreads();
    find_bin(gh + s.slot[t] * kBins, nb, s.rank[t], sc, &res_bin[t], &res_rem[t]);
  }
  __syncthreads();
  // consumed histograms -> zero for the next level
  for (int i = threadIdx.x; i < (int)s.nslot * kBins; i += kBlock) gh[i] = 0;
  if (threadIdx.x == 0) {
    const int bits = LEVEL == 2 ? 10 : 11;
    for (int t = 0; t < (int)s.ntgt; ++t) {
      s.prefix[t] = (s.prefix[t] << bits) | res_bin[t];
      s.rank[t] = res_rem[t];
    }
    // distinct prefixes -> histogram slots for the next level
    s.nslot = 0;
    for (int t = 0; t < (int)s.ntgt; ++t) {
      int found = -1;
      for (int q = 0; q < (int)s.nslot; ++q) if (s.slot_prefix[q] == s.prefix[t]) found = q;
      if (found < 0) { found = (int)s.nslot; s.slot_prefix[s.nslot++] = s.prefix[t]; }
      s.slot[t] = (uint32_t)found;
    }
    if (LEVEL == 2) {
      if (s.phase == PH_MED) {
        const float a = key2f(s.prefix[0]);
        const float c = key2f(s.prefix[1]);
        s.med = s.med_ranks == 1 ? a : (a + c) / 2.0f;  // np.mean of the middle pair in float32
        s.has_med = 1;
        s.phase = PH_PCT2_INIT;
        if (isnan(s.med)) {  // e.g. median of {-inf, +inf}: the filled map has NaNs -> np.percentile is NaN
          s.mode = 2;
          s.p2 = s.p98 = (double)s.med;
          s.phase = PH_DONE;
        }
        s.kmin = 0xffffffffu;
        s.kmax = 0u;
        s.nslot = 1;
        s.slot_prefix[0] = 0;
      } else {
        finalize_pct(s);
      }
    }
    st[b] = s;
  }
}

struct Norm {
  int mode, invert;
  double p2, p98, den64, rden64;
  float lo32, hi32, den32;
};

__device__ __forceinline__ Norm load_norm(const SelState* S, int invert) {
  Norm nm;
  nm.mode = S->mode;
  nm.invert = invert;
  nm.p2 = S->p2;
  nm.p98 = S->p98;
  nm.den64 = S->den64;
  nm.rden64 = S->rden64;
  nm.lo32 = S->lo32;
  nm.hi32 = S->hi32;
  nm.den32 = S->den32;
  return nm;
}

// app.py:200-206 in the dtype numpy uses for the branch taken.
__device__ __forceinline__ double normalize(float val, const Norm& nm) {
  if (nm.mode == 0) {
    double d = (double)val;
    d = d < nm.p2 ? nm.p2 : d;          // np.clip -> min(max(x, lo), hi)
    d = d > nm.p98 ? nm.p98 : d;
    d = div_rn(d - nm.p2, nm.den64, nm.rden64);
    if (nm.invert) d = 1.0 - d;
    return d;
  }
  if (nm.mode == 1) {
    float f = val < nm.lo32 ? nm.lo32 : val;
    f = f > nm.hi32 ? nm.hi32 : f;
    f = (f - nm.lo32) / nm.den32;
    if (nm.invert) f = 1.0f - f;
    return (double)f;
  }
  return nm.invert ? 1.0 : 0.0;
}

struct Cam {
  double cx, cy, f, rf, scale;   // rf = RN(1 / f)
  int step, Wn, N;
};

__device__ __forceinline__ void project(double d, int v, int u, const Cam& c, float& x, float& y, float& z) {
  const double zd = d * c.scale;                       // app.py:233
  const double zz = zd != 0.0 ? zd : 1e-6;             // app.py:234-235
  x = (float)div_rn(((double)u - c.cx) * zz, c.f, c.rf);
  y = (float)div_rn(((double)v - c.cy) * zz, c.f, c.rf);
  z = (float)zd;
}

// Row-blocked unprojection: workgroup = image b x output point rows [r0, r1);
// thread = 4 consecutive points of a row (+1024 per column chunk).  Model rows
// staged in LDS (shared with the select sweeps' geometry); RGB of 4 pixels read
// as 12 contiguous bytes when step == 1; xyz stored as 3 x 16 B and rgb as
// 3 x 4 B per thread (a wave writes 3 KiB + 768 B contiguous).
template <bool kField>
__global__ __launch_bounds__(kBlock) void k_unproject(Geo g, const SelState* st, const double* field,
                                                      const uint8_t* img, int C, int B, Sweep sw, int invert,
                                                      Cam cam, float* xyz, uint8_t* rgb, SelState* stw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_u[];
  float* rows = reinterpret_cast<float*>(smem_u);
  __shared__ uint32_t red[6][4];
  int b, rb;
  map_rows(blockIdx.x, B, sw.nrb, b, rb);
  const SelState* S = st + b;
  const Norm nm = load_norm(S, invert);
  const bool fill = S->has_med != 0;
  const float med = S->med;
  const int Hn = cam.N / cam.Wn;
  const int r0 = sw.row0 + rb * sw.R;
  const int r1 = min(min(Hn, sw.row_end), r0 + sw.R);
  const int step = cam.step;
  const bool use_lds = !kField && sw.lds_rows > 0;
  int lo = 0;
  if (!kField) lo = stage_rows(g, b, r0 * step, (r1 - 1) * step + 1, rows, sw.lds_rows);
  __syncthreads();
  const bool vec_ok = (cam.N & 3) == 0 && (cam.Wn & 3) == 0;
  const bool rgb_vec = step == 1 && C == 3 && (g.W & 3) == 0;
  const size_t img_base = (size_t)b * g.H * g.W;
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int cb = 0; cb < cam.Wn; cb += 4 * kBlock) {
    const int ui0 = cb + threadIdx.x * 4;
    const int cnt = min(4, cam.Wn - ui0);
    if (cnt <= 0) continue;
    // column taps once per chunk
    Tap tx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) tx[j] = (!g.same && !kField && j < cnt) ? g.xt[(ui0 + j) * step] : Tap{0, -1, 1.f, 0.f};
    // prefetch the RGB of every row of the block (HBM latency overlaps the whole row loop)
    uint32_t q[kMaxRows][3];
    const bool rgbv = rgb_vec && cnt == 4;
    if (rgbv) {
#pragma unroll
      for (int k = 0; k < kMaxRows; ++k) {
        if (r0 + k < r1) {
          const uint32_t* p32 = reinterpret_cast<const uint32_t*>(img + (img_base + (size_t)(r0 + k) * g.W + ui0) * 3);
          q[k][0] = p32[0]; q[k][1] = p32[1]; q[k][2] = p32[2];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kMaxRows; ++k) {
      const int ri = r0 + k;
      if (ri >= r1) break;
      const int v = ri * step;
      const Tap ty = g.same ? Tap{0, 0, 1.f, 0.f} : g.yt[v];
      float px[4][3];
      uint8_t pc[4][3];
      if (rgbv) {
        const uint32_t w0 = q[k][0], w1 = q[k][1], w2 = q[k][2];
        const uint8_t bytes[12] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                                   (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24),
                                   (uint8_t)w2, (uint8_t)(w2 >> 8), (uint8_t)(w2 >> 16), (uint8_t)(w2 >> 24)};
#pragma unroll
        for (int j = 0; j < 4; ++j) { pc[j][0] = bytes[3 * j + 2]; pc[j][1] = bytes[3 * j + 1]; pc[j][2] = bytes[3 * j]; }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int u = (ui0 + (j < cnt ? j : 0)) * step;
          if (C >= 3) {
            const uint8_t* qq = img + (img_base + (size_t)v * g.W + u) * C;
            pc[j][0] = qq[2]; pc[j][1] = qq[1]; pc[j][2] = qq[0];
          } else {
            pc[j][0] = pc[j][1] = pc[j][2] = 128;
          }
        }
      }
      const float* rr0 = use_lds ? rows + (ty.i0 - lo) * g.dw : g.depth + ((size_t)b * g.dh + ty.i0) * g.dw;
      const float* rr1 = use_lds ? rows + (ty.i1 - lo) * g.dw : g.depth + ((size_t)b * g.dh + ty.i1) * g.dw;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < cnt) {
          const int u = (ui0 + j) * step;
          double d;
          if (kField) {
            d = field[img_base + (size_t)v * g.W + u];
          } else {
            float val;
            if (g.same) {
              val = g.depth[((size_t)b * g.dh + v) * g.dw + u];
            } else if (tx[j].i1 < 0) {
              val = rr0[tx[j].i0] * ty.w0 + rr1[tx[j].i0] * ty.w1;
            } else {
              const float h0 = rr0[tx[j].i0] * tx[j].w0 + rr0[tx[j].i1] * tx[j].w1;
              const float h1 = rr1[tx[j].i0] * tx[j].w0 + rr1[tx[j].i1] * tx[j].w1;
              val = h0 * ty.w0 + h1 * ty.w1;
            }
            if (fill && !isfinite(val)) val = med;
            d = normalize(val, nm);
          }
          project(d, v, u, cam, px[j][0], px[j][1], px[j][2]);
#pragma unroll
          for (int c = 0; c < 3; ++c) { mn[c] = fminf(mn[c], px[j][c]); mx[c] = fmaxf(mx[c], px[j][c]); }
        }
      }
      const size_t o = (size_t)b * cam.N + (size_t)ri * cam.Wn + ui0;
      if (vec_ok && cnt == 4) {
        float4* dst = reinterpret_cast<float4*>(xyz + o * 3);
        dst[0] = make_float4(px[0][0], px[0][1], px[0][2], px[1][0]);
        dst[1] = make_float4(px[1][1], px[1][2], px[2][0], px[2][1]);
        dst[2] = make_float4(px[2][2], px[3][0], px[3][1], px[3][2]);
        uint32_t* cd = reinterpret_cast<uint32_t*>(rgb + o * 3);
        cd[0] = pc[0][0] | (pc[0][1] << 8) | (pc[0][2] << 16) | (pc[1][0] << 24);
        cd[1] = pc[1][1] | (pc[1][2] << 8) | (pc[2][0] << 16) | (pc[2][1] << 24);
        cd[2] = pc[2][2] | (pc[3][0] << 8) | (pc[3][1] << 16) | (pc[3][2] << 24);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < cnt)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              xyz[(o + j) * 3 + c] = px[j][c];
              rgb[(o + j) * 3 + c] = pc[j][c];
            }
      }
    }
  }
  // per-image bbox: wave reduce -> LDS -> one atomic per block and component
  uint32_t kk[6];
  for (int k = 0; k < 3; ++k) {
    const bool any = mn[k] <= mx[k];
    kk[2 * k] = any ? f2key(mn[k]) : 0xffffffffu;
    kk[2 * k + 1] = any ? f2key(mx[k]) : 0u;
  }
  const int wid = threadIdx.x >> 6;
  for (int k = 0; k < 6; ++k) {
    uint32_t x = (k & 1) ? wave_max_u32(kk[k]) : wave_min_u32(kk[k]);
    if ((threadIdx.x & 63) == 0) red[k][wid] = x;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int k = threadIdx.x;
    uint32_t x = red[k][0];
    for (int w = 1; w < kBlock / 64; ++w) x = (k & 1) ? max(x, red[k][w]) : min(x, red[k][w]);
    uint32_t* dst = &stw[b].bbox_key[k];
    if (k & 1) { if (x) atomicMax(dst, x); }
    else { if (x != 0xffffffffu) atomicMin(dst, x); }
  }
}

__device__ __forceinline__ Tap xtap(const Geo& g, int u) {
  Tap t = make_tap(u, g.dw, g.sx);
  if (g.dw == 1) { t.i0 = 0; t.i1 = -1; t.w0 = 1.f; t.w1 = 0.f; }
  return t;
}
__device__ __forceinline__ Tap ytap(const Geo& g, int v) {
  Tap t = make_tap(v, g.dh, g.sy);
  if (t.i1 < 0) t.i1 = t.i0;
  return t;
}

// Fast unprojection (no smoothing, N % 4 == 0, ceil(W/step) % 4 == 0, 3 channels):
// every load is unconditional (indices clamped, only the stores are predicated) so
// the compiler never parks a wave on a divergent vmcnt(0); the RGB of both point
// groups a thread owns is in flight before any arithmetic; cv2 taps are recomputed
// in registers (no table loads).
template <int STEP>
__global__ __launch_bounds__(kBlock) void k_unproject_fast(Geo g, const SelState* st, const uint8_t* img, int B,
                                                           Sweep sw, int invert, Cam cam, float* xyz, uint8_t* rgb,
                                                           SelState* stw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_u[];
  float* rows = reinterpret_cast<float*>(smem_u);
  __shared__ uint32_t red[6][4];
  __shared__ float4 sx[kBlock / 64][192];
  __shared__ uint32_t sc[kBlock / 64][192];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int b, rb;
  map_rows(blockIdx.x, B, sw.nrb, b, rb);
  const SelState* S = st + b;
  const Norm nm = load_norm(S, invert);
  const bool fill = S->has_med != 0;
  const float med = S->med;
  const int Hn = cam.N / cam.Wn;
  const int r0 = sw.row0 + rb * sw.R;
  const int r1 = min(min(Hn, sw.row_end), r0 + sw.R);
  const bool use_lds = sw.lds_rows > 0 && !g.same;
  int lo = 0;
  if (use_lds) {
    lo = ytap(g, r0 * STEP).i0;
    const int hi = ytap(g, (r1 - 1) * STEP).i1;
    const int n = (hi - lo + 1) * g.dw;
    const float* src = g.depth + ((size_t)b * g.dh + lo) * g.dw;
    for (int i = threadIdx.x; i < n; i += kBlock) rows[i] = src[i];
  }
  __syncthreads();
  const int Wn4 = cam.Wn >> 2;
  const int G = (r1 - r0) * Wn4;
  const size_t img_base = (size_t)b * g.H * g.W;
  const float* dimg = g.depth + (size_t)b * g.dh * g.dw;
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  // groups of 4 points whose RGB a thread has in flight at once (3 dwords each at STEP 1)
  constexpr int kGroupsPerThread = STEP == 1 ? 4 : 2;
  for (int base = 0; base < G; base += kGroupsPerThread * kBlock) {
    int row[kGroupsPerThread], ui0[kGroupsPerThread];
    uint32_t q[kGroupsPerThread][4][3];
#pragma unroll
    for (int k = 0; k < kGroupsPerThread; ++k) {
      const int gi = min(base + k * kBlock + (int)threadIdx.x, G - 1);
      row[k] = r0 + gi / Wn4;
      ui0[k] = (gi - (row[k] - r0) * Wn4) * 4;
      const int v = row[k] * STEP;
      if (STEP == 1) {
        const uint32_t* p32 = reinterpret_cast<const uint32_t*>(img + (img_base + (size_t)v * g.W + ui0[k]) * 3);
        q[k][0][0] = p32[0]; q[k][0][1] = p32[1]; q[k][0][2] = p32[2];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint8_t* px = img + (img_base + (size_t)v * g.W + (ui0[k] + j) * STEP) * 3;
          q[k][j][0] = px[0]; q[k][j][1] = px[1]; q[k][j][2] = px[2];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kGroupsPerThread; ++k) {
      const int gidx = base + k * kBlock + (int)threadIdx.x;
      const int v = row[k] * STEP;
      uint32_t pc[4][3];   // [point][r,g,b] (source is BGR)
      if (STEP == 1) {
        const uint32_t w[3] = {q[k][0][0], q[k][0][1], q[k][0][2]};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int byte = 3 * j + (2 - c);
            pc[j][c] = (w[byte >> 2] >> (8 * (byte & 3))) & 0xffu;
          }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) { pc[j][0] = q[k][j][2]; pc[j][1] = q[k][j][1]; pc[j][2] = q[k][j][0]; }
      }
      const Tap ty = ytap(g, v);
      const float* rr0 = use_lds ? rows + (ty.i0 - lo) * g.dw : dimg + (size_t)ty.i0 * g.dw;
      const float* rr1 = use_lds ? rows + (ty.i1 - lo) * g.dw : dimg + (size_t)ty.i1 * g.dw;
      float px[4][3];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int u = (ui0[k] + j) * STEP;
        float val;
        if (g.same) {
          val = dimg[(size_t)v * g.dw + u];
        } else {
          const Tap tx = xtap(g, u);
          const int i1 = tx.i1 < 0 ? tx.i0 : tx.i1;
          const float a0 = rr0[tx.i0], a1 = rr0[i1], c0 = rr1[tx.i0], c1 = rr1[i1];
          const float h0 = tx.i1 < 0 ? a0 : a0 * tx.w0 + a1 * tx.w1;
          const float h1 = tx.i1 < 0 ? c0 : c0 * tx.w0 + c1 * tx.w1;
          val = h0 * ty.w0 + h1 * ty.w1;
        }
        if (fill && !isfinite(val)) val = med;
        project(normalize(val, nm), v, u, cam, px[j][0], px[j][1], px[j][2]);
      }
      if (gidx < G) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int c = 0; c < 3; ++c) { mn[c] = fminf(mn[c], px[j][c]); mx[c] = fmaxf(mx[c], px[j][c]); }
      }
      // The wave's 64 groups are 256 consecutive points: stage its 3 KB of xyz and 768 B of
      // rgb through LDS so every store instruction writes one contiguous 1 KB / 256 B run
      // (the direct per-lane 48 B / 12 B strided stores left 2/3 of each request empty).
      float4* wx = sx[wid];
      uint32_t* wc = sc[wid];
      wx[lane * 3 + 0] = make_float4(px[0][0], px[0][1], px[0][2], px[1][0]);
      wx[lane * 3 + 1] = make_float4(px[1][1], px[1][2], px[2][0], px[2][1]);
      wx[lane * 3 + 2] = make_float4(px[2][2], px[3][0], px[3][1], px[3][2]);
      wc[lane * 3 + 0] = pc[0][0] | (pc[0][1] << 8) | (pc[0][2] << 16) | (pc[1][0] << 24);
      wc[lane * 3 + 1] = pc[1][1] | (pc[1][2] << 8) | (pc[2][0] << 16) | (pc[2][1] << 24);
      wc[lane * 3 + 2] = pc[2][2] | (pc[3][0] << 8) | (pc[3][1] << 16) | (pc[3][2] << 24);
      __builtin_amdgcn_wave_barrier();
      const int wbase = base + k * kBlock + wid * 64;             // first group of this wave
      const size_t o = (size_t)b * cam.N + (size_t)r0 * cam.Wn + (size_t)wbase * 4;
      float4* dx = reinterpret_cast<float4*>(xyz + o * 3);
      uint32_t* dc = reinterpret_cast<uint32_t*>(rgb + o * 3);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int f = q * 64 + lane;
        if (wbase + f / 3 < G) {      // streamed once: non-temporal (no cache residency to keep)
          const float4 vx = wx[f];
          __builtin_nontemporal_store(vx.x, &dx[f].x);
          __builtin_nontemporal_store(vx.y, &dx[f].y);
          __builtin_nontemporal_store(vx.z, &dx[f].z);
          __builtin_nontemporal_store(vx.w, &dx[f].w);
          __builtin_nontemporal_store(wc[f], &dc[f]);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  uint32_t kk[6];
  for (int c = 0; c < 3; ++c) {
    const bool any = mn[c] <= mx[c];
    kk[2 * c] = any ? f2key(mn[c]) : 0xffffffffu;
    kk[2 * c + 1] = any ? f2key(mx[c]) : 0u;
  }
  for (int c = 0; c < 6; ++c) {
    uint32_t x = (c & 1) ? wave_max_u32(kk[c]) : wave_min_u32(kk[c]);
    if ((threadIdx.x & 63) == 0) red[c][wid] = x;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int c = threadIdx.x;
    uint32_t x = red[c][0];
    for (int w = 1; w < kBlock / 64; ++w) x = (c & 1) ? max(x, red[c][w]) : min(x, red[c][w]);
    uint32_t* dst = &stw[b].bbox_key[c];
    if (c & 1) { if (x) atomicMax(dst, x); }
    else { if (x != 0xffffffffu) atomicMin(dst, x); }
  }
}

// Smooth path (app.py:209-214): materialise the normalised field, blur, unproject.
__global__ void k_norm_field(Geo g, const SelState* st, int B, int invert, double* field) {
  const size_t n = (size_t)g.H * g.W;
  const size_t total = n * B;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / n);
    const int p = (int)(i - (size_t)b * n);
    const int v = p / g.W, u = p - v * g.W;
    const SelState* S = st + b;
    float val = sample(g, b, v, u);
    if (S->has_med && !isfinite(val)) val = S->med;
    field[i] = normalize(val, load_norm(S, invert));
  }
}

// cv2 borderInterpolate(BORDER_REFLECT_101), repeated reflection for kernels wider than the image
__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while ((unsigned)i >= (unsigned)n) i = i < 0 ? -i : 2 * (n - 1) - i;
  return i;
}

// Separable Gaussian taps of cv2.GaussianBlur(d, (k, k), 0) (getGaussianKernel, sigma 0):
// the fixed small-kernel tables for k <= 7, else sigma = 0.15 k + 0.35 sampled and normalised.
constexpr int kMaxBlur = 63;
struct BlurTaps {
  int k;
  double w[kMaxBlur];
};

// Tap-order accumulation (k taps, BORDER_REFLECT_101) in the branch dtype (float64 for
// mode 0, float32 with float32 taps otherwise).
template <bool kRows>
__global__ void k_blur(const double* src, double* dst, const SelState* st, int B, int H, int W, BlurTaps taps) {
  const size_t n = (size_t)H * W;
  const size_t total = n * B;
  const int r = taps.k / 2;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / n);
    const int p = (int)(i - (size_t)b * n);
    const int v = p / W, u = p - v * W;
    const double* s = src + (size_t)b * n;
    if (st[b].mode == 0) {
      double acc = 0.0;
      for (int t = 0; t < taps.k; ++t) {
        const double x = kRows ? s[(size_t)v * W + reflect101(u + t - r, W)] : s[(size_t)reflect101(v + t - r, H) * W + u];
        acc = acc + x * taps.w[t];
      }
      dst[i] = acc;
    } else {
      float acc = 0.f;
      for (int t = 0; t < taps.k; ++t) {
        const float x = (float)(kRows ? s[(size_t)v * W + reflect101(u + t - r, W)] : s[(size_t)reflect101(v + t - r, H) * W + u]);
        acc = acc + x * (float)taps.w[t];
      }
      dst[i] = (double)acc;
    }
  }
}

static BlurTaps gaussian_taps(int k) {
  BlurTaps t{};
  t.k = k;
  static const double small[4][7] = {{1.0},
                                     {0.25, 0.5, 0.25},
                                     {0.0625, 0.25, 0.375, 0.25, 0.0625},
                                     {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125}};
  if (k <= 7) {
    for (int i = 0; i < k; ++i) t.w[i] = small[k / 2][i];
    return t;
  }
  const double sigma = 0.15 * k + 0.35;                 // ((k - 1) * 0.5 - 1) * 0.3 + 0.8
  const double scale2x = -0.125 / (sigma * sigma);      // x below is 2 * (i - (k - 1) / 2)
  const int h = (k - 1) / 2;
  double v[kMaxBlur], sum = 0.0;
  for (int i = 0, x = 1 - k; i < h; ++i, x += 2) {
    v[i] = std::exp((double)(x * x) * scale2x);
    sum += v[i];
  }
  sum = sum * 2.0 + 1.0;
  const double mul = 1.0 / sum;
  for (int i = 0; i < h; ++i) t.w[i] = t.w[k - 1 - i] = v[i] * mul;
  t.w[h] = mul;
  return t;
}

__global__ void k_finalize(const SelState* st, int B, double* bbox, double* stats) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const SelState& s = st[b];
  if (bbox)
    for (int k = 0; k < 6; ++k) bbox[b * 6 + k] = (double)key2f(s.bbox_key[k]);
  if (stats) {
    stats[b * 4 + 0] = s.p2;
    stats[b * 4 + 1] = s.p98;
    stats[b * 4 + 2] = (double)s.mode;
    stats[b * 4 + 3] = s.has_med ? (double)s.med : (double)__uint_as_float(0x7fc00000u);
  }
}

// Depth preview colouring (create_depth_preview, app.py:124-172): the model-res depth
// after fill / p2-p98 normalise / invert, (d * 255).astype(uint8) in the branch's dtype,
// then a 256-entry BGR colour table (cv2.applyColorMap).
__global__ void k_preview(const float* depth, const SelState* st, int B, int n, int invert, const uint8_t* lut,
                          uint8_t* out) {
  __shared__ uint8_t tab[768];
  for (int i = threadIdx.x; i < 768; i += blockDim.x) tab[i] = lut[i];
  __syncthreads();
  const int64_t total = (int64_t)B * n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / n);
    const SelState* S = st + b;
    const Norm nm = load_norm(S, invert);
    float val = depth[i];
    if (S->has_med && !isfinite(val)) val = S->med;
    const double d = normalize(val, nm);
    const int q = nm.mode == 0 ? (int)(d * 255.0) : (int)((float)d * 255.0f);   // astype(uint8) truncates
    const int k = min(max(q, 0), 255) * 3;
    out[i * 3 + 0] = tab[k];
    out[i * 3 + 1] = tab[k + 1];
    out[i * 3 + 2] = tab[k + 2];
  }
}

__global__ void k_gather_stride(const float* xyz, const uint8_t* rgb, int64_t n, int64_t stride,
                                float* oxyz, float* orgb) {
  const int64_t cnt = (n + stride - 1) / stride;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = i * stride;
    for (int k = 0; k < 3; ++k) {
      oxyz[i * 3 + k] = xyz[s * 3 + k];
      orgb[i * 3 + k] = (float)rgb[s * 3 + k];
    }
  }
}

constexpr int kRowBudget = 31 * 1024;   // LDS bytes for the staged model-row window (+32 KiB hist < 64 KiB)

// Rows per workgroup so that the model-row window fits the LDS budget.
static Sweep plan_sweep(int rows_out, int step, int dh, int dw, int H, bool same, int target_rows, int row0 = 0,
                        int row1 = -1) {
  Sweep sw{};
  int cap_rows = same ? 0 : kRowBudget / (int)(sizeof(float) * dw);
  int R = target_rows;
  if (!same && cap_rows >= 3) {
    // model rows spanned by R output rows (image rows (R-1)*step apart): <= (R-1)*step*dh/H + 3
    while (R > 1 && (double)(R - 1) * step * dh / H + 3.0 > cap_rows) R /= 2;
  } else {
    cap_rows = 0;
  }
  sw.R = std::max(1, R);
  if (row1 < 0) row1 = rows_out;
  sw.row0 = row0;
  sw.row_end = row1;
  sw.nrb = std::max(1, (row1 - row0 + sw.R - 1) / sw.R);
  // allocate only the window R output rows can span (not the whole budget): occupancy
  if (cap_rows) cap_rows = std::min(cap_rows, (int)std::floor((double)(sw.R - 1) * step * dh / H) + 3);
  sw.lds_rows = cap_rows;
  return sw;
}

static size_t sweep_lds(const Sweep& sw, int dw) { return sw.lds_rows ? (size_t)sw.lds_rows * dw * sizeof(float) : 0; }

// Tile-parallel mode: the level-0 counters a sweep accumulates, out of / back into the
// per-image state, as int64 [4][B] = {nan counts, non-finite counts, min key, max key}
// (sum, sum, min, max across the bands).
__global__ void k_band_export(const SelState* st, int B, int64_t* ex) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    ex[b] = st[b].nan_count;
    ex[B + b] = st[b].nonfinite_count;
    ex[2 * B + b] = st[b].kmin;
    ex[3 * B + b] = st[b].kmax;
  }
}
__global__ void k_band_import(SelState* st, int B, const int64_t* ex) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    st[b].nan_count = (uint32_t)ex[b];
    st[b].nonfinite_count = (uint32_t)ex[B + b];
    st[b].kmin = (uint32_t)ex[2 * B + b];
    st[b].kmax = (uint32_t)ex[3 * B + b];
  }
}

struct Exchange {
  i2pc_exchange_fn fn;
  void* user;
  int64_t* ex;     // device int64 [4][B]
};

// Between a histogram sweep and its resolve, a band run hands the partial histograms (and,
// at level 0, the counters) to the caller's collective, which must leave the sums (min /
// max for the keys) over every band in place, ordered on `s`.
template <int LEVEL>
static int exchange(const Exchange* x, uint32_t* hist, SelState* st, int B, hipStream_t s) {
  if (!x || !x->fn) return I2PC_OK;
  if (LEVEL == 0) hipLaunchKernelGGL(k_band_export, dim3(1), dim3(64), 0, s, st, B, x->ex);
  if (x->fn(x->user, hist, (int64_t)kSlots * kBins * B, LEVEL == 0 ? x->ex : nullptr, B, s) != 0)
    return set_error(I2PC_ELAUNCH, "exchange callback failed at selection level %d", LEVEL);
  if (LEVEL == 0) hipLaunchKernelGGL(k_band_import, dim3(1), dim3(64), 0, s, st, B, x->ex);
  return I2PC_OK;
}

template <int PASS>
static int launch_select(const Geo& g, SelState* st, uint32_t* hist, int B, const Sweep& sw, hipStream_t s,
                         const Exchange* x = nullptr) {
  // level 0 histograms one slot (8 KB of LDS); levels 1-2 up to kSlots target prefixes
  const size_t lds0 = sizeof(uint32_t) * kBins + sweep_lds(sw, g.dw);
  const size_t lds = sizeof(uint32_t) * kSlots * kBins + sweep_lds(sw, g.dw);
  const dim3 grid(B * sw.nrb), block(kBlock);
  int rc;
  hipLaunchKernelGGL((k_sel_hist<0, PASS>), grid, block, lds0, s, g, st, hist, B, sw);
  if ((rc = exchange<0>(x, hist, st, B, s))) return rc;
  hipLaunchKernelGGL((k_sel_resolve<0, PASS>), dim3(B), block, 0, s, st, hist, B);
  hipLaunchKernelGGL((k_sel_hist<1, PASS>), grid, block, lds, s, g, st, hist, B, sw);
  if ((rc = exchange<1>(x, hist, st, B, s))) return rc;
  hipLaunchKernelGGL((k_sel_resolve<1, PASS>), dim3(B), block, 0, s, st, hist, B);
  hipLaunchKernelGGL((k_sel_hist<2, PASS>), grid, block, lds, s, g, st, hist, B, sw);
  if ((rc = exchange<2>(x, hist, st, B, s))) return rc;
  hipLaunchKernelGGL((k_sel_resolve<2, PASS>), dim3(B), block, 0, s, st, hist, B);
  return check_launch("select");
}

}  // namespace unproj
}  // namespace i2pc

using namespace i2pc;
using namespace i2pc::unproj;

// ---- profiling hook: HIP events around the unprojection kernel (bench.py's roofline)
namespace {
hipEvent_t g_prof_ev[2] = {nullptr, nullptr};
bool g_prof_on = false;
bool g_prof_recorded = false;
void prof_mark(int i, hipStream_t s) {
  if (!g_prof_on) return;
  (void)hipEventRecord(g_prof_ev[i], s);
  if (i == 1) g_prof_recorded = true;
}
}  // namespace

extern "C" int i2pc_profile_enable(int on) {
  clear_error();
  if (on && !g_prof_ev[0]) {
    for (auto& e : g_prof_ev)
      if (hipEventCreate(&e) != hipSuccess) return set_error(I2PC_ELAUNCH, "hipEventCreate failed");
  }
  g_prof_on = on != 0;
  g_prof_recorded = false;
  return I2PC_OK;
}

extern "C" float i2pc_profile_unproject_ms(void) {
  if (!g_prof_recorded) return -1.f;
  float ms = -1.f;
  if (hipEventSynchronize(g_prof_ev[1]) != hipSuccess) return -1.f;
  if (hipEventElapsedTime(&ms, g_prof_ev[0], g_prof_ev[1]) != hipSuccess) return -1.f;
  return ms;
}

extern "C" size_t i2pc_unproject_workspace_bytes(int batch, int img_h, int img_w, int smooth) {
  if (batch <= 0 || img_h <= 0 || img_w <= 0) return 0;
  return layout(batch, img_h, img_w, smooth).total;
}

// Band [row0, row1) of the image rows (the whole image when row0 = 0, row1 = img_h);
// `image`, `xyz`, `rgb` address the full image (band runs pass offset pointers).
static int run_unproject(const float* depth, int dep_h, int dep_w, const uint8_t* image, int channels,
                         int batch, int img_h, int img_w, const i2pc_unproject_params* params,
                         float* xyz, uint8_t* rgb, double* bbox, double* stats,
                         void* workspace, size_t workspace_bytes, void* stream, int row0, int row1,
                         const Exchange* xch) {
  I2PC_REQUIRE(params != nullptr, "params is NULL");
  I2PC_REQUIRE(depth && image && xyz && rgb && workspace, "NULL device pointer");
  I2PC_REQUIRE(batch > 0 && img_h > 0 && img_w > 0 && dep_h > 0 && dep_w > 0, "empty shape");
  I2PC_REQUIRE(channels >= 1 && channels <= 4, "channels must be 1..4");
  const int step = params->step;
  I2PC_REQUIRE(step == 1 || step == 2 || step == 4, "step must be 1, 2 or 4 (low/medium/high)");
  I2PC_REQUIRE((int64_t)img_h * img_w < (1ll << 31), "image too large");
  const int blur_k = params->smooth_ksize < 3 ? 3 : params->smooth_ksize / 2 * 2 + 1;   // app.py:211
  if (params->smooth)
    I2PC_REQUIRE(blur_k <= kMaxBlur, "smooth_ksize -> kernel %d: at most %d taps", blur_k, kMaxBlur);
  const Layout L = layout(batch, img_h, img_w, params->smooth);
  if (workspace_bytes < L.total) return set_error(I2PC_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, L.total);
  hipStream_t s = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  SelState* st = reinterpret_cast<SelState*>(ws + L.state);
  uint32_t* hist = reinterpret_cast<uint32_t*>(ws + L.hist);
  Tap* xt = reinterpret_cast<Tap*>(ws + L.xtab);
  Tap* yt = reinterpret_cast<Tap*>(ws + L.ytab);

  if (hipMemsetAsync(hist, 0, sizeof(uint32_t) * kSlots * kBins * (size_t)batch, s) != hipSuccess)
    return set_error(I2PC_ELAUNCH, "memset failed");
  const int n = img_h * img_w;
  const int init_threads = std::max(std::max(batch, img_h), img_w);
  hipLaunchKernelGGL(k_init, dim3((init_threads + 255) / 256), dim3(256), 0, s, st, batch, n, xt, yt, dep_h, dep_w, img_h, img_w,
                     cv_scale(dep_w, img_w), cv_scale(dep_h, img_h));

  Geo g{depth, dep_h, dep_w, img_h, img_w, xt, yt, (dep_h == img_h && dep_w == img_w) ? 1 : 0,
        cv_scale(dep_w, img_w), cv_scale(dep_h, img_h)};
  // selection sweeps: I2PC_SEL_PTS points per workgroup (default 8 rows of a 1024-wide image)
  // (measured r02, B = 32 x 1024^2: 4096 pts 476 us, 8192 462 us, 16384 505 us, 32768 598 us per call)
  static const int sel_pts = [] { const char* e = getenv("I2PC_SEL_PTS"); return e ? atoi(e) : 8192; }();
  const int sel_rows = std::max(1, std::min(64, (sel_pts + img_w - 1) / img_w));
  const Sweep ssel = plan_sweep(img_h, 1, dep_h, dep_w, img_h, g.same != 0, sel_rows, row0, row1);
  Exchange xb = xch ? *xch : Exchange{nullptr, nullptr, nullptr};
  xb.ex = reinterpret_cast<int64_t*>(ws + L.ex);
  int rc = launch_select<0>(g, st, hist, batch, ssel, s, xch ? &xb : nullptr);
  if (rc) return rc;
  rc = launch_select<1>(g, st, hist, batch, ssel, s, xch ? &xb : nullptr);
  if (rc) return rc;

  Cam cam;
  cam.cx = img_w / 2.0;
  cam.cy = img_h / 2.0;
  const double fov = params->fov_deg;
  if (fov > 0) {  // app.py:220-221 (NaN compares false -> else branch)
    cam.f = (img_w / 2.0) / std::tan((fov * (3.141592653589793 / 180.0)) / 2.0);
  } else {
    cam.f = (double)std::max(img_w, img_h) * 1.2;     // app.py:223
  }
  cam.rf = 1.0 / cam.f;
  cam.scale = params->depth_scale;
  cam.step = step;
  cam.Wn = (img_w + step - 1) / step;
  const int Hn = (img_h + step - 1) / step;
  cam.N = cam.Wn * Hn;
  const int unp_rows = std::max(1, std::min(kMaxRows, (4 * 1024 + cam.Wn - 1) / cam.Wn));
  const int prow0 = row0 / step, prow1 = (row1 + step - 1) / step;   // point rows of the band
  const Sweep sunp = plan_sweep(Hn, step, dep_h, dep_w, img_h, g.same != 0, unp_rows, prow0, prow1);
  const size_t unp_lds = sweep_lds(sunp, dep_w);
  const double* field = nullptr;
  if (params->smooth) {
    double* f0 = reinterpret_cast<double*>(ws + L.field);
    double* f1 = reinterpret_cast<double*>(ws + L.tmp);
    const int nb = 2048;
    hipLaunchKernelGGL(k_norm_field, dim3(nb), dim3(256), 0, s, g, st, batch, params->invert, f0);
    const BlurTaps taps = gaussian_taps(blur_k);
    hipLaunchKernelGGL((k_blur<true>), dim3(nb), dim3(256), 0, s, f0, f1, st, batch, img_h, img_w, taps);
    hipLaunchKernelGGL((k_blur<false>), dim3(nb), dim3(256), 0, s, f1, f0, st, batch, img_h, img_w, taps);
    field = f0;
    hipLaunchKernelGGL((k_unproject<true>), dim3(batch * sunp.nrb), dim3(kBlock), 0, s, g, st, field, image,
                       channels, batch, sunp, params->invert, cam, xyz, rgb, st);
  } else if (channels == 3 && cam.N % 4 == 0 && cam.Wn % 4 == 0) {
    // 8 rows of 1024 points (or the equivalent) per workgroup
    static const int pts_per_wg = [] { const char* e = getenv("I2PC_UNP_PTS"); return e ? atoi(e) : 8192; }();
    const int fast_rows = std::max(1, std::min(16, (pts_per_wg + cam.Wn - 1) / cam.Wn));
    const Sweep sf = plan_sweep(Hn, step, dep_h, dep_w, img_h, g.same != 0, fast_rows, prow0, prow1);
    const size_t lf = sweep_lds(sf, dep_w);
    const dim3 grid(batch * sf.nrb), block(kBlock);
    prof_mark(0, s);
    if (step == 1)
      hipLaunchKernelGGL((k_unproject_fast<1>), grid, block, lf, s, g, st, image, batch, sf, params->invert, cam, xyz, rgb, st);
    else if (step == 2)
      hipLaunchKernelGGL((k_unproject_fast<2>), grid, block, lf, s, g, st, image, batch, sf, params->invert, cam, xyz, rgb, st);
    else
      hipLaunchKernelGGL((k_unproject_fast<4>), grid, block, lf, s, g, st, image, batch, sf, params->invert, cam, xyz, rgb, st);
    prof_mark(1, s);
  } else {
    hipLaunchKernelGGL((k_unproject<false>), dim3(batch * sunp.nrb), dim3(kBlock), unp_lds, s, g, st, field, image,
                       channels, batch, sunp, params->invert, cam, xyz, rgb, st);
  }
  hipLaunchKernelGGL(k_finalize, dim3((batch + 63) / 64), dim3(64), 0, s, st, batch, bbox, stats);
  return check_launch("unproject");
}

extern "C" int i2pc_unproject(const float* depth, int dep_h, int dep_w, const uint8_t* image, int channels,
                              int batch, int img_h, int img_w, const i2pc_unproject_params* params,
                              float* xyz, uint8_t* rgb, double* bbox, double* stats,
                              void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  return run_unproject(depth, dep_h, dep_w, image, channels, batch, img_h, img_w, params, xyz, rgb, bbox, stats,
                       workspace, workspace_bytes, stream, 0, img_h, nullptr);
}

extern "C" int i2pc_unproject_band(const float* depth, int dep_h, int dep_w, const uint8_t* image_band, int channels,
                                   int img_h, int img_w, int row0, int row1, const i2pc_unproject_params* params,
                                   float* xyz_band, uint8_t* rgb_band, double* bbox, double* stats,
                                   void* workspace, size_t workspace_bytes, i2pc_exchange_fn exchange_fn,
                                   void* user, void* stream) {
  clear_error();
  I2PC_REQUIRE(params != nullptr, "params is NULL");
  I2PC_REQUIRE(image_band && xyz_band && rgb_band, "NULL device pointer");
  I2PC_REQUIRE(img_h > 0 && img_w > 0 && channels >= 1 && channels <= 4, "bad image shape");
  const int step = params->step;
  I2PC_REQUIRE(step == 1 || step == 2 || step == 4, "step must be 1, 2 or 4 (low/medium/high)");
  I2PC_REQUIRE(0 <= row0 && row0 < row1 && row1 <= img_h, "band rows [%d, %d) outside [0, %d)", row0, row1, img_h);
  I2PC_REQUIRE(row0 % step == 0 && (row1 % step == 0 || row1 == img_h),
               "band rows must start (and end, unless at the bottom) on a multiple of the step %d", step);
  if (params->smooth) return set_error(I2PC_EUNSUPPORTED, "smooth_depth blurs across bands: not in tile-parallel mode");
  // the kernels address the full image: shift the band buffers back to row 0
  const int Wn = (img_w + step - 1) / step;
  const uint8_t* image = image_band - (ptrdiff_t)row0 * img_w * channels;
  float* xyz = xyz_band - (ptrdiff_t)(row0 / step) * Wn * 3;
  uint8_t* rgb = rgb_band - (ptrdiff_t)(row0 / step) * Wn * 3;
  const Exchange x{exchange_fn, user, nullptr};
  return run_unproject(depth, dep_h, dep_w, image, channels, 1, img_h, img_w, params, xyz, rgb, bbox, stats,
                       workspace, workspace_bytes, stream, row0, row1, exchange_fn ? &x : nullptr);
}

extern "C" int i2pc_gather_stride(const float* xyz, const uint8_t* rgb, int64_t n, int64_t stride,
                                  float* out_xyz, float* out_rgb, void* stream) {
  clear_error();
  I2PC_REQUIRE(xyz && rgb && out_xyz && out_rgb, "NULL device pointer");
  I2PC_REQUIRE(n > 0 && stride > 0, "n and stride must be positive");
  const int64_t cnt = (n + stride - 1) / stride;
  const int blocks = (int)std::min<int64_t>((cnt + 255) / 256, 4096);
  hipLaunchKernelGGL(k_gather_stride, dim3(blocks), dim3(256), 0, as_stream(stream), xyz, rgb, n, stride, out_xyz, out_rgb);
  return check_launch("gather_stride");
}

extern "C" int i2pc_depth_preview(const float* depth, int batch, int h, int w, int invert, const uint8_t* lut_bgr,
                                  uint8_t* out_bgr, double* stats, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  clear_error();
  I2PC_REQUIRE(depth && lut_bgr && out_bgr && workspace, "NULL device pointer");
  I2PC_REQUIRE(batch > 0 && h > 0 && w > 0, "empty shape");
  I2PC_REQUIRE((int64_t)h * w < (1ll << 31), "depth map too large");
  const Layout L = layout(batch, h, w, 0);
  if (workspace_bytes < L.total) return set_error(I2PC_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, L.total);
  hipStream_t s = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  SelState* st = reinterpret_cast<SelState*>(ws + L.state);
  uint32_t* hist = reinterpret_cast<uint32_t*>(ws + L.hist);
  Tap* xt = reinterpret_cast<Tap*>(ws + L.xtab);
  Tap* yt = reinterpret_cast<Tap*>(ws + L.ytab);
  if (hipMemsetAsync(hist, 0, sizeof(uint32_t) * kSlots * kBins * (size_t)batch, s) != hipSuccess)
    return set_error(I2PC_ELAUNCH, "memset failed");
  const int n = h * w;
  const int init_threads = std::max(std::max(batch, h), w);
  hipLaunchKernelGGL(k_init, dim3((init_threads + 255) / 256), dim3(256), 0, s, st, batch, n, xt, yt, h, w, h, w, 1.0, 1.0);
  Geo g{depth, h, w, h, w, xt, yt, 1, 1.0, 1.0};
  const int sel_rows = std::max(1, std::min(16, (8 * 1024 + w - 1) / w));
  const Sweep ssel = plan_sweep(h, 1, h, w, h, true, sel_rows);
  int rc = launch_select<0>(g, st, hist, batch, ssel, s);
  if (rc) return rc;
  rc = launch_select<1>(g, st, hist, batch, ssel, s);
  if (rc) return rc;
  const int64_t total = (int64_t)batch * n;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_preview, dim3(blocks), dim3(256), 0, s, depth, st, batch, n, invert ? 1 : 0, lut_bgr, out_bgr);
  if (stats) hipLaunchKernelGGL(k_finalize, dim3((batch + 63) / 64), dim3(64), 0, s, st, batch, nullptr, stats);
  return check_launch("depth_preview");
}

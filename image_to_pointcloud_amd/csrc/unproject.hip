// Batched depth -> (x, y, z, rgb) back-projection for gfx950 (MI355X).
//
// Replaces backend/app.py:174-250 (depth_to_point_cloud) and the bounds of
// generate_gis_metadata (app.py:393-400) for a whole batch of images.
//
// Pipeline per call (all stream-ordered, graph-capturable, fixed launch list):
//   k_prepare         per-image selection state, cv2 INTER_LINEAR tap tables,
//                     zeroed histograms, model-map key range partials
//   k_model_hist / k_window   the model map's level-0 histogram -> windows around
//                     its p2 / p98 whose full-resolution keys the first sweep compacts
//   k_sweep/k_resolve x3 levels   exact order statistics of the full-resolution
//                     depth (recomputed on the fly from the model-resolution map,
//                     which stays L2-resident): the p2/p98 ranks of np.percentile
//                     (app.py:197) by interval narrowing -- usually a histogram
//                     sweep, a compaction sweep and a no-op third level
//   k_sel_slow        maps holding NaN/Inf only (np.nanmedian fill, app.py:194-196):
//                     the whole selection of such an image in one workgroup
//   [k_norm_field, k_blur<rows>, k_blur<cols>]  only when smooth=True (app.py:209-214), any odd k
//   k_unproject       normalise (fp64 / fp32 / constant branch exactly as
//                     numpy evaluates app.py:198-206), pinhole back-projection in
//                     Python-double semantics (app.py:219-238), RGB gather
//                     (app.py:239-244), per-image bbox via wave reductions
//   k_finalize        bbox / stats to float64
//
// Selection: see the "selection" section (linear key bins over the model map's range,
// run-length aggregated LDS histograms, candidate compaction).
// Arithmetic is bit-faithful: no FMA contraction in this file.
#include "common.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <cstring>
#include <cmath>

#pragma clang fp contract(off)

namespace i2pc {
namespace unproj {

constexpr int kSlots = 4;
constexpr int kMaxTgt = 10;  // p2 / p98 ranks (4); with NaN / Inf also their shifted twins (4) + the median (2)
// the selection from scratch: per image a level-0 histogram (top 11 key bits), kMaxTgt level-1
// histograms (next 11 bits) and kMaxTgt level-2 histograms (last 10 bits)
constexpr int kScrL1 = 2048, kScrL2 = kScrL1 + kMaxTgt * 2048, kScrWords = kScrL2 + kMaxTgt * 1024;
constexpr int kBins = 2048;
constexpr int kBlock = 256;
constexpr int kMaxRows = 4;   // unprojection rows per workgroup (register-prefetched RGB)
constexpr int kSlowBlock = 1024;
constexpr int kRangeChunks = 32;         // k_prepare workgroups per image, at least (range_chunks)
constexpr int kSampleChunks = 8;          // k_model_hist workgroups (partial sample histograms) per image, at least
constexpr int kMaxSampleChunks = 256;     // ... at most (large images: up to ~1 M samples, 4 K per workgroup)
constexpr int kSamplesPerChunk = 8192;    // ~8 per thread: one batch of loads in flight, then the LDS adds
// (4096 when the batch has too few images to fill the chip: the C4 panorama 25 -> 19.5 us;
// with 32 images the extra workgroups' histogram atomics cost more than they hide, 17 -> 27 us)
constexpr int kHistBlock = 1024;          // k_model_hist: threads per (image, chunk) workgroup (~8 samples each)
// Level 0 bins values (one bin ~ up to 2^31 keys near 0); levels 1-3 bin keys 2048 ways each:
// 2^31 -> 2^20 -> 2^9 -> 1 key, so the last level always resolves.
constexpr int kLastLevel = 3;
constexpr int kLdsCand = 10240;  // candidate keys a resolve keeps in LDS
constexpr int kWinKeys = 6144;   // expected full-resolution keys per level-0 window
constexpr int kTileW = 1024;     // selection sweep column tile (4 columns per thread)
constexpr int kSlotWords = kBins / 2;   // sweep LDS per slot: 2048 packed 16-bit counts or 1024 staged keys
constexpr int kHrowBudget = 40 * 1024;   // LDS bytes of staged + horizontally interpolated model rows
constexpr int kStageW = 1024;            // k_sweep_w: window keys a workgroup stages in LDS per window
constexpr int kWaveBuf = kStageW / 4;     // ... per wave (4 waves)
constexpr int kMaxSelRows = 64;          // k_sweep_w: output rows per workgroup at most
// window-selection band runs (C4): after the window sweep each band bins its window keys into
// kBins fine bins per window (all-reduced), then hands over only the keys of each target's fine
// bin: per target slot its count, min / max key and up to kPick keys (the all-gather)
constexpr int kPick = 1024;
constexpr int kPickWords = 3 + kPick;
constexpr int kBandWords = kMaxTgt * kPickWords;
constexpr int kBandEx = 8;               // row length of the window exchange's int64 [4][8] counters
// k_sweep_w's per-workgroup "finite keys below window w" counts go to kBelowSlots slots per image
// (workgroup i -> slot i % kBelowSlots) instead of one counter: a single large image (C4) had
// its 2048 workgroups' atomics on the same three words
constexpr int kBelowSlots = 64;
constexpr int kMaxBandRanks = 256;

// PH_INIT: level-0 sweep pending; PH_SEL: targets being narrowed; PH_SLOW: handed to
// k_sel_slow (non-finite map); PH_DONE: p2 / p98 / mode final.
// PH_SCR1 / PH_SCR2: the selection from scratch between its grid-wide radix levels (k_sel_slow ->
// k_scratch<1> -> k_scratch<2>)
constexpr uint32_t kLevelScratch = 16;   // SelState.level of an image selected from scratch (k_sel_slow)
enum Phase : uint32_t { PH_INIT = 0, PH_SEL = 1, PH_SLOW = 2, PH_SCR1 = 3, PH_SCR2 = 4, PH_DONE = 5 };
enum SlotMode : uint32_t { SM_HIST = 0, SM_COMPACT = 1 };
constexpr uint32_t kNoSlot = 0xffffffffu;

struct Tap {
  int i0, i1;     // i1 < 0: single tap (cv2 HResizeLinear right border copies S[sx])
  float w0, w1;
};

struct alignas(16) SelState {
  uint32_t phase;
  uint32_t n;              // pixels per image
  uint32_t nan_count;      // NaN / non-finite pixel counts (band exchange rows 0-1)
  uint32_t nonfinite_count;
  uint32_t kmin, kmax;     // ordered keys: min / max over the image (level-0 sweep)
  uint32_t rlo, rhi;       // finite key range of the model-resolution map (k_prepare / k_model_hist)
  uint32_t ntgt, nslot, nwin, fill;   // fill: NaN / Inf present (nanmedian fill targets)
  uint32_t wbin[6];        // level-0 window w = level-0 bins [wbin[2w], wbin[2w+1]] (k_window)
  uint32_t ninf_neg, ninf_pos;   // -inf / +inf pixel counts (level-0 sweep)
  uint32_t rank[kMaxTgt];  // remaining rank of target t inside its key interval
  uint32_t tlo[kMaxTgt], thi[kMaxTgt];   // key interval holding target t (tlo == thi: resolved)
  uint32_t tslot[kMaxTgt]; // slot target t is swept in next (kNoSlot: resolved)
  uint32_t slo[4], shi[4]; // key interval of slot q
  uint32_t smult[4];       // bin multiplier of slot q (0: one key per bin)
  uint32_t smode[4];       // SM_HIST / SM_COMPACT
  uint32_t ccount[4];      // candidate keys appended to slot q by a compaction sweep
  uint32_t med_ranks;      // 1 = odd count (one rank), 2 = even
  uint32_t has_med;
  float med;
  int32_t mode;            // 0: float64 branch, 1: float32 min/max branch, 2: constant
  uint32_t err;
  uint32_t level;          // last selection level that worked on the image (diagnostics)
  double p2, p98, den64;
  float lo32, hi32, den32, pad2;
  uint32_t bbox_key[6];
  uint32_t pad3[2];
  double rden64;           // RN(1 / den64): quotient seed for div_rn
  double pad4;
  // window-only selection (k_sweep_w / k_resolve_w): per level-0 window w the finite keys below it,
  // and for its end bins when k_window flagged them as spikes (wspike bit 0: first bin, bit 1:
  // last bin; such a bin is counted with its min / max key instead of compacted)
  uint32_t wspike[3];
  uint32_t wbelow[3];
  uint32_t wcntF[3], wminF[3], wmaxF[3];
  uint32_t wcntL[3], wminL[3], wmaxL[3];
  // window w as values (k_window): finite values < wvlo[w] lie below it, values in [wvlo, wvhi]
  // inside; a spike first bin ends at wvF[w], a spike last bin starts at wvL[w]
  float wvlo[3], wvhi[3], wvF[3], wvL[3];
  uint32_t twin[kMaxTgt];  // window-selection band runs: the window of target t's fine bin
};
static_assert(sizeof(SelState) == 624, "tools/sel_diag.py mirrors this layout");

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
  size_t state, hist, cand, rpart, xtab, ytab, trig, ex, mhist, gsend, grecv, wpart, slow, scr, field, tmp, total;
  uint32_t cap;   // candidate keys per slot and image (compaction sweeps)
};

// Candidate capacity per target interval: a level-0 bin holds ~n / 2048 keys on average, so
// n / 64 leaves a 32x margin for dense bins before the slower histogram level is taken.
static uint32_t cand_cap(int64_t n) {
  return (uint32_t)std::min<int64_t>(1 << 20, std::max<int64_t>(4096, n / 64)) / 256 * 256;   // DMA-able slots
}

// nranks > 0: a window-selection band run's all-gather buffers (send: one band's
// kBandWords, receive: nranks of them; the fine histograms use the level histograms' slots)
// The full-resolution sample k_model_hist bins: a jittered lattice of stride `stride` (ns
// points), nch partial histograms.  64 K points for images up to 2 M pixels; larger images
// sample n / 32 (at most ~1 M points), so the windows' sampling noise -- n / sqrt(ns) keys --
// stays a few tens of thousands of keys (an 8192 x 4096 panorama: ~1.1 M points).
struct SamplePlan {
  int stride, ns, nch;
};
static SamplePlan sample_plan(int H, int W, int B) {
  const double n = (double)H * W;
  const double target = std::min(1048576.0, std::max(65536.0, n / 32.0));
  SamplePlan sp;
  sp.stride = std::max(1, (int)std::sqrt(n / target));
  sp.ns = ((H + sp.stride - 1) / sp.stride) * ((W + sp.stride - 1) / sp.stride);
  const int spc = (int64_t)B * ((sp.ns + kSamplesPerChunk - 1) / kSamplesPerChunk) >= 256 ? kSamplesPerChunk
                                                                                        : kSamplesPerChunk / 2;
  sp.nch = std::min(kMaxSampleChunks, std::max(kSampleChunks, (sp.ns + spc - 1) / spc));
  return sp;
}

// k_prepare's workgroups per image (the model map's key-range partials): 32, more for small
// batches so a single large image still spreads over the chip
static int range_chunks(int B) { return std::min(256, std::max(kRangeChunks, 256 / std::max(B, 1))); }

static Layout layout(int B, int H, int W, int smooth, int nranks = 0) {
  Layout L{};
  size_t off = 0;
  L.cap = cand_cap((int64_t)H * W);
  L.state = off; off = align_up(off + sizeof(SelState) * (size_t)B, 256);
  L.hist = off;  off = align_up(off + sizeof(uint32_t) * kSlots * kBins * (size_t)B, 256);
  L.cand = off;  off = align_up(off + sizeof(uint32_t) * kSlots * (size_t)L.cap * B, 256);
  L.rpart = off; off = align_up(off + sizeof(uint32_t) * 2 * range_chunks(B) * (size_t)B, 256);
  L.xtab = off;  off = align_up(off + sizeof(Tap) * (size_t)W, 256);
  L.ytab = off;  off = align_up(off + sizeof(Tap) * (size_t)H, 256);
  L.trig = off;  off = align_up(off + sizeof(double) * 2 * ((size_t)W + H), 256);
  L.ex = off;    off = align_up(off + sizeof(int64_t) * 4 * (size_t)std::max(B, kBandEx), 256);
  L.mhist = off; off = align_up(off + sizeof(uint32_t) * kBins * (size_t)B, 256);
  // (B = 1: also the single-image path's local band chain, run_unproject)
  L.gsend = off; off = align_up(off + (nranks > 0 || B == 1 ? sizeof(uint32_t) * kBandWords : 0), 256);
  L.grecv = off; off = align_up(off + sizeof(uint32_t) * kBandWords * (size_t)std::max(nranks, 0), 256);
  L.wpart = off; off = align_up(off + sizeof(uint32_t) * kBelowSlots * 4 * (size_t)B, 256);
  L.slow = off;  off = align_up(off + sizeof(uint32_t) * 8 * (size_t)B, 256);   // k_sel_slow's ticket, range, counts
  L.scr = off;   off = align_up(off + sizeof(uint32_t) * kScrWords * (size_t)B, 256);   // from-scratch histograms
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

// cv2 taps of output column u / row v (the vertical pass always uses two rows: the second
// clamps to the last row) -- as k_prepare's tables
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

// ---------------------------------------------------------------- selection
//
// Exact p2 / p98 ranks of the full-resolution map (np.percentile, app.py:197) by narrowing
// key intervals.  A key is the order-preserving 32-bit image of a float (f2key), so every
// order statistic is a key, and a monotone map key -> bin turns counting into selection:
//   level 0  bins every key linearly over the finite key range of the MODEL-resolution map
//            (k_prepare; the bilinear resize stays within it up to rounding, keys outside
//            clamp to the end bins) -> the bin of each target rank + its rank inside it;
//   level 1  keys inside a target's bin interval are binned again (2048 finer bins), or --
//            when the bin holds at most `cap` keys, the usual case -- appended to a
//            candidate list, from which the resolve selects the exact key;
//   level 2  the same again (a level-1 bin spans at most 1024 keys: one key per bin).
// So a typical call sweeps the image twice (histogram, compaction).  The histogram adds are
// run-length aggregated per thread: a thread walks down its columns, consecutive keys of a
// smooth map fall in the same bin, and one LDS atomic carries the run.
// Non-finite maps (the nanmedian fill of app.py:194-196) go to k_sel_slow, which redoes the
// whole selection of such an image in one workgroup.

// Linear bins over a key interval starting at lo: bin = floor(d * kBins / span) for
// d = key - lo, as umulhi(d, mult) with mult = floor(kBins * 2^32 / span) (mult = 0 when
// span <= kBins: one key per bin).  Keys below lo go to bin 0, above the span to the last.
__host__ __device__ inline uint32_t bin_mult(uint32_t lo, uint32_t hi) {
  const uint64_t span = (uint64_t)hi - lo + 1;
  return span <= (uint64_t)kBins ? 0u : (uint32_t)(((uint64_t)kBins << 32) / span);
}
__device__ __forceinline__ uint32_t bin_of(uint32_t key, uint32_t lo, uint32_t mult) {
  const uint32_t d = key > lo ? key - lo : 0u;
  const uint32_t bn = mult ? __umulhi(d, mult) : d;
  return min(bn, (uint32_t)kBins - 1);
}
// key interval of bin bn (smallest offset of a bin: ceil(bn * 2^32 / mult)), clipped to [clo, chi]
__device__ inline void bin_interval(uint32_t bn, uint32_t lo, uint32_t mult, uint32_t clo, uint32_t chi,
                                    uint32_t& a, uint32_t& z) {
  auto first = [&](uint64_t k) -> uint64_t { return mult ? ((k << 32) + mult - 1) / mult : k; };
  uint64_t A = bn == 0 ? 0ull : (uint64_t)lo + first(bn);
  uint64_t Z = bn == (uint32_t)kBins - 1 ? 0xffffffffull : (uint64_t)lo + first((uint64_t)bn + 1) - 1;
  A = A < clo ? (uint64_t)clo : A;
  Z = Z > chi ? (uint64_t)chi : Z;
  a = (uint32_t)A;
  z = (uint32_t)(Z < A ? A : Z);
}
// Level 0 bins VALUES linearly over the model map's finite range [lo, hi]:
// bin = (v - lo) * 2048 / (hi - lo) in float32, clamped.  Float subtraction and multiplication
// round monotonically, so the map is monotone in the value -- hence in the key -- and each bin
// is a key interval (found by bisection, vbin_interval).  Linear-in-value bins keep ~n/2048 keys
// per bin for depth-like data; linear-in-key bins would give most bins to the binades near 0
// (a map with a few zero pixels puts 96 % of its key range below the smallest real depth).
struct VBins {
  float lo, inv;
};
__device__ __forceinline__ VBins level0_vbins(uint32_t rlo, uint32_t rhi) {
  VBins vb{0.f, 0.f};
  if (rlo <= rhi) {
    vb.lo = key2f(rlo);
    const float span = key2f(rhi) - vb.lo;
    vb.inv = (span > 0.f && span < INFINITY) ? (float)(kBins - 1) / span : 0.f;
  }
  return vb;
}
// bin 0 holds the values <= the model map's minimum -- usually one key: the exact zeros a
// network's final ReLU leaves are a spike no candidate list could hold, resolved here at once;
// bins 1..2047 split (minimum, maximum] linearly
__device__ __forceinline__ uint32_t vbin(float v, const VBins& vb) {
  if (!(v > vb.lo)) return 0u;
  const float t = (v - vb.lo) * vb.inv;
  if (!(t > 0.f)) return 1u;                       // (also NaN: inv 0 with an infinite difference)
  return t >= (float)(kBins - 2) ? (uint32_t)(kBins - 1) : 1u + (uint32_t)t;
}
// key interval of level-0 bin bn, clipped to the finite keys [clo, chi]
__device__ inline void vbin_interval(uint32_t bn, const VBins& vb, uint32_t clo, uint32_t chi, uint32_t& a,
                                     uint32_t& z) {
  auto first = [&](uint32_t target) -> uint64_t {   // smallest key in [clo, chi] with vbin >= target
    uint64_t lo = clo, hi = (uint64_t)chi + 1;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (vbin(key2f((uint32_t)mid), vb) >= target) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  };
  const uint64_t A = bn == 0 ? clo : first(bn);
  const uint64_t Z = bn + 1 >= (uint32_t)kBins ? (uint64_t)chi : first(bn + 1) - 1;
  a = (uint32_t)A;
  z = (uint32_t)(Z < A ? A : Z);
}

constexpr uint32_t kKeyPosInf = 0xff800000u;   // f2key(+inf); larger keys are +NaN payloads
constexpr uint32_t kKeyNegInf = 0x007fffffu;   // f2key(-inf); smaller keys are -NaN payloads
__device__ __forceinline__ bool key_nonfinite(uint32_t k) { return k >= kKeyPosInf || k <= kKeyNegInf; }

// First launch of a call (kRangeChunks workgroups per image): per-image selection state,
// cv2 tap tables, zeroed histograms, and the finite key range of each model-resolution map
// as per-chunk partials (k_model_hist reduces them).
__global__ __launch_bounds__(kBlock) void k_prepare(const float* depth, int B, int m, int n, SelState* st,
                                                    uint32_t* hist, uint32_t* rpart, Tap* xt, Tap* yt, int dh, int dw,
                                                    int H, int W, double sx, double sy, double* trig, uint32_t* mhist,
                                                    int nrc, uint32_t* wpart, uint32_t* slow, uint32_t* scr) {
  __shared__ uint32_t red[2][kBlock / 64];
  const int gtid = blockIdx.x * kBlock + threadIdx.x;
  const int nthr = gridDim.x * kBlock;
  if (gtid < B) {
    SelState s{};
    s.phase = PH_INIT;
    s.n = (uint32_t)n;
    s.kmin = 0xffffffffu;
    s.kmax = 0u;
    s.rlo = 0xffffffffu;
    s.rhi = 0u;
    for (int i = 0; i < 6; i += 2) { s.bbox_key[i] = 0xffffffffu; s.bbox_key[i + 1] = 0u; }
    for (int w = 0; w < 3; ++w) { s.wminF[w] = s.wminL[w] = 0xffffffffu; }
    for (int t = 0; t < kMaxTgt; ++t) s.tslot[t] = kNoSlot;
    s.med = __uint_as_float(0x7fc00000u);
    st[gtid] = s;
  }
  for (int i = gtid; i < W; i += nthr) {
    Tap t = make_tap(i, dw, sx);
    if (dw == 1) { t.i0 = 0; t.i1 = -1; t.w0 = 1.f; t.w1 = 0.f; }
    xt[i] = t;
  }
  for (int i = gtid; i < H; i += nthr) {
    Tap t = make_tap(i, dh, sy);
    // vertical pass always uses two rows: the second clamps to the last row
    if (t.i1 < 0) t.i1 = t.i0;
    yt[i] = t;
  }
  if (hist)        // (the level histograms: band path only)
    for (size_t i = gtid; i < (size_t)B * kSlots * kBins; i += nthr) hist[i] = 0;
  if (mhist)       // the sample histograms k_model_hist adds into
    for (size_t i = gtid; i < (size_t)B * kBins; i += nthr) mhist[i] = 0;
  if (wpart)       // k_sweep_w's below-window slots
    for (size_t i = gtid; i < (size_t)B * kBelowSlots * 4; i += nthr) wpart[i] = 0;
  if (slow)        // k_sel_slow: {ticket, min key, max key, NaN, non-finite, -inf, +inf, -} per image
    for (int i = gtid; i < 8 * B; i += nthr) slow[i] = (i & 7) == 1 ? 0xffffffffu : 0u;
  if (scr)         // the from-scratch level-0 histograms (the later levels: zeroed by the level before)
    for (size_t i = gtid; i < (size_t)B * kScrL1; i += nthr) scr[(i / kScrL1) * kScrWords + i % kScrL1] = 0;
  if (trig) {       // equirectangular ray tables (the oracle evaluates the same expressions)
    const double pi = 3.141592653589793;
    for (int i = gtid; i < W + H; i += nthr) {
      const double a = i < W ? ((double)i + 0.5) * (2.0 * pi / (double)W) - pi
                             : pi / 2.0 - ((double)(i - W) + 0.5) * (pi / (double)H);
      trig[2 * i] = sin(a);
      trig[2 * i + 1] = cos(a);
    }
  }
  const int b = blockIdx.x % B, c = blockIdx.x / B;
  const float* D = depth + (size_t)b * m;
  uint32_t lo = 0xffffffffu, hi = 0u;
  auto take = [&](float v) {
    if (isfinite(v)) {
      const uint32_t k = f2key(v);
      lo = min(lo, k);
      hi = max(hi, k);
    }
  };
  if ((m & 3) == 0) {
    const int m4 = m >> 2;
    const int per = (m4 + nrc - 1) / nrc;
    const int i1 = min(m4, (c + 1) * per);
    const float4* D4 = reinterpret_cast<const float4*>(D);
    for (int i = c * per + threadIdx.x; i < i1; i += kBlock) {
      const float4 v = D4[i];
      take(v.x); take(v.y); take(v.z); take(v.w);
    }
  } else {
    const int per = (m + nrc - 1) / nrc;
    const int i1 = min(m, (c + 1) * per);
    for (int i = c * per + threadIdx.x; i < i1; i += kBlock) take(D[i]);
  }
  lo = wave_min_u32(lo);
  hi = wave_max_u32(hi);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = lo; red[1][threadIdx.x >> 6] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) { lo = min(lo, red[0][w]); hi = max(hi, red[1][w]); }
    rpart[((size_t)b * nrc + c) * 2] = lo;
    rpart[((size_t)b * nrc + c) * 2 + 1] = hi;
  }
}

// Level-0 histogram of a sample of each full-resolution map (finite values, the level-0 binning):
// every (image, chunk) workgroup adds its LDS histogram's non-empty bins into `mhist` [B][kBins]
// (zeroed by k_prepare) with global atomics.  The estimate k_window
// predicts the target bins from.
__global__ __launch_bounds__(kHistBlock) void k_model_hist(Geo g, int B, SelState* st, uint32_t* mhist,
                                                       const uint32_t* rpart, int stride, int nch, int nrc) {
  __shared__ __attribute__((aligned(16))) uint32_t lh[kBins];
  __shared__ uint32_t rr[2];
  const int b = blockIdx.x % B, c = blockIdx.x / B;
  SelState* S = st + b;
  for (int i = threadIdx.x; i < kBins; i += kHistBlock) lh[i] = 0;
  if (threadIdx.x < 64) {     // the image's key range from k_prepare's partials
    uint32_t lo = 0xffffffffu, hi = 0u;
    for (int i = threadIdx.x; i < nrc; i += 64) {
      lo = min(lo, rpart[((size_t)b * nrc + i) * 2]);
      hi = max(hi, rpart[((size_t)b * nrc + i) * 2 + 1]);
    }
    lo = wave_min_u32(lo);
    hi = wave_max_u32(hi);
    if (threadIdx.x == 0) {
      rr[0] = lo;
      rr[1] = hi;
      if (c == 0) { S->rlo = lo; S->rhi = hi; }
    }
  }
  __syncthreads();
  const VBins vb = level0_vbins(rr[0], rr[1]);
  // the histogram of a stratified random sample of the FULL-resolution map (values recomputed
  // with the cv2 taps): one point per cell at a hashed offset (lowbias32 of the cell index), so
  // its quantiles are the full map's up to sampling noise, unlike the model
  // pixels' (a zero floor of isolated model pixels all but vanishes in the resize).  A lattice
  // with a deterministic jitter aliased with the resize's tap phases: on a noisy 518 x 1036 map
  // upsampled 7.9x its p2 was 10 standard deviations off (phase-0 pixels, the raw model values,
  // make the tails).  Each thread walks a run of consecutive cells (neighbours share bins: one
  // LDS atomic per run), 8 samples' loads in flight at a time.
  const int nsx = (g.W + stride - 1) / stride, nsy = (g.H + stride - 1) / stride, ns = nsx * nsy;
  const int per = (ns + nch - 1) / nch;
  const int i0 = c * per, i1 = min(ns, i0 + per);
  const int tper = (per + kHistBlock - 1) / kHistBlock;
  const int t0 = i0 + threadIdx.x * tper, t1 = min(i1, t0 + tper);
  int run = -1;
  uint32_t cnt = 0;
  int sy = t0 / nsx, sx = t0 - sy * nsx;
  // cells of H / nsy x W / nsx pixels exactly (integer strides would leave a partial last cell
  // whose few rows get a whole cell's weight: the image's border, often extreme, over-sampled)
  const float cy = (float)g.H / (float)nsy, cx = (float)g.W / (float)nsx;
  for (int i = t0; i < t1; i += 8) {
    int py[8], px[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {       // (past t1: a repeat of the last sample, not counted)
      uint32_t h = (uint32_t)min(i + k, t1 - 1);
      h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
      py[k] = min((int)(((float)sy + (float)(h & 0xffffu) * (1.f / 65536.f)) * cy), g.H - 1);
      px[k] = min((int)(((float)sx + (float)(h >> 16) * (1.f / 65536.f)) * cx), g.W - 1);
      if (i + k + 1 < t1 && ++sx == nsx) { sx = 0; ++sy; }
    }
    float v[8];
    if (g.same) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = sample(g, b, py[k], px[k]);
    } else {
      Tap ty[8], tx[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ty[k] = g.yt[py[k]];
        tx[k] = g.xt[px[k]];
      }
      const float* D = g.depth + (size_t)b * g.dh * g.dw;
      float a0[8], a1[8], c0[8], c1[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float* r0 = D + (size_t)ty[k].i0 * g.dw;
        const float* r1 = D + (size_t)ty[k].i1 * g.dw;
        const int x1 = tx[k].i1 < 0 ? tx[k].i0 : tx[k].i1;
        a0[k] = r0[tx[k].i0]; a1[k] = r0[x1];
        c0[k] = r1[tx[k].i0]; c1[k] = r1[x1];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {     // sample()'s arithmetic (single-tap columns: the raw value)
        float h0, h1;
        if (tx[k].i1 < 0) { h0 = a0[k]; h1 = c0[k]; }
        else { h0 = a0[k] * tx[k].w0 + a1[k] * tx[k].w1; h1 = c0[k] * tx[k].w0 + c1[k] * tx[k].w1; }
        v[k] = h0 * ty[k].w0 + h1 * ty[k].w1;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int bn = (i + k < t1 && isfinite(v[k])) ? (int)vbin(v[k], vb) : -1;
      if (bn != run && run >= 0) atomicAdd(&lh[run], cnt);
      cnt = (bn == run ? cnt : 0u) + 1u;
      run = bn;
    }
  }
  if (run >= 0) atomicAdd(&lh[run], cnt);
  __syncthreads();
  uint32_t* gh = mhist + (size_t)b * kBins;       // (zeroed by k_prepare)
  for (int i = threadIdx.x; i < kBins; i += kHistBlock)
    if (lh[i]) atomicAdd(&gh[i], lh[i]);
}

// Block histogram in LDS as packed 16-bit counts (bin pairs share a word; a sweep workgroup
// covers at most 32 * kTileW < 65536 pixels, so a half never carries into its neighbour).
__device__ __forceinline__ void hist_add(uint32_t* sh, int bin, uint32_t cnt) {
  atomicAdd(&sh[bin >> 1], cnt << ((bin & 1) << 4));
}

// Copy n floats global -> LDS (256 threads) with each thread's loads all in flight before its
// first store; 16-byte accesses when the source is 16-byte aligned and n % 4 == 0.
__device__ __forceinline__ void stage_floats(float* dst, const float* src, int n) {
  if (((uintptr_t)src & 15) == 0 && (n & 3) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    const int n4 = n >> 2;
    for (int base = 0; base < n4; base += 4 * 256) {
      float4 r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = s4[min(base + k * 256 + (int)threadIdx.x, n4 - 1)];
      // stores clamped too (past the end: the last element's own value again), so hipcc cannot
      // sink each load into a predicated store block and wait for it there
#pragma unroll
      for (int k = 0; k < 4; ++k) d4[min(base + k * 256 + (int)threadIdx.x, n4 - 1)] = r[k];
    }
  } else {
    for (int base = 0; base < n; base += 8 * 256) {
      float r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = src[min(base + k * 256 + (int)threadIdx.x, n - 1)];
#pragma unroll
      for (int k = 0; k < 8; ++k) dst[min(base + k * 256 + (int)threadIdx.x, n - 1)] = r[k];
    }
  }
}

// Row-blocked sweep geometry: a workgroup owns image b and output rows [v0, v1);
// the model-resolution rows feeding them are staged once into LDS, every thread
// owns 4 columns (+1024 per chunk), the row taps are wave-uniform.
struct Sweep {
  int R;         // output rows per workgroup
  int nrb;       // row blocks per image
  int lds_rows;  // capacity of the LDS row window (0: sample from global)
  int row0;      // first output row swept (a band of the image in tile-parallel mode)
  int row_end;   // one past the last output row swept
  int ntiles;    // selection sweeps: column tiles of kTileW per row block (others: 1)
  int raw;       // selection sweeps: raw model rows staged in LDS before interpolation
  int tpr;       // k_unproject_rows: threads per point row (a multiple of 64; kBlock / tpr rows per pass)
  int nt;        // k_unproject_rows: non-temporal output stores
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

// One selection sweep over the full-resolution depth.  Workgroup = image b x output rows
// [v0, v1) x a column tile of kTileW; the model rows feeding it are interpolated horizontally
// once (cv2's first pass) into LDS, so a pixel costs two LDS reads and the vertical blend.
// (For finite values the generic a0*w0 + a1*w1 equals cv2's single-tap copy at the right
// border, whose weights are (1, 0); a non-finite tap only has to be detected here.)
// Level 0 bins every key over the model map's key range; levels 1-2 match each key against
// the slots' key intervals and either bin it (SM_HIST) or append it to the slot's candidate
// list (SM_COMPACT, staged in the slot's LDS region).  Histogram adds are run-length
// aggregated per thread down its columns.
template <int LEVEL, bool SAME>
__global__ __launch_bounds__(kBlock) void k_sweep(Geo g, SelState* st, uint32_t* hist, uint32_t* cand, uint32_t cap,
                                                  int B, Sweep sw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_u[];
  uint32_t* sh = smem_u;                                        // [slots * kSlotWords]
  // LDS: level 0 = [histogram | window 0-2 keys], levels 1-2 = one region per slot
  float* hrow = reinterpret_cast<float*>(smem_u + kSlots * kSlotWords);   // [rows][kTileW]
  __shared__ uint32_t red[3][kBlock / 64];
  __shared__ uint32_t lcnt[kSlots], gbase[kSlots];
  int b, chunk;
  map_block(blockIdx.x, B, sw.nrb * sw.ntiles, b, chunk);
  const int rb = chunk / sw.ntiles, c0 = (chunk - rb * sw.ntiles) * kTileW;
  const int cw = min(kTileW, g.W - c0);
  SelState* S = st + b;
  if (S->phase != (LEVEL == 0 ? PH_INIT : PH_SEL)) return;

  int nslot = 1;
  uint32_t slo[kSlots], shi[kSlots], smult[kSlots];
  bool scomp[kSlots];
  // level 0: windows of level-0 bins whose keys are compacted (k_window); empty = [1, 0]
  int wlo[3] = {1, 1, 1}, whi[3] = {0, 0, 0}, nwin = 0;
  VBins vb0{0.f, 0.f};
  if (LEVEL == 0) {
    vb0 = level0_vbins(S->rlo, S->rhi);
    nwin = (int)S->nwin;
#pragma unroll
    for (int w = 0; w < 3; ++w)
      if (w < nwin) { wlo[w] = (int)S->wbin[2 * w]; whi[w] = (int)S->wbin[2 * w + 1]; }
  } else {
    nslot = (int)S->nslot;
#pragma unroll
    for (int q = 0; q < kSlots; ++q) {
      slo[q] = S->slo[q];
      shi[q] = S->shi[q];
      smult[q] = S->smult[q];
      scomp[q] = S->smode[q] == SM_COMPACT;
    }
  }
  const int v0 = sw.row0 + rb * sw.R;
  const int v1 = min(sw.row_end, v0 + sw.R);
  for (int i = threadIdx.x; i < (LEVEL == 0 ? 1 : nslot) * kSlotWords; i += kBlock) sh[i] = 0;
  if (threadIdx.x < kSlots) lcnt[threadIdx.x] = 0;
  int lo = 0;
  if (!SAME) {
    // cv2's horizontal pass over the model rows of this block, into LDS: from raw rows staged
    // in LDS when they fit (else straight from the L2-resident map)
    lo = g.yt[v0].i0;
    const int nr = g.yt[v1 - 1].i1 - lo + 1;
    const float* D = g.depth + ((size_t)b * g.dh + lo) * g.dw;
    float* raw = hrow + (size_t)sw.lds_rows * kTileW;
    Tap tx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) tx[j] = g.xt[c0 + min(j * kBlock + (int)threadIdx.x, cw - 1)];
    if (sw.raw) {
      stage_floats(raw, D, nr * g.dw);
      __syncthreads();
    }
    const float* src = sw.raw ? raw : D;
    for (int k = 0; k < nr; ++k) {
      const float* r = src + (size_t)k * g.dw;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int u = j * kBlock + (int)threadIdx.x;
        if (u < cw) hrow[k * kTileW + u] = r[tx[j].i0] * tx[j].w0 + r[tx[j].i1 < 0 ? tx[j].i0 : tx[j].i1] * tx[j].w1;
      }
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const float* Dimg = g.depth + (size_t)b * g.dh * g.dw;
  uint32_t nf = 0, nnan = 0, nneg = 0, npos = 0, kmin = 0xffffffffu, kmax = 0u;
  int run_bin[4] = {-1, -1, -1, -1};
  uint32_t run_cnt[4] = {0, 0, 0, 0};
  Tap ty_next = SAME ? Tap{0, 0, 1.f, 0.f} : g.yt[v0];
  for (int v = v0; v < v1; ++v) {
    // every load unconditional (columns clamped into the tile), all issued before any use;
    // the next row's taps are loaded a row ahead
    float ha[4], hc[4];
    const Tap ty = ty_next;
    if (!SAME) ty_next = g.yt[min(v + 1, v1 - 1)];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int uc = min(j * kBlock + (int)threadIdx.x, cw - 1);
      if (SAME) {
        ha[j] = Dimg[(size_t)v * g.dw + c0 + uc];
      } else {
        ha[j] = hrow[(ty.i0 - lo) * kTileW + uc];
        hc[j] = hrow[(ty.i1 - lo) * kTileW + uc];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool active = j * kBlock + (int)threadIdx.x < cw;
      const float val = SAME ? ha[j] : ha[j] * ty.w0 + hc[j] * ty.w1;
      const uint32_t key = f2key(val);
      int hb = -1;
      int cq = -1;
      if (LEVEL == 0) {
        // finite keys only are binned (NaN / +-Inf are counted: the nanmedian fill)
        const bool fin = active && !key_nonfinite(key);
        if (active && !fin) {
          ++nf;
          nnan += (key != kKeyPosInf && key != kKeyNegInf) ? 1u : 0u;
          nneg += key == kKeyNegInf ? 1u : 0u;
          npos += key == kKeyPosInf ? 1u : 0u;
        }
        kmin = min(kmin, fin ? key : 0xffffffffu);
        kmax = max(kmax, fin ? key : 0u);
        hb = fin ? (int)vbin(val, vb0) : -1;
        cq = (hb >= wlo[0] && hb <= whi[0]) ? 0 : (hb >= wlo[1] && hb <= whi[1]) ? 1 : (hb >= wlo[2] && hb <= whi[2]) ? 2 : -1;
      } else {
#pragma unroll
        for (int q = 0; q < kSlots; ++q) {
          const bool in = active && q < nslot && key >= slo[q] && key <= shi[q];
          cq = (in && scomp[q]) ? q : cq;
          hb = (in && !scomp[q]) ? q * kBins + (int)bin_of(key, slo[q], smult[q]) : hb;
        }
      }
      if (hb != run_bin[j] && run_bin[j] >= 0) hist_add(sh, run_bin[j], run_cnt[j]);
      run_cnt[j] = (hb == run_bin[j] ? run_cnt[j] : 0u) + 1u;
      run_bin[j] = hb;
      if ((LEVEL > 0 || nwin > 0) && __ballot(cq >= 0)) {
        // a compaction slot's LDS region (unused by a histogram) stages its keys; one
        // LDS atomic per slot and wave, global appends only past kSlotWords keys per block
#pragma unroll
        for (int q = 0; q < (LEVEL == 0 ? 3 : kSlots); ++q) {
          const uint64_t m = __ballot(cq == q);
          if (!m) continue;
          const int leader = __ffsll((unsigned long long)m) - 1;
          uint32_t base = 0;
          if (lane == leader) base = atomicAdd(&lcnt[q], (uint32_t)__popcll(m));
          base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
          if (cq == q) {
            const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (pos < (uint32_t)kSlotWords) {
              sh[(LEVEL == 0 ? q + 1 : q) * kSlotWords + pos] = key;
            } else {
              const uint32_t gpos = atomicAdd(&S->ccount[q], 1u);
              if (gpos < cap) cand[((size_t)b * kSlots + q) * cap + gpos] = key;
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (run_bin[j] >= 0) hist_add(sh, run_bin[j], run_cnt[j]);
  if (LEVEL == 0) {
    const int wid = threadIdx.x >> 6;
    nf = wave_sum_u32(nf);
    kmin = wave_min_u32(kmin);
    kmax = wave_max_u32(kmax);
    if (lane == 0) { red[0][wid] = nf; red[1][wid] = kmin; red[2][wid] = kmax; }
    if (__builtin_amdgcn_readfirstlane(nf)) {       // rare: split the non-finite count
      nnan = wave_sum_u32(nnan);
      nneg = wave_sum_u32(nneg);
      npos = wave_sum_u32(npos);
      if (lane == 0) {
        if (nnan) atomicAdd(&S->nan_count, nnan);
        if (nneg) atomicAdd(&S->ninf_neg, nneg);
        if (npos) atomicAdd(&S->ninf_pos, npos);
      }
    }
  }
  __syncthreads();
  if (LEVEL == 0 && threadIdx.x == 0) {
    uint32_t c = 0, mn = 0xffffffffu, mx = 0;
    for (int w = 0; w < kBlock / 64; ++w) { c += red[0][w]; mn = min(mn, red[1][w]); mx = max(mx, red[2][w]); }
    if (c) atomicAdd(&S->nonfinite_count, c);
    if (mn != 0xffffffffu) atomicMin(&S->kmin, mn);
    if (mx) atomicMax(&S->kmax, mx);
  }
  uint32_t* gh = hist + (size_t)b * kSlots * kBins;
  // compaction slots: q -> LDS region (level 0: the windows, regions 1-3), cand slot q
  const int ncq = LEVEL == 0 ? nwin : nslot;
  for (int q = 0; q < ncq; ++q) {
    if (LEVEL > 0 && !scomp[q]) continue;
    if (threadIdx.x == 0) {
      const uint32_t nq = min(lcnt[q], (uint32_t)kSlotWords);
      gbase[q] = nq ? atomicAdd(&S->ccount[q], nq) : 0u;
    }
  }
  // histogram slots (packed 16-bit LDS counts -> global)
  for (int q = 0; q < (LEVEL == 0 ? 1 : nslot); ++q) {
    if (LEVEL > 0 && scomp[q]) continue;
    for (int i = threadIdx.x; i < kSlotWords; i += kBlock) {
      const uint32_t w = sh[q * kSlotWords + i];
      if (w & 0xffffu) atomicAdd(&gh[q * kBins + 2 * i], w & 0xffffu);
      if (w >> 16) atomicAdd(&gh[q * kBins + 2 * i + 1], w >> 16);
    }
  }
  if (ncq > 0) {
    __syncthreads();
    for (int q = 0; q < ncq; ++q) {
      if (LEVEL > 0 && !scomp[q]) continue;
      const uint32_t nq = min(lcnt[q], (uint32_t)kSlotWords);
      const uint32_t* src = sh + (LEVEL == 0 ? q + 1 : q) * kSlotWords;
      uint32_t* dst = cand + ((size_t)b * kSlots + q) * cap;
      for (uint32_t i = threadIdx.x; i < nq; i += kBlock)
        if (gbase[q] + i < cap) dst[gbase[q] + i] = src[i];
    }
  }
}

// Window-only selection sweep (the batch path's only full-resolution pass before the
// unprojection): no histogram at all.  Per k_window window w it counts the finite values below
// the window, compacts the keys inside it into w's candidate list, and -- for an end bin
// k_window flagged as a spike -- counts that bin's keys with their min / max key instead of
// compacting them; plus the non-finite counts.  k_resolve_w turns this into exact keys; a target
// outside every window (or in an unresolvable part) falls to k_sel_slow.
//
// The window bounds arrive as VALUES (k_window: the first / last key of the window's level-0
// bins, as floats), so a pixel costs its cv2 interpolation, one class test and two float
// compares per window (VALU) plus a few mask operations (SALU, balanced against the VALU: both
// issue about once per CU cycle).  Lanes past the tile's edge carry NaN (below no window, in
// none); keys are formed only in the rare waves that hold a window pixel.  Float order is key order on finite values
// except -0 < +0, and a bin bound never separates the two zeros (vbin maps both to one bin).
template <bool SAME, int NW>
__device__ __forceinline__ void sweep_w_rows(const Geo& g, SelState* S, uint32_t* cand, uint32_t cap, int b,
                                             int v0, int v1, int cw, int c0, const Tap* tys,
                                             uint32_t (*sh)[kStageW], uint32_t (*red)[32],
                                             const float* vlo, const float* vhi, const float* vF,
                                             const float* vL, const uint32_t* spk) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float* Dimg = g.depth + (size_t)b * g.dh * g.dw;
  int ucol[4];
  bool act[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    act[j] = j * kBlock + (int)threadIdx.x < cw;
    ucol[j] = c0 + min(j * kBlock + (int)threadIdx.x, cw - 1);
  }
  bool any_spike = false;
#pragma unroll
  for (int w = 0; w < NW; ++w) any_spike |= spk[w] != 0u;
  Tap tx[4];
  // rows ra (hA) and ra + 1 (hB) interpolated, the raw taps of rows ra + 2 (p2) and ra + 3 (p3)
  // in flight: an advance waits on loads issued two advances earlier
  float hA[4], hB[4], p2[8], p3[8];
  int ra = 0;
  auto load_raw = [&](int r, float (&q)[8]) {
    const float* R0 = Dimg + (size_t)min(r, g.dh - 1) * g.dw;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q[2 * j] = R0[tx[j].i0];
      q[2 * j + 1] = R0[tx[j].i1 < 0 ? tx[j].i0 : tx[j].i1];
    }
  };
  auto interp = [&](const float (&q)[8], float (&h)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)     // cv2 HResizeLinear (a single-tap column: the raw value, as sample())
      h[j] = !act[j] ? __builtin_nanf("")      // (past the tile: NaN, in no window, below none)
                     : (tx[j].i1 < 0 ? q[2 * j] : q[2 * j] * tx[j].w0 + q[2 * j + 1] * tx[j].w1);
  };
  float cur[4];
  if (SAME) {
#pragma unroll
    for (int j = 0; j < 4; ++j) cur[j] = Dimg[(size_t)v0 * g.dw + ucol[j]];
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) tx[j] = g.xt[ucol[j]];
    ra = tys[0].i0;
    float q0[8], q1[8];
    load_raw(ra, q0);
    load_raw(ra + 1, q1);
    load_raw(ra + 2, p2);
    load_raw(ra + 3, p3);
    interp(q0, hA);
    interp(q1, hB);
  }

  // non-finite counts: wave-uniform (scalar registers); the rest per lane (wave-reduced at the end)
  uint32_t nf = 0, nnan = 0, nneg = 0, npos = 0;
  uint32_t below[NW], cF[NW], cL[NW];
  uint32_t mnF[NW], mxF[NW], mnL[NW], mxL[NW];
  uint32_t wc[NW];                 // keys in this wave's LDS buffer of window w (wave-uniform)
  uint32_t* wbuf = &sh[0][0] + wid * kWaveBuf;      // + w * kStageW
  // the finite range of the swept pixels (r04: app.py:198-199's min / max branch for near-constant
  // maps, so k_sel_slow needs no pass of its own): float min / max, NaN ignored (minnum), +-inf
  // masked in the rare non-finite branch; key order == float order on finite values but -0 < +0,
  // which the end of k_sweep_w checks
  float fmn = INFINITY, fmx = -INFINITY;
  uint32_t* cw_dst[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    wc[w] = 0u;
    cw_dst[w] = cand + ((size_t)b * kSlots + w) * cap;
    below[w] = cF[w] = cL[w] = 0u;
    mnF[w] = mnL[w] = 0xffffffffu;
    mxF[w] = mxL[w] = 0u;
  }
  for (int v = v0; v < v1; ++v) {
    float val[4];
    if (SAME) {
      // the next row's values in flight while this row is counted
      const int vn = min(v + 1, v1 - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        val[j] = act[j] ? cur[j] : __builtin_nanf("");
        cur[j] = Dimg[(size_t)vn * g.dw + ucol[j]];
      }
    } else {
      const Tap ty = tys[v - v0];
      // advance the register rows to ty.i0 (wave-uniform; once per ~H / dh output rows)
      while (ra < ty.i0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) hA[j] = hB[j];
        interp(p2, hB);
#pragma unroll
        for (int i = 0; i < 8; ++i) p2[i] = p3[i];
        ++ra;
        load_raw(ra + 3, p3);
      }
      const bool second_is_a = ty.i1 == ra;     // (the bottom rows clamp i1 to i0)
#pragma unroll
      for (int j = 0; j < 4; ++j) val[j] = hA[j] * ty.w0 + (second_is_a ? hA[j] : hB[j]) * ty.w1;   // cv2 VResizeLinear
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = val[j];
      float xr = x;                                   // x for the range: NaN unless finite
      if (__ballot(!__builtin_isfinite(x))) {     // rare: split the non-finite pixels (edge lanes' NaN aside)
        xr = __builtin_isfinite(x) ? x : __builtin_nanf("");
        const uint64_t am = __ballot(act[j]);
        const bool ni = x == -INFINITY;
        const uint64_t nfm = __ballot(!__builtin_isfinite(x)) & am;
        const uint64_t negm = __ballot(ni) & am;
        const uint64_t posm = __ballot(x == INFINITY) & am;
        nf += (uint32_t)__popcll(nfm);
        nneg += (uint32_t)__popcll(negm);
        npos += (uint32_t)__popcll(posm);
        nnan += (uint32_t)__popcll(nfm & ~(negm | posm));
#pragma unroll
        for (int w = 0; w < NW; ++w) below[w] -= ni ? 1u : 0u;   // -inf compares below every window
      }
      fmn = fminf(fmn, xr);
      fmx = fmaxf(fmx, xr);
      bool inw[NW], anyl = false;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const bool bl = x < vlo[w];
        below[w] += bl ? 1u : 0u;
        inw[w] = !bl && x <= vhi[w];               // (NaN / +inf: neither)
        anyl |= inw[w];
      }
      if (!__ballot(anyl)) continue;
      const uint32_t key = f2key(x);
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        uint64_t m = __ballot(inw[w]);
        if (!m) continue;
        if (any_spike && spk[w]) {
          const uint64_t fm = (spk[w] & 1u) ? __ballot(x <= vF[w]) & m : 0ull;
          const uint64_t lm = (spk[w] & 2u) ? __ballot(x >= vL[w]) & m & ~fm : 0ull;
          const bool inF = (fm >> lane) & 1ull, inL = (lm >> lane) & 1ull;
          cF[w] += inF ? 1u : 0u;
          cL[w] += inL ? 1u : 0u;
          mnF[w] = inF ? min(mnF[w], key) : mnF[w];
          mxF[w] = inF ? max(mxF[w], key) : mxF[w];
          mnL[w] = inL ? min(mnL[w], key) : mnL[w];
          mxL[w] = inL ? max(mxL[w], key) : mxL[w];
          m &= ~(fm | lm);
          if (!m) continue;
        }
        // the wave's own LDS buffer (kWaveBuf keys per window); a full buffer leaves as one
        // reservation of kWaveBuf candidate slots and four contiguous 256-B stores, so a
        // spatially dense window (a smooth map puts a quantile's pixels in a few blocks; one
        // large image has them all) costs one global atomic per kWaveBuf keys
        const uint32_t cnt = (uint32_t)__popcll(m);
        const bool mine = (m >> lane) & 1ull;
        const uint32_t pos = wc[w] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        uint32_t* buf = wbuf + w * kStageW;
        if (mine && pos < (uint32_t)kWaveBuf) buf[pos] = key;
        if (wc[w] + cnt >= (uint32_t)kWaveBuf) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's buffer writes, then its reads
          uint32_t gb = 0;
          if (lane == 0) gb = atomicAdd(&S->ccount[w], (uint32_t)kWaveBuf);
          gb = (uint32_t)__builtin_amdgcn_readfirstlane((int)gb);
          uint32_t kk[kWaveBuf / 64];
#pragma unroll
          for (int i = 0; i < kWaveBuf / 64; ++i) kk[i] = buf[i * 64 + lane];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int i = 0; i < kWaveBuf / 64; ++i)
            if (gb + i * 64 + lane < cap) cw_dst[w][gb + i * 64 + lane] = kk[i];
          if (mine && pos >= (uint32_t)kWaveBuf) buf[pos - kWaveBuf] = key;
          wc[w] = wc[w] + cnt - (uint32_t)kWaveBuf;
        } else {
          wc[w] += cnt;
        }
      }
    }
  }
  // the wave's finite range -> red (the image's key range: k_sweep_w, once per workgroup).  The float min / max
  // may pick +0 over -0 (or the reverse): exact keys unless a zero is an end of the range and the
  // model map holds a value <= -0 (only then can a -0 pixel exist); such an image is flagged and
  // k_sel_slow counts its range itself (SelState::pad3[0] bit 1)
  for (int o = 32; o > 0; o >>= 1) {
    fmn = fminf(fmn, __shfl_xor(fmn, o));
    fmx = fmaxf(fmx, __shfl_xor(fmx, o));
  }
  // (the workgroup's range goes to the image with one check-then-atomic pair at the end of k_sweep_w)
  uint32_t rk_lo = 0xffffffffu, rk_hi = 0u;
  if (fmn <= fmx) {
    if ((fmn == 0.f || fmx == 0.f) && S->rlo < f2key(0.f)) {
      if (lane == 0) atomicOr(&S->pad3[0], 2u);
    } else {
      rk_lo = f2key(fmn); rk_hi = f2key(fmx);
    }
  }
  if (lane == 0) { red[wid][28] = rk_lo; red[wid][29] = rk_hi; }
  // wave totals -> red[wave][...]: 0 nf, 1 nnan, 2 nneg, 3 npos, 4 + w below, then per window
  // 7 + 6 w: F count / min / max, L count / min / max; 25 + w: keys left in the wave's buffer;
  // 28 / 29: the finite key range (r03 put window 0's spike count on 6 = below[2])
#pragma unroll
  for (int w = 0; w < NW; ++w) below[w] = wave_sum_u32(below[w]);
  if (lane == 0) {
    red[wid][0] = nf; red[wid][1] = nnan; red[wid][2] = nneg; red[wid][3] = npos;
#pragma unroll
    for (int w = 0; w < NW; ++w) { red[wid][4 + w] = below[w]; red[wid][25 + w] = wc[w]; }
  }
  if (any_spike) {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t a = wave_sum_u32(cF[w]), c = wave_min_u32(mnF[w]), d = wave_max_u32(mxF[w]);
      const uint32_t e = wave_sum_u32(cL[w]), f = wave_min_u32(mnL[w]), h = wave_max_u32(mxL[w]);
      if (lane == 0) {
        red[wid][7 + 6 * w] = a; red[wid][8 + 6 * w] = c; red[wid][9 + 6 * w] = d;
        red[wid][10 + 6 * w] = e; red[wid][11 + 6 * w] = f; red[wid][12 + 6 * w] = h;
      }
    }
  }
}

template <bool SAME>
__global__ __launch_bounds__(kBlock) void k_sweep_w(Geo g, SelState* st, uint32_t* cand, uint32_t cap, int B,
                                                    Sweep sw, uint32_t* wpart) {
  // thread = 4 columns c0 + j * kBlock + tid of a kTileW-column tile, walking down the block's
  // R output rows.  The horizontal cv2 pass of a model row is a thread's own business (its 4
  // columns), so it stays in registers.
  __shared__ uint32_t sh[3][kStageW];               // per window: the waves' key buffers (kWaveBuf each)
  __shared__ uint32_t red[kBlock / 64][32];
  __shared__ uint32_t gbase[3];
  __shared__ Tap tys[kMaxSelRows];                  // the block's row taps (no global load in the row loop)
  int b, chunk;
  map_block(blockIdx.x, B, sw.nrb * sw.ntiles, b, chunk);
  const int rb = chunk / sw.ntiles, c0 = (chunk - rb * sw.ntiles) * kTileW;
  const int cw = min(kTileW, g.W - c0);
  SelState* S = st + b;
  if (S->phase != PH_INIT) return;
  const int nwin = (int)S->nwin;
  if (nwin == 0) return;                            // (no window: every target goes to k_sel_slow)
  float vlo[3], vhi[3], vF[3], vL[3];
  uint32_t spk[3];
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    vlo[w] = S->wvlo[w]; vhi[w] = S->wvhi[w]; vF[w] = S->wvF[w]; vL[w] = S->wvL[w];
    spk[w] = w < nwin ? S->wspike[w] : 0u;
  }
  const int v0 = sw.row0 + rb * sw.R;
  const int v1 = min(sw.row_end, v0 + sw.R);
  if (!SAME && (int)threadIdx.x < v1 - v0) tys[threadIdx.x] = g.yt[v0 + threadIdx.x];
  __syncthreads();
  switch (nwin) {
    case 1: sweep_w_rows<SAME, 1>(g, S, cand, cap, b, v0, v1, cw, c0, tys, sh, red, vlo, vhi, vF, vL, spk); break;
    case 2: sweep_w_rows<SAME, 2>(g, S, cand, cap, b, v0, v1, cw, c0, tys, sh, red, vlo, vhi, vF, vL, spk); break;
    default: sweep_w_rows<SAME, 3>(g, S, cand, cap, b, v0, v1, cw, c0, tys, sh, red, vlo, vhi, vF, vL, spk); break;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c[4] = {0, 0, 0, 0};
    for (int w = 0; w < kBlock / 64; ++w)
      for (int i = 0; i < 4; ++i) c[i] += red[w][i];
    // kmin only falls and kmax only rises, so the atomic is skipped when a relaxed read already
    // shows a value at least as extreme (a stale read errs towards issuing it): one 8192x4096 image
    // is 2 K workgroups on the same two words (per-wave unconditional atomics: C4 sweep 61 -> 210 us)
    uint32_t klo = 0xffffffffu, khi = 0u;
    for (int w = 0; w < kBlock / 64; ++w) { klo = min(klo, red[w][28]); khi = max(khi, red[w][29]); }
    if (klo <= khi) {
      if (klo < __hip_atomic_load(&S->kmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&S->kmin, klo);
      if (khi > __hip_atomic_load(&S->kmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&S->kmax, khi);
    }
    if (c[0]) {
      atomicAdd(&S->nonfinite_count, c[0]);
      if (c[1]) atomicAdd(&S->nan_count, c[1]);
      if (c[2]) atomicAdd(&S->ninf_neg, c[2]);
      if (c[3]) atomicAdd(&S->ninf_pos, c[3]);
    }
    for (int q = 0; q < nwin; ++q) {
      uint32_t bw = 0;
      for (int w = 0; w < kBlock / 64; ++w) bw += red[w][4 + q];
      if (bw) atomicAdd(&wpart[((size_t)b * kBelowSlots + (blockIdx.x % kBelowSlots)) * 4 + q], bw);
      uint32_t nq = 0;                 // the waves' leftover keys: one reservation per window
      for (int w = 0; w < kBlock / 64; ++w) nq += red[w][25 + q];
      gbase[q] = nq ? atomicAdd(&S->ccount[q], nq) : 0u;
      if (spk[q]) {
        uint32_t a = 0, cmn = 0xffffffffu, dmx = 0, e = 0, fmn = 0xffffffffu, hmx = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
          a += red[w][7 + 6 * q]; cmn = min(cmn, red[w][8 + 6 * q]); dmx = max(dmx, red[w][9 + 6 * q]);
          e += red[w][10 + 6 * q]; fmn = min(fmn, red[w][11 + 6 * q]); hmx = max(hmx, red[w][12 + 6 * q]);
        }
        if (a) { atomicAdd(&S->wcntF[q], a); atomicMin(&S->wminF[q], cmn); atomicMax(&S->wmaxF[q], dmx); }
        if (e) { atomicAdd(&S->wcntL[q], e); atomicMin(&S->wminL[q], fmn); atomicMax(&S->wmaxL[q], hmx); }
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int q = 0; q < nwin; ++q) {
    uint32_t off = gbase[q];
    for (int w = 0; w < wid; ++w) off += red[w][25 + q];
    const uint32_t nq = red[wid][25 + q];
    uint32_t* dst = cand + ((size_t)b * kSlots + q) * cap;
    for (uint32_t i = lane; i < nq; i += 64)
      if (off + i < cap) dst[off + i] = sh[q][wid * kWaveBuf + i];
  }
}

// For one histogram of `nb` bins, the bins holding the 0-based ranks[0..nt) and the ranks
// inside them (all NT threads call; results in out_bin / out_rem after the closing barrier).
// Each thread owns nb / NT consecutive bins; the segment sums are scanned per wave with
// lane shuffles and offset by the preceding waves' totals.
template <int NT = kBlock>
__device__ void find_bins(const uint32_t* h, int nb, const uint32_t* ranks, int nt, uint32_t* wsum,
                          uint32_t* out_bin, uint32_t* out_rem) {
  const int per = nb / NT;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t local = 0;
  for (int i = 0; i < per; ++i) local += h[t * per + i];
  uint32_t x = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t off = 0;
  for (int i = 0; i < w; ++i) off += wsum[i];
  const uint32_t incl = x + off;
  const uint32_t excl = incl - local;
  for (int k = 0; k < nt; ++k) {
    const uint32_t rank = ranks[k];
    if (rank >= excl && rank < incl) {
      uint32_t c = excl;
      for (int i = 0; i < per; ++i) {
        const uint32_t hv = h[t * per + i];
        if (rank < c + hv) { out_bin[k] = (uint32_t)(t * per + i); out_rem[k] = rank - c; break; }
        c += hv;
      }
    }
  }
  __syncthreads();
}

__device__ void pct_ranks(uint32_t n, uint32_t* rank) {
  const double qs[2] = {2.0 / 100.0, 98.0 / 100.0};   // q = [2,98] / float32(100) -> float64
  for (int j = 0; j < 2; ++j) {
    const double v = (double)(n - 1) * qs[j];
    uint32_t i0, i1;
    if (v >= (double)(n - 1)) { i0 = i1 = n - 1; }
    else { i0 = (uint32_t)floor(v); i1 = i0 + 1; }
    rank[2 * j] = i0;
    rank[2 * j + 1] = i1;
  }
}

// np.percentile's linear interpolation between the keys of ranks i0 / i1 (keys[4]), then
// app.py:198-206's branch choice.  have_mm: s.kmin / s.kmax hold the map's finite key range (the
// window path does not count it: it returns false, s unchanged, when the branch needs it).
__device__ bool finalize_pct(SelState& s, const uint32_t* keys, bool have_mm = true) {
  const uint32_t n = s.n;
  const double qs[2] = {2.0 / 100.0, 98.0 / 100.0};
  double r[2];
  for (int j = 0; j < 2; ++j) {
    const double v = (double)(n - 1) * qs[j];
    const double t = v - floor(v);
    const float a = key2f(keys[2 * j]);
    const float bb = key2f(keys[2 * j + 1]);
    const float diff = bb - a;
    r[j] = t >= 0.5 ? (double)bb - (double)diff * (1.0 - t) : (double)a + (double)diff * t;
  }
  double p2 = r[0], p98 = r[1];
  int branch = 0;
  if (p98 <= p2) {                       // app.py:198-199
    if (!have_mm) return false;
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
  return true;
}

// n 32-bit words global -> LDS by global_load_lds (16 B per lane, 1 KiB per wave-instruction,
// every piece in flight at once; 256 threads).  src 16-byte aligned and readable up to the next
// multiple of 256 words past n (the tail lanes copy that slack); dst holds that many words.
// Ends with the wait and the barrier.
__device__ __forceinline__ void dma_words(uint32_t* dst, const uint32_t* src, uint32_t n) {
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t base = w * 256; base < n; base += 4 * 256)
    __builtin_amdgcn_global_load_lds(src + base + lane * 4, (__attribute__((address_space(3))) void*)(dst + base), 16,
                                     0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// Candidate keys global -> LDS, 4 loads per thread in flight.
__device__ __forceinline__ void load_keys(uint32_t* dst, const uint32_t* src, uint32_t c) {
  for (uint32_t i0 = 0; i0 < c; i0 += 4 * kBlock) {
    uint32_t kk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) kk[k] = src[min(i0 + k * kBlock + threadIdx.x, c - 1)];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i0 + k * kBlock + threadIdx.x < c) dst[i0 + k * kBlock + threadIdx.x] = kk[k];
  }
}

// One narrowing round over candidate keys: a linear 2048-bin histogram of [lo, hi] and the
// bins of ranks[0..nt) (block-wide; results in rbin / rrem).
__device__ void cand_round(const uint32_t* keys, uint32_t c, uint32_t lo, uint32_t hi, const uint32_t* ranks, int nt,
                           uint32_t* lh, uint32_t* wsum, uint32_t* rbin, uint32_t* rrem) {
  const uint32_t mult = bin_mult(lo, hi);
  for (int i = threadIdx.x; i < kBins; i += kBlock) lh[i] = 0;
  if (threadIdx.x < nt) { rbin[threadIdx.x] = 0; rrem[threadIdx.x] = 0; }
  __syncthreads();
  for (uint32_t i0 = 0; i0 < c; i0 += 4 * kBlock) {
    uint32_t kk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) kk[k] = keys[min(i0 + k * kBlock + threadIdx.x, c - 1)];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i0 + k * kBlock + threadIdx.x < c && kk[k] >= lo && kk[k] <= hi) atomicAdd(&lh[bin_of(kk[k], lo, mult)], 1u);
  }
  __syncthreads();
  find_bins(lh, kBins, ranks, nt, wsum, rbin, rrem);
}

// Exact keys of ranks[0..nt) among one slot's candidate keys, all inside [lo, hi]: one round
// for every target of the slot; a target whose bin then holds at most kGatherMax keys is settled
// by gathering them and counting ranks (one pass over the candidates), the rest narrow by further
// rounds (at most 1024 keys wide after level 0, so one key per bin) until one key wide.
// Block-wide; out, tl, tz, tr are shared arrays of nt entries.
constexpr uint32_t kGatherMax = 256;
__device__ void cand_select(const uint32_t* keys, uint32_t c, uint32_t lo, uint32_t hi, const uint32_t* ranks, int nt,
                            uint32_t* out, uint32_t* lh, uint32_t* wsum, uint32_t* rbin, uint32_t* rrem,
                            uint32_t* tl, uint32_t* tz, uint32_t* tr) {
  __shared__ uint32_t tn[kMaxTgt], gcnt;
  cand_round(keys, c, lo, hi, ranks, nt, lh, wsum, rbin, rrem);
  if (threadIdx.x == 0) {
    const uint32_t mult = bin_mult(lo, hi);
    for (int j = 0; j < nt; ++j) {
      bin_interval(rbin[j], lo, mult, lo, hi, tl[j], tz[j]);
      tr[j] = rrem[j];
      tn[j] = lh[rbin[j]];
    }
  }
  __syncthreads();
  uint32_t grank[kMaxTgt];
  int gidx[kMaxTgt];
  // gather-and-count: the keys of a small bin into LDS (lh reused), then each key's rank range
  for (int j = 0; j < nt; ++j) {
    if (!(tl[j] < tz[j] && tn[j] <= kGatherMax)) continue;
    const uint32_t l = tl[j], z = tz[j];
    int ng = 0;
    for (int k = j; k < nt; ++k)
      if (tl[k] == l && tz[k] == z) { gidx[ng] = k; grank[ng++] = tr[k]; }
    if (threadIdx.x == 0) gcnt = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < c; i += kBlock) {
      const uint32_t k = keys[i];
      if (k >= l && k <= z) {
        const uint32_t pos = atomicAdd(&gcnt, 1u);
        if (pos < kGatherMax) lh[pos] = k;
      }
    }
    __syncthreads();
    const uint32_t m = min(gcnt, kGatherMax);
    for (uint32_t i = threadIdx.x; i < m; i += kBlock) {
      const uint32_t k = lh[i];
      uint32_t less = 0, leq = 0;
      for (uint32_t q = 0; q < m; ++q) {
        const uint32_t v = lh[q];
        less += v < k ? 1u : 0u;
        leq += v <= k ? 1u : 0u;
      }
      for (int q = 0; q < ng; ++q)
        if (less <= grank[q] && grank[q] < leq) { tl[gidx[q]] = k; tz[gidx[q]] = k; }   // (equal keys: same value)
    }
    __syncthreads();
  }
  // narrow every unresolved target; targets sharing an interval (the adjacent ranks i0, i0 + 1 of
  // one percentile, usually) share each round
  for (int j = 0; j < nt; ++j) {
    for (int it = 0; it < 4 && tl[j] < tz[j]; ++it) {
      const uint32_t l = tl[j], z = tz[j];
      int ng = 0;
      for (int k = j; k < nt; ++k)
        if (tl[k] == l && tz[k] == z) { gidx[ng] = k; grank[ng++] = tr[k]; }
      cand_round(keys, c, l, z, grank, ng, lh, wsum, rbin, rrem);
      if (threadIdx.x == 0) {
        const uint32_t mult = bin_mult(l, z);
        for (int q = 0; q < ng; ++q) {
          bin_interval(rbin[q], l, mult, l, z, tl[gidx[q]], tz[gidx[q]]);
          tr[gidx[q]] = rrem[q];
        }
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) out[j] = tl[j];
  }
  __syncthreads();
}

// Speculative level-0 windows.  k_model_hist's full-resolution sample has the map's quantiles up
// to sampling noise: around the sample's bin of each quantile,
// a run of level-0 bins expected to hold about kWinKeys full-resolution keys becomes a window
// whose keys the level-0 sweep compacts.  When a target's bin lies inside a window (and the
// window did not overflow), the level-0 resolve selects the exact key from those candidates
// and the later levels are no-ops; otherwise they run as usual.  Consumes histogram slot 3.
__global__ __launch_bounds__(kBlock) void k_window(SelState* st, const uint32_t* mhist, uint32_t cap, int B,
                                                   int enable, int m, int nch) {
  __shared__ __attribute__((aligned(16))) uint32_t mh[kBins];
  __shared__ uint32_t wsum[kBlock / 64], wb[6], tot, wtot[3];
  __shared__ double wlim[3];
  const int b = blockIdx.x;
  if (b >= B) return;
  SelState* S = st + b;
  // the sample histogram (8 bins per thread)
  uint32_t local = 0;
  {
    static_assert(kBins == 8 * kBlock, "k_window: 8 bins per thread");
    const uint4* src = reinterpret_cast<const uint4*>(mhist + (size_t)b * kBins) + 2 * threadIdx.x;
    const uint4 acc0 = src[0], acc1 = src[1];
    reinterpret_cast<uint4*>(mh)[2 * threadIdx.x] = acc0;
    reinterpret_cast<uint4*>(mh)[2 * threadIdx.x + 1] = acc1;
    local = acc0.x + acc0.y + acc0.z + acc0.w + acc1.x + acc1.y + acc1.z + acc1.w;
  }
  if (threadIdx.x == 0) tot = 0;
  __syncthreads();
  local = wave_sum_u32(local);
  if ((threadIdx.x & 63) == 0) atomicAdd(&tot, local);
  __syncthreads();
  const uint32_t mtot = tot;
  if (!enable || mtot == 0) {
    if (threadIdx.x == 0) S->nwin = 0;
    return;
  }
  // window k = the bins whose cumulative model counts overlap [r_k - h, r_k + h]: model rank
  // r_k of the quantile, h = half the candidate budget in model counts
  const double scale = (double)S->n / (double)mtot;
  const double h = 0.5 * (double)kWinKeys / scale;
  const int per = kBins / kBlock;
  uint32_t seg = 0;
  for (int i = 0; i < per; ++i) seg += mh[threadIdx.x * per + i];
  uint32_t x = seg;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  // a sample holding NaN / Inf adds a window at its median (the nanmedian fill); m = samples
  const int nq = (uint32_t)m > mtot ? 3 : 2;
  if (threadIdx.x < 6) wb[threadIdx.x] = (threadIdx.x & 1) ? 0u : (uint32_t)kBins;
  __syncthreads();
  uint32_t off = 0;
  for (int i = 0; i < wv; ++i) off += wsum[i];
  double cum = (double)(x + off - seg);   // exclusive prefix of this thread's first bin
  // half-width of window k in sample counts: the candidate budget, but at least 4.5 standard
  // deviations of the sample's rank of the quantile (large images: a sample point stands for
  // hundreds of keys), at most 0.8 of a candidate list
  double hks[3];
  for (int k = 0; k < nq; ++k) {
    const double q = k == 0 ? 0.02 : (k == nq - 1 ? 0.98 : 0.5);
    hks[k] = fmin(fmax(h, 4.5 * sqrt((double)mtot * q * (1.0 - q)) + 1.0), 0.4 * (double)cap / scale);
  }
  for (int k = 0; k < nq; ++k) {
    const double q = k == 0 ? 0.02 : (k == nq - 1 ? 0.98 : 0.5);
    const double r = floor((double)(mtot - 1) * q);
    const double hk = hks[k];
    double c = cum;
    for (int i = 0; i < per; ++i) {
      const int bn = threadIdx.x * per + i;
      const double c1 = c + mh[bn];
      // every bin overlapping the rank's uncertainty interval; one that alone outgrows the window (a
      // spike such as the zero floor) can only sit at an end of it, where it is flagged below and
      // counted with its min / max key.  (r04 left such a bin out unless the SAMPLE's rank fell in
      // it: C2 image 5, whose ReLU floor holds 2.0x % of the pixels, had the sample's p2 rank just
      // above the floor and the image's just inside it -- a rank outside every window, so the
      // selection from scratch on every call, +0.64 ms per C2 step.)
      if (c1 > r - hk && c <= r + hk) { atomicMin(&wb[2 * k], (uint32_t)bn); atomicMax(&wb[2 * k + 1], (uint32_t)bn); }
      c = c1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // ascending windows; overlapping neighbours merge (touching ones stay apart, so a spike
    // bin stays at a window's end)
    uint32_t w[6];
    double lim[3];                   // spike limit of each window: more samples than its full width
    int nw = 0;
    for (int k = 0; k < nq; ++k) {
      const uint32_t lo = wb[2 * k], hi = wb[2 * k + 1];
      if (lo > hi) continue;
      if (nw > 0 && lo <= w[2 * nw - 1]) {
        w[2 * nw - 1] = max(w[2 * nw - 1], hi);
        lim[nw - 1] = fmax(lim[nw - 1], 2.0 * hks[k]);
      } else {
        w[2 * nw] = lo;
        w[2 * nw + 1] = hi;
        lim[nw] = 2.0 * hks[k];
        ++nw;
      }
    }
    for (int i = 0; i < 2 * nw; ++i) S->wbin[i] = w[i];
    S->nwin = (uint32_t)nw;
    for (int i = 0; i < 2 * nw; ++i) wb[i] = w[i];
    for (int k = 0; k < nw; ++k) wlim[k] = lim[k];
    for (int k = 0; k < 3; ++k) wtot[k] = 0;
    tot = (uint32_t)nw;
  }
  __syncthreads();
  // each window's sample count (the bins of a thread, added per window)
  for (int k = 0; k < (int)tot; ++k) {
    uint32_t part = 0;
    for (int i = 0; i < per; ++i) {
      const uint32_t bn = (uint32_t)(threadIdx.x * per + i);
      if (bn >= wb[2 * k] && bn <= wb[2 * k + 1]) part += mh[bn];
    }
    part = wave_sum_u32(part);
    if ((threadIdx.x & 63) == 0 && part) atomicAdd(&wtot[k], part);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // end bins expected to outgrow the window budget (the zero floor of a ReLU head, a saturated
    // maximum): counted with their min / max key by k_sweep_w instead of compacted; a window
    // holds such a bin only at an end (a bin larger than the window cannot have neighbours on
    // both sides within the rank budget).  Beyond a bin larger than the budget alone (lim: twice
    // the half-width, at most 0.8 of a candidate list), a window whose compacted part would still
    // exceed the budget has its larger remaining end bin split off too, when that bin holds at
    // least a quarter of the budget: r05, a DPT-Large map whose ReLU zero floor (a bin holding the
    // p2 rank itself, so kept in the window) was just under the budget while its neighbours brought
    // the window past the list capacity -- the list overflowed and the image went to the selection
    // from scratch every call (+0.64 ms per C2 step).
    for (int k = 0; k < (int)tot; ++k) {
      const uint32_t lo = wb[2 * k], hi = wb[2 * k + 1];
      const double lk = wlim[k];
      uint32_t f = 0;
      if ((double)mh[lo] > lk) f |= 1u;
      if (hi > lo && (double)mh[hi] > lk) f |= 2u;
      double rest = (double)wtot[k] - ((f & 1u) ? (double)mh[lo] : 0.0) - ((f & 2u) ? (double)mh[hi] : 0.0);
      for (int it = 0; it < 2 && rest > lk && hi > lo; ++it) {
        const double cl = (f & 1u) ? -1.0 : (double)mh[lo], ch = (f & 2u) ? -1.0 : (double)mh[hi];
        const bool take_lo = cl >= ch;
        const double c = take_lo ? cl : ch;
        if (c < 0.25 * lk) break;
        f |= take_lo ? 1u : 2u;
        rest -= c;
      }
      S->wspike[k] = f;
    }
  }
  __syncthreads();
  // the windows as values for k_sweep_w: the first / last finite key of the window's bins, and of
  // its first bin's end / last bin's start (spike split).  Each is the smallest finite key whose
  // level-0 bin reaches a target (vbin is monotone in the key): a 64-way search per wave (each
  // round every lane tests one key, the range shrinks 64x), searches spread over the waves.
  const int nw = (int)tot;
  const VBins vb = level0_vbins(S->rlo, S->rhi);
  const uint64_t clo = kKeyNegInf + 1u, chi = kKeyPosInf - 1u;
  for (int sidx = wv; sidx < 4 * nw; sidx += kBlock / 64) {
    const int k = sidx >> 2, kind = sidx & 3;
    const uint32_t lo = wb[2 * k], hi = wb[2 * k + 1];
    const uint32_t target = kind == 0 ? lo : (kind == 1 ? hi + 1u : (kind == 2 ? lo + 1u : hi));
    uint64_t a = clo, z = chi + 1;       // answer in [a, z]; z = chi + 1: no finite key reaches target
    while (a < z) {
      const uint64_t step = (z - a + 63) >> 6;
      const uint64_t q = a + (uint64_t)lane * step;
      const bool hit = q < z && vbin(key2f((uint32_t)q), vb) >= target;
      const uint64_t m = __ballot(hit);
      if (!m) {                          // every tested key short: past the last one tested
        a += min<uint64_t>(63, (z - a - 1) / step) * step + 1;
      } else {
        const int f = __ffsll((unsigned long long)m) - 1;
        const uint64_t qf = a + (uint64_t)f * step;
        if (f == 0) z = a;               // (a itself reaches the target)
        else { a = a + (uint64_t)(f - 1) * step + 1; z = qf; }
      }
    }
    // a: smallest finite key with vbin >= target (chi + 1 if none)
    const uint32_t key = (kind == 1 || kind == 2) ? (uint32_t)(a - 1) : (uint32_t)a;   // (kKeyPosInf: +inf)
    if (lane == 0) {
      const float v = key2f(key);
      if (kind == 0) S->wvlo[k] = v;
      if (kind == 1) S->wvhi[k] = v;
      if (kind == 2) S->wvF[k] = v;
      if (kind == 3) S->wvL[k] = v;
    }
  }
}

// Targets of a map holding NaN / +-Inf (app.py:194-197: np.nanmedian of the non-NaN values,
// then np.percentile of the map with every non-finite value replaced by it), all as order
// statistics of the FINITE keys F, known right after level 0 (k = non-finite count):
//   non-NaN sorted    = [-inf x nneg] + F + [+inf x npos]           -> median targets 8, 9
//   filled map sorted = [F < med] + [med x (#F == med + k)] + [F > med]
// so the filled map's rank-r value is F_(r) if F_(r) < med, else F_(r-k) if F_(r-k) > med,
// else med: targets t = F_(r_t) and 4 + t = F_(r_t - k) for the four percentile ranks.
// Ranks outside F are resolved at once to the +-inf keys (they never win those tests).
__device__ void fill_targets(SelState& s, bool drop_unread = false) {
  const uint32_t n = s.n, k = s.nonfinite_count, nfin = n - k, nneg = s.ninf_neg;
  uint32_t r[4];
  pct_ranks(n, r);
  auto set = [&](int t, int64_t j) {      // F rank j, or a resolved +-inf sentinel
    if (j < 0) { s.tlo[t] = s.thi[t] = kKeyNegInf; s.tslot[t] = kNoSlot; return; }
    if (j >= (int64_t)nfin) { s.tlo[t] = s.thi[t] = kKeyPosInf; s.tslot[t] = kNoSlot; return; }
    s.rank[t] = (uint32_t)j;
    s.tlo[t] = 0;
    s.thi[t] = 0xffffffffu;
    s.tslot[t] = 0;
  };
  for (int t = 0; t < 4; ++t) {
    set(t, (int64_t)r[t]);
    set(4 + t, (int64_t)r[t] - (int64_t)k);
  }
  const uint32_t m = n - s.nan_count, hm = m / 2;
  s.med_ranks = (m & 1u) ? 1u : 2u;
  const uint32_t g[2] = {s.med_ranks == 1 ? hm : hm - 1, hm};
  for (int i = 0; i < 2; ++i) {
    if (g[i] < nneg) set(8 + i, -1);
    else if (g[i] >= nneg + nfin) set(8 + i, (int64_t)nfin);
    else set(8 + i, (int64_t)(g[i] - nneg));
  }
  // Only one of a percentile's pair is ever read (finish_targets: F(r) < med ? F(r) : max(F(r-k),
  // med)), and which one follows from the ranks alone when the median is finite: below the lower
  // median rank F(r) <= med, so the value is F(r) (at F(r) == med the twin gives med too); above
  // the upper one F(r) >= med, so it is max(F(r-k), med).  The other target is marked resolved
  // with a key that sends finish_targets the right way, so it needs no window: with a few %
  // non-finite pixels the unused twin sits k ranks away from every window and used to send the
  // whole image to k_sel_slow's selection from scratch (~5 ms for 32 x 1024^2 at 0.1 % NaN pixels).
  // Window paths only (drop_unread): the histogram levels group targets by bin and keep them all.
  // The argument needs a FINITE median: np.mean of two middle values near +-FLT_MAX overflows to
  // +-inf, and then F(r) above the upper rank compares below med after all.  fill = 2 records that
  // targets were dropped; finish_targets refuses such an image when med is not finite, and it goes
  // to the selection from scratch.
  bool dropped = false;
  if (drop_unread && g[0] >= nneg && g[1] < nneg + nfin) {
    const int64_t lo = (int64_t)(g[0] - nneg), hi = (int64_t)(g[1] - nneg);
    for (int t = 0; t < 4; ++t) {
      if ((int64_t)r[t] < lo && s.tlo[4 + t] != s.thi[4 + t]) {            // the twin is never read
        s.tlo[4 + t] = s.thi[4 + t] = kKeyNegInf;
        s.tslot[4 + t] = kNoSlot;
        dropped = true;
      } else if ((int64_t)r[t] > hi && s.tlo[t] != s.thi[t]) {             // F(r) only compares >= med
        s.tlo[t] = s.thi[t] = kKeyPosInf;
        s.tslot[t] = kNoSlot;
        dropped = true;
      }
    }
  }
  s.ntgt = kMaxTgt;
  s.fill = dropped ? 2 : 1;
}

// All targets resolved: p2 / p98 (and their branch) from the target keys (false: the
// min / max branch without have_mm -- finalize_pct).
__device__ bool finish_targets(SelState& s, bool have_mm = true) {
  if (!s.fill) return finalize_pct(s, s.tlo, have_mm);
  const float a = key2f(s.tlo[8]), c = key2f(s.tlo[9]);
  const float med = s.med_ranks == 1 ? a : (a + c) / 2.0f;   // np.mean of the middle pair in float32
  s.med = med;
  s.has_med = 1;
  if (isnan(med)) {   // e.g. median of {-inf, +inf}: the filled map has NaNs -> np.percentile is NaN
    s.mode = 2;
    s.p2 = s.p98 = (double)med;
    s.phase = PH_DONE;
    return true;
  }
  if (s.fill == 2 && !isfinite(med)) {   // dropped targets assumed a finite median (fill_targets)
    s.err = 1;
    return false;
  }
  const uint32_t mk = f2key(med);
  uint32_t pk[4];
  for (int t = 0; t < 4; ++t) pk[t] = s.tlo[t] < mk ? s.tlo[t] : (s.tlo[4 + t] > mk ? s.tlo[4 + t] : mk);
  s.kmin = min(s.kmin, mk);            // min / max of the filled map (app.py:198-199 branch)
  s.kmax = max(s.kmax, mk);
  return finalize_pct(s, pk, have_mm);
}

// One resolve per level (a workgroup per image): histogram slots -> the bin of each target
// (its key interval narrows ~2048x), compaction slots -> the exact key; then the next
// level's slots (compaction when the interval holds <= cap keys and `compact` is set).
template <int LEVEL>
__global__ __launch_bounds__(kBlock) void k_resolve(SelState* st, uint32_t* hist, const uint32_t* cand, uint32_t cap,
                                                    int B, int compact) {
  __shared__ uint32_t lh[kBins];
  __shared__ uint32_t ck[kLdsCand];
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ uint32_t rbin[kMaxTgt], rrem[kMaxTgt], tcnt[kMaxTgt], qr[kMaxTgt], qk[kMaxTgt], tl[kMaxTgt],
      tz[kMaxTgt], tr[kMaxTgt], tbin[kMaxTgt];
  __shared__ SelState s;
  const int b = blockIdx.x;
  if (b >= B) return;
  if (threadIdx.x == 0) s = st[b];
  __syncthreads();
  if (s.phase != (LEVEL == 0 ? PH_INIT : PH_SEL)) return;
  uint32_t* gh = hist + (size_t)b * kSlots * kBins;
  uint32_t clo[kSlots], chi[kSlots];
  if (threadIdx.x == 0) s.level = LEVEL;
  if (LEVEL == 0) {
    __syncthreads();
    if (threadIdx.x == 0) {
      s.nslot = 1;
      s.slo[0] = 0;                      // (level 0 bins values: vbin / vbin_interval)
      s.smult[0] = 0;
      s.smode[0] = SM_HIST;
      if (s.nonfinite_count == 0) {
        pct_ranks(s.n, s.rank);
        s.ntgt = 4;
        for (int t = 0; t < 4; ++t) s.tslot[t] = 0;
      } else if (s.nan_count == s.n) {   // all-NaN: nanmedian is NaN, every value stays NaN
        s.has_med = 1;
        s.mode = 2;
        s.p2 = s.p98 = (double)__uint_as_float(0x7fc00000u);
        s.phase = PH_DONE;
      } else {
        fill_targets(s);
      }
    }
    __syncthreads();
    if (s.phase != PH_INIT) {
      for (int i = threadIdx.x; i < kBins; i += kBlock) gh[i] = 0;
      if (threadIdx.x == 0) st[b] = s;
      return;
    }
    clo[0] = s.kmin;
    chi[0] = s.kmax;
  } else {
    for (int q = 0; q < kSlots; ++q) { clo[q] = s.slo[q]; chi[q] = s.shi[q]; }
    bool overflow = false;
    for (int q = 0; q < (int)s.nslot; ++q) overflow |= s.smode[q] == SM_COMPACT && s.ccount[q] > cap;
    if (overflow) {      // (cannot happen: the counts come from the previous histogram)
      __syncthreads();
      if (threadIdx.x == 0) { s.phase = PH_SLOW; st[b] = s; }
      return;
    }
  }
  for (int q = 0; q < (int)s.nslot; ++q) {
    // the targets swept in slot q (every thread builds the same list)
    int nq = 0, tq[kMaxTgt];
    for (int t = 0; t < (int)s.ntgt; ++t)
      if (s.tslot[t] == (uint32_t)q) tq[nq++] = t;
    if (nq == 0) continue;
    if (threadIdx.x < nq) qr[threadIdx.x] = s.rank[tq[threadIdx.x]];
    if (threadIdx.x < kMaxTgt) { rbin[threadIdx.x] = 0; rrem[threadIdx.x] = 0; }
    __syncthreads();
    if (s.smode[q] == SM_HIST) {
      dma_words(lh, gh + q * kBins, kBins);     // the slot's histogram into LDS
      find_bins(lh, kBins, qr, nq, wsum, rbin, rrem);
      if (threadIdx.x == 0) {
        for (int k = 0; k < nq; ++k) {
          const int t = tq[k];
          tcnt[t] = lh[rbin[k]];
          tbin[t] = rbin[k];
          if (LEVEL == 0) vbin_interval(rbin[k], level0_vbins(s.rlo, s.rhi), clo[q], chi[q], s.tlo[t], s.thi[t]);
          else bin_interval(rbin[k], s.slo[q], s.smult[q], clo[q], chi[q], s.tlo[t], s.thi[t]);
          s.rank[t] = rrem[k];
        }
        if (LEVEL >= 1 && LEVEL < kLastLevel && nq > 1) {
          // unresolved targets of this slot whose bins lie within kBins keys of each other share
          // the level-2 slot (one key per bin there, so it resolves them all): the group's
          // interval spans their bins, ranks re-based by the counts of the bins before them
          int ord[kMaxTgt], no = 0;
          for (int k = 0; k < nq; ++k)
            if (s.tlo[tq[k]] != s.thi[tq[k]]) ord[no++] = k;
          for (int i = 1; i < no; ++i)
            for (int j = i; j > 0 && rbin[ord[j]] < rbin[ord[j - 1]]; --j) { const int x = ord[j]; ord[j] = ord[j - 1]; ord[j - 1] = x; }
          for (int i = 0; i < no;) {
            const int t0 = tq[ord[i]];
            const uint32_t glo = s.tlo[t0];
            int e = i + 1;
            while (e < no && (uint64_t)s.thi[tq[ord[e]]] - glo + 1 <= (uint64_t)kBins) ++e;
            if (e - i > 1) {
              const uint32_t b0 = rbin[ord[i]], ghi = s.thi[tq[ord[e - 1]]];
              uint32_t below = 0, bcur = b0;
              for (int j = i; j < e; ++j) {
                const int t = tq[ord[j]];
                for (; bcur < rbin[ord[j]]; ++bcur) below += lh[bcur];
                s.rank[t] = below + rrem[ord[j]];
                s.tlo[t] = glo;
                s.thi[t] = ghi;
              }
              uint32_t cnt = below;
              for (; bcur <= rbin[ord[e - 1]]; ++bcur) cnt += lh[bcur];
              for (int j = i; j < e; ++j) tcnt[tq[ord[j]]] = cnt;
            }
            i = e;
          }
        }
      }
    } else {
      const uint32_t c = s.ccount[q];
      const uint32_t* keys = cand + ((size_t)b * kSlots + q) * cap;
      if (c <= (uint32_t)kLdsCand) {
        dma_words(ck, keys, c);
        keys = ck;
        __syncthreads();
      }
      cand_select(keys, c, s.slo[q], s.shi[q], qr, nq, qk, lh, wsum, rbin, rrem, tl, tz, tr);
      if (threadIdx.x == 0) {
        for (int k = 0; k < nq; ++k) {
          const int t = tq[k];
          s.tlo[t] = s.thi[t] = qk[k];
          s.rank[t] = 0;
        }
      }
    }
    __syncthreads();
  }
  if (LEVEL == 0 && s.nwin > 0) {
    // targets whose level-0 bin lies in a k_window window: exact key from its candidates
    for (int t = 0; t < (int)s.ntgt; ++t) {
      if (s.tlo[t] == s.thi[t]) continue;
      int w = -1;
      for (int k = 0; k < (int)s.nwin; ++k)
        if (tbin[t] >= s.wbin[2 * k] && tbin[t] <= s.wbin[2 * k + 1]) w = k;
      if (w < 0 || s.ccount[w] > cap) continue;
      // the unresolved targets of the same bin go together
      int ng = 0, tg[kMaxTgt];
      for (int u = t; u < (int)s.ntgt; ++u)
        if (s.tlo[u] != s.thi[u] && tbin[u] == tbin[t]) tg[ng++] = u;
      if (threadIdx.x < ng) qr[threadIdx.x] = s.rank[tg[threadIdx.x]];
      const uint32_t c = s.ccount[w];
      const uint32_t* keys = cand + ((size_t)b * kSlots + w) * cap;
      if (c <= (uint32_t)kLdsCand) {
        dma_words(ck, keys, c);
        keys = ck;
      }
      __syncthreads();
      cand_select(keys, c, s.tlo[t], s.thi[t], qr, ng, qk, lh, wsum, rbin, rrem, tl, tz, tr);
      if (threadIdx.x == 0) {
        for (int k = 0; k < ng; ++k) {
          s.tlo[tg[k]] = s.thi[tg[k]] = qk[k];
          s.rank[tg[k]] = 0;
        }
      }
      __syncthreads();
    }
  }
  // consumed histograms -> zero for the next level
  for (int i = threadIdx.x; i < (int)s.nslot * kBins; i += kBlock) gh[i] = 0;
  if (threadIdx.x == 0) {
    // unresolved targets -> next level's slots (targets with equal intervals share one)
    int nslot = 0;
    bool all = true;
    for (int t = 0; t < (int)s.ntgt; ++t) {
      if (s.tlo[t] == s.thi[t]) { s.tslot[t] = kNoSlot; continue; }
      all = false;
      int found = -1;
      for (int q = 0; q < nslot; ++q)
        if (s.slo[q] == s.tlo[t] && s.shi[q] == s.thi[t]) found = q;
      if (found < 0) {
        if (nslot == kSlots) { s.phase = PH_SLOW; break; }   // more distinct intervals than slots
        found = nslot++;
        s.slo[found] = s.tlo[t];
        s.shi[found] = s.thi[t];
        s.smult[found] = bin_mult(s.tlo[t], s.thi[t]);
        s.smode[found] = (compact && tcnt[t] <= cap) ? SM_COMPACT : SM_HIST;
        s.ccount[found] = 0;
      }
      s.tslot[t] = (uint32_t)found;
    }
    s.nslot = (uint32_t)nslot;
    if (s.phase != PH_SLOW) {
      if (all) finish_targets(s);
      else s.phase = LEVEL == kLastLevel ? PH_SLOW : PH_SEL;   // (a last-level interval is one key wide)
    }
    st[b] = s;
  }
}

// Window-only resolve (after k_sweep_w): workgroup = (image b, window w).  Every workgroup of an
// image derives the same targets (the four percentile ranks, or with NaN / Inf the ten fill
// targets -- fill_targets); the workgroup of window w resolves the targets whose rank among the
// finite keys falls inside w:
//   rank r' = rank - (finite keys below w), the window's keys ordered [first bin | compacted | last bin]
//   (bins are key intervals, ascending): a spike end bin resolves when it holds one key (min ==
//   max), the compacted part by exact selection among its candidates (cand_select).
// Anything else (a rank outside every window, a multi-key spike, an overflowed candidate list)
// sets the image's err flag: k_sel_slow then selects it from scratch.  Window 0's workgroup
// also stores the target bookkeeping k_sel_slow's finish needs.
// wave 0: the image's kBelowSlots below-window partial counts of k_sweep_w summed into dst[3]
__device__ __forceinline__ void sum_below(const uint32_t* wpart, int b, uint32_t* dst) {
  if (threadIdx.x < 64) {
    const uint4 v = threadIdx.x < kBelowSlots
                        ? *reinterpret_cast<const uint4*>(wpart + ((size_t)b * kBelowSlots + threadIdx.x) * 4)
                        : make_uint4(0, 0, 0, 0);
    const uint32_t a = wave_sum_u32(v.x), c = wave_sum_u32(v.y), d = wave_sum_u32(v.z);
    if (threadIdx.x == 0) { dst[0] = a; dst[1] = c; dst[2] = d; }
  }
}

__global__ __launch_bounds__(kBlock) void k_resolve_w(SelState* st, const uint32_t* cand, uint32_t cap, int B,
                                                      const uint32_t* wpart) {
  __shared__ uint32_t lh[kBins];
  __shared__ uint32_t ck[kLdsCand];
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ uint32_t rbin[kMaxTgt], rrem[kMaxTgt], qr[kMaxTgt], qk[kMaxTgt], tl[kMaxTgt], tz[kMaxTgt], tr[kMaxTgt];
  __shared__ int tq[kMaxTgt], nc;
  __shared__ uint32_t clo, chi, fail;
  __shared__ SelState s;
  const int b = blockIdx.x / 3, w = blockIdx.x % 3;
  if (b >= B) return;
  auto body = [&]() {
  if (threadIdx.x == 0) s = st[b];
  __syncthreads();
  sum_below(wpart, b, s.wbelow);
  __syncthreads();
  if (s.phase != PH_INIT) return;
  if (w > 0 && w >= (int)s.nwin) return;
  SelState* S = st + b;
  if (threadIdx.x == 0) {
    fail = 0;
    nc = 0;
    bool done = false;
    if (s.nonfinite_count == 0) {
      pct_ranks(s.n, s.rank);
      s.ntgt = 4;
      for (int t = 0; t < 4; ++t) { s.tlo[t] = 0; s.thi[t] = 0xffffffffu; }
    } else if (s.nan_count == s.n) {   // all-NaN: nanmedian is NaN, every value stays NaN
      if (w == 0) {
        S->has_med = 1;
        S->mode = 2;
        S->p2 = S->p98 = (double)__uint_as_float(0x7fc00000u);
        S->phase = PH_DONE;
      }
      done = true;
    } else {
      fill_targets(s, true);   // (+-inf sentinel and unread targets come back resolved: tlo == thi)
    }
    if (!done) {
      const uint32_t nwin = s.nwin;
      if (w == 0) {         // bookkeeping for k_sel_slow's finish
        S->ntgt = s.ntgt;
        S->fill = s.fill;
        S->med_ranks = s.med_ranks;
        for (int t = 0; t < (int)s.ntgt; ++t) {
          S->rank[t] = s.rank[t];
          if (s.tlo[t] == s.thi[t]) { S->tlo[t] = s.tlo[t]; S->thi[t] = s.thi[t]; }
        }
      }
      const uint32_t cF = (s.wspike[w] & 1u) ? s.wcntF[w] : 0u, cL = (s.wspike[w] & 2u) ? s.wcntL[w] : 0u;
      const uint32_t cC = s.ccount[w];
      const uint64_t bw = s.wbelow[w];
      for (int t = 0; t < (int)s.ntgt; ++t) {
        if (s.tlo[t] == s.thi[t]) continue;
        const uint64_t r = s.rank[t];
        int in = -1;
        for (uint32_t k = 0; k < nwin; ++k) {
          const uint64_t lo = s.wbelow[k];
          const uint64_t cnt = (uint64_t)((s.wspike[k] & 1u) ? s.wcntF[k] : 0u) + s.ccount[k] +
                               ((s.wspike[k] & 2u) ? s.wcntL[k] : 0u);
          if (r >= lo && r < lo + cnt) in = (int)k;
        }
        if (in < 0) { if (w == 0) fail = 1; continue; }
        if (in != w) continue;
        const uint64_t rp = r - bw;
        if (rp < cF) {
          if (s.wminF[w] == s.wmaxF[w]) { S->tlo[t] = S->thi[t] = s.wminF[w]; } else fail = 1;
        } else if (rp < (uint64_t)cF + cC) {
          if (cC > cap) { fail = 1; continue; }
          qr[nc] = (uint32_t)(rp - cF);
          tq[nc++] = t;
        } else {
          if (s.wminL[w] == s.wmaxL[w]) { S->tlo[t] = S->thi[t] = s.wminL[w]; } else fail = 1;
        }
      }
    } else {
      nc = 0;
    }
  }
  __syncthreads();
  if (fail) atomicOr(&S->err, 1u);     // (every thread: the same word, same value)
  if (nc == 0 || fail) return;
  const uint32_t c = s.ccount[w];
  const uint32_t* keys = cand + ((size_t)b * kSlots + w) * cap;
  if (c <= (uint32_t)kLdsCand) {
    dma_words(ck, keys, c);
    keys = ck;
  }
  // the candidates' key range (the interval cand_select narrows)
  {
    uint32_t mn = 0xffffffffu, mx = 0u;
    for (uint32_t i = threadIdx.x; i < c; i += kBlock) { mn = min(mn, keys[i]); mx = max(mx, keys[i]); }
    mn = wave_min_u32(mn);
    mx = wave_max_u32(mx);
    if ((threadIdx.x & 63) == 0) { rbin[threadIdx.x >> 6] = mn; rrem[threadIdx.x >> 6] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int k = 1; k < kBlock / 64; ++k) { mn = min(mn, rbin[k]); mx = max(mx, rrem[k]); }
      clo = mn;
      chi = mx < mn ? mn : mx;
    }
  }
  __syncthreads();
  cand_select(keys, c, clo, chi, qr, nc, qk, lh, wsum, rbin, rrem, tl, tz, tr);
  if (threadIdx.x < nc) {
    const int t = tq[threadIdx.x];
    S->tlo[t] = S->thi[t] = qk[threadIdx.x];
  }
  };
  body();
}

// Pixels of rows [v0, v1) of image b, resampled as sample() (the cv2 taps), handed to f(val);
// thread-strided columns, one row at a time.
template <class F>
__device__ __forceinline__ void for_rows(const Geo& g, int b, int v0, int v1, F&& f) {
  const float* D = g.depth + (size_t)b * g.dh * g.dw;
  for (int v = v0; v < v1; ++v) {
    if (g.same) {
      for (int u = threadIdx.x; u < g.W; u += kSlowBlock) f(D[(size_t)v * g.dw + u]);
      continue;
    }
    const Tap ty = g.yt[v];
    const float* r0 = D + (size_t)ty.i0 * g.dw;
    const float* r1 = D + (size_t)ty.i1 * g.dw;
    for (int u = threadIdx.x; u < g.W; u += kSlowBlock) {
      const Tap tx = g.xt[u];
      float h0, h1;
      if (tx.i1 < 0) {
        h0 = r0[tx.i0];
        h1 = r1[tx.i0];
      } else {
        h0 = r0[tx.i0] * tx.w0 + r0[tx.i1] * tx.w1;
        h1 = r1[tx.i0] * tx.w0 + r1[tx.i1] * tx.w1;
      }
      f(h0 * ty.w0 + h1 * ty.w1);
    }
  }
}

// A workgroup's share of a grid-wide pass is published (its atomics / stores done: every wave's
// vmcnt(0), the barrier, one agent release), then it takes the image's ticket; true in the one
// workgroup that arrives last, which then acquires (cdna_hip_programming.md Guideline 16).
__device__ __forceinline__ bool arrive_last(uint32_t* ticket, int P, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *flag = P == 1 || atomicAdd(ticket, 1u) == (uint32_t)(P - 1);
    if (*flag) {
      atomicExch(ticket, 0u);    // (every workgroup has arrived: the next pass reuses it)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return *flag != 0;
}

// The from-scratch selection's level resolve (the last arriving workgroup): every unresolved target
// t (tslot != kNoSlot) has its key prefix in tlo[t] and its rank among the F keys under that prefix
// in rank[t]; slot q of `hist` (global, nb bins each) holds the next `bits` key bits of the keys
// under prefix pre[q].  Narrows every target; returns the number still unresolved.
__device__ int scratch_resolve(SelState& s, const uint32_t* hist, int nb, int bits, const uint32_t* pre, int nslot,
                               bool last_level, uint32_t* lh, uint32_t* wsum, uint32_t* rb, uint32_t* rr) {
  __shared__ uint32_t trk[kMaxTgt];
  __shared__ int tq[kMaxTgt], ntq;
  for (int q = 0; q < nslot; ++q) {
    for (int i = threadIdx.x; i < nb; i += kSlowBlock) lh[i] = hist[q * nb + i];
    if (threadIdx.x == 0) {
      ntq = 0;
      for (int t = 0; t < (int)s.ntgt; ++t)
        if (s.tslot[t] != kNoSlot && s.tlo[t] == pre[q]) { tq[ntq] = t; trk[ntq++] = s.rank[t]; }
    }
    __syncthreads();
    find_bins<kSlowBlock>(lh, nb, trk, ntq, wsum, rb, rr);
    if (threadIdx.x == 0)
      for (int i = 0; i < ntq; ++i) {
        const int t = tq[i];
        s.tlo[t] = (s.tlo[t] << bits) | rb[i];
        s.rank[t] = rr[i];
        if (last_level) { s.thi[t] = s.tlo[t]; s.tslot[t] = kNoSlot; }
      }
    __syncthreads();
  }
  int open = 0;
  for (int t = 0; t < (int)s.ntgt; ++t) open += s.tslot[t] != kNoSlot ? 1 : 0;
  return open;
}

// Distinct prefixes of the unresolved targets (the level's histogram slots).
__device__ __forceinline__ int scratch_slots(const SelState& s, uint32_t* pre) {
  int n = 0;
  for (int t = 0; t < (int)s.ntgt; ++t) {
    if (s.tslot[t] == kNoSlot) continue;
    bool seen = false;
    for (int q = 0; q < n; ++q) seen |= pre[q] == s.tlo[t];
    if (!seen) pre[n++] = s.tlo[t];
  }
  return n;
}

// Grid: P workgroups per image (b = blockIdx.x / P).  Every workgroup of an image derives the same
// decision from st[b] (which only the image's last arriving workgroup writes, after all have read
// it):
//  1  finish from the resolved targets;
//  2  the near-constant branch (p98 <= p2: app.py:198-199 needs the map's min / max) with a range
//     k_sweep_w could not give (a band of a C4 run, a signed zero at an end): a grid-wide pass, each
//     workgroup a 1/P share of the rows, partial keys combined by agent-scope atomics;
//  0  the selection from scratch (a window missed, a spike or an overflowed list: err; the levels
//     path's PH_SLOW): level 0 here -- every workgroup counts its rows' NaN / +-inf pixels and
//     histograms their finite keys' top 11 bits; the last arriver places the targets (the four
//     percentile ranks, or fill_targets' ten order statistics of the finite keys with NaN / Inf)
//     and resolves their level-0 bins -- then k_scratch<1> / <2> narrow them over the grid too.
// (r04: one workgroup per image did passes 2 and 0: 833 us for 32 x 1024^2 near-constant maps, ~95 ms
// for one 8192 x 4096 panorama.)  slow[b] = {ticket, min key, max key, NaN, non-finite, -inf, +inf, -}
// and scr[b]'s level-0 histogram are reset by k_prepare.
__global__ __launch_bounds__(kSlowBlock) void k_sel_slow(Geo g, SelState* st, int B, int P, uint32_t* slow,
                                                          int swept_range, uint32_t* scr) {
  __shared__ uint32_t sh[kBins];
  __shared__ uint32_t wsum[kSlowBlock / 64], rb[kMaxTgt], rr[kMaxTgt], pre[kMaxTgt];
  __shared__ int done, last;
  __shared__ SelState s;
  const int b = blockIdx.x / P, part = blockIdx.x - (blockIdx.x / P) * P;
  if (b >= B) return;
  if (threadIdx.x == 0) {     // (usually done: only the phase is read)
    const uint32_t ph = st[b].phase;
    done = ph == PH_INIT || ph == PH_SLOW ? 0 : 1;
  }
  __syncthreads();
  if (done) return;
  if (threadIdx.x == 0) {
    s = st[b];
    done = 0;
    if (s.phase == PH_INIT && s.err == 0) {
      // window path (k_sweep_w / k_resolve_w): every target resolved unless err
      done = finish_targets(s, false) ? 1 : 0;
      // every target resolved, only the min / max branch's range is missing (p98 <= p2: a
      // constant or near-constant map)
      bool resolved = !done && s.err == 0;
      for (int t = 0; t < (int)s.ntgt; ++t) resolved = resolved && s.tlo[t] == s.thi[t];
      if (resolved) done = 2;
      // k_sweep_w counted the whole image's finite range (kmin / kmax) unless it flagged a signed zero
      // at an end of it, or the sweep covered a band only (swept_range = 0: C4 runs)
      if (resolved && swept_range && !(s.pad3[0] & 2u)) done = finish_targets(s, true) ? 1 : 0;
    }
  }
  __syncthreads();
  uint32_t* sl = slow + 8 * (size_t)b;
  const int v0 = (int)((int64_t)g.H * part / P), v1 = (int)((int64_t)g.H * (part + 1) / P);
  const int lane = threadIdx.x & 63;
  if (done == 2) {
    uint32_t lo = 0xffffffffu, hi = 0u;
    for_rows(g, b, v0, v1, [&](float val) {
      if (isfinite(val)) { const uint32_t k = f2key(val); lo = min(lo, k); hi = max(hi, k); }
    });
    lo = wave_min_u32(lo);
    hi = wave_max_u32(hi);
    if (lane == 0) {
      if (lo != 0xffffffffu) atomicMin(&sl[1], lo);
      if (hi) atomicMax(&sl[2], hi);
    }
  } else if (done == 0) {
    for (int i = threadIdx.x; i < kBins; i += kSlowBlock) sh[i] = 0;
    __syncthreads();
    uint32_t nnan = 0, nnf = 0, nneg = 0, npos = 0, lo = 0xffffffffu, hi = 0u;
    for_rows(g, b, v0, v1, [&](float val) {
      if (!isfinite(val)) {
        ++nnf;
        nnan += isnan(val) ? 1u : 0u;
        nneg += val == -INFINITY ? 1u : 0u;
        npos += val == INFINITY ? 1u : 0u;
        return;
      }
      const uint32_t k = f2key(val);
      lo = min(lo, k);
      hi = max(hi, k);
      atomicAdd(&sh[k >> 21], 1u);
    });
    nnan = wave_sum_u32(nnan); nnf = wave_sum_u32(nnf); nneg = wave_sum_u32(nneg); npos = wave_sum_u32(npos);
    lo = wave_min_u32(lo); hi = wave_max_u32(hi);
    if (lane == 0) {
      if (nnf) { atomicAdd(&sl[3], nnan); atomicAdd(&sl[4], nnf); atomicAdd(&sl[5], nneg); atomicAdd(&sl[6], npos); }
      if (lo != 0xffffffffu) atomicMin(&sl[1], lo);
      if (hi) atomicMax(&sl[2], hi);
    }
    __syncthreads();
    uint32_t* h0 = scr + (size_t)b * kScrWords;
    for (int i = threadIdx.x; i < kBins; i += kSlowBlock)
      if (sh[i]) atomicAdd(&h0[i], sh[i]);
  }
  if (!arrive_last(&sl[0], P, &last)) return;
  if (done == 1) {
    if (threadIdx.x == 0) st[b] = s;
    return;
  }
  if (done == 2) {
    if (threadIdx.x == 0) {
      const uint32_t lo = atomicMin(&sl[1], 0xffffffffu), hi = atomicMax(&sl[2], 0u);   // read at the coherence point
      s.kmin = min(s.kmin, lo);      // (with a fill, finish_targets already merged the median)
      s.kmax = max(s.kmax, hi);
      if (finish_targets(s, true)) {
        st[b] = s;
      } else {
        // Not reachable by finish_targets as it stands (the range was the only thing missing); should a
        // change ever make it so, the image is not left unresolved (no later launch of the chain takes
        // PH_SLOW) but finishes LOUDLY as the all-NaN map does: NaN median and percentiles, every point
        // NaN, stats p2 / p98 NaN -- never a silent output from stale selection state.
        s.err = 2;
        s.has_med = 1;
        s.mode = 2;
        s.med = __uint_as_float(0x7fc00000u);
        s.p2 = s.p98 = (double)s.med;
        s.phase = PH_DONE;
        st[b] = s;
      }
    }
    return;
  }
  // from scratch, level 0 resolved by this (last) workgroup
  if (threadIdx.x == 0) {
    s.level = kLevelScratch;          // diagnostics: this image's percentiles came from the fallback
    s.nan_count = atomicAdd(&sl[3], 0u);
    s.nonfinite_count = atomicAdd(&sl[4], 0u);
    s.ninf_neg = atomicAdd(&sl[5], 0u);
    s.ninf_pos = atomicAdd(&sl[6], 0u);
    s.kmin = atomicMin(&sl[1], 0xffffffffu);
    s.kmax = atomicMax(&sl[2], 0u);
    s.err = 0;
    s.has_med = 0;
    s.fill = 0;
    done = 0;
    if (s.nonfinite_count == 0) {
      uint32_t r[4];
      pct_ranks(s.n, r);
      s.ntgt = 4;
      for (int t = 0; t < 4; ++t) { s.rank[t] = r[t]; s.tslot[t] = 0; s.tlo[t] = 0; s.thi[t] = 0xffffffffu; }
    } else if (s.nan_count == s.n) {   // all-NaN: nanmedian is NaN, every value stays NaN
      s.has_med = 1;
      s.mode = 2;
      s.p2 = s.p98 = (double)__uint_as_float(0x7fc00000u);
      s.phase = PH_DONE;
      done = 1;
    } else {
      fill_targets(s, false);          // ten order statistics of the finite keys (tslot 0 = open)
      for (int t = 0; t < (int)s.ntgt; ++t) if (s.tslot[t] != kNoSlot) s.tlo[t] = 0;
    }
    pre[0] = 0;
  }
  __syncthreads();
  if (done) {
    if (threadIdx.x == 0) st[b] = s;
    return;
  }
  const int open = scratch_resolve(s, scr + (size_t)b * kScrWords, kBins, 11, pre, 1, false, sh, wsum, rb, rr);
  // the next level's histograms start from zero
  for (int i = threadIdx.x; i < kMaxTgt * kBins; i += kSlowBlock) scr[(size_t)b * kScrWords + kScrL1 + i] = 0;
  if (threadIdx.x == 0) {
    if (open) s.phase = PH_SCR1;
    else finish_targets(s, true);    // (every target was a +-inf sentinel)
    st[b] = s;
  }
}

// The from-scratch selection's radix levels 1 (key bits 20..10) and 2 (bits 9..0), grid-wide like
// k_sel_slow: each workgroup histograms its rows' finite keys under each open target's prefix, the
// last arriver narrows the targets (level 2: to the exact keys, then the finish).  Returns at once for
// an image in any other phase (one launch each in every selection chain).
template <int LEVEL>
__global__ __launch_bounds__(kSlowBlock) void k_scratch(Geo g, SelState* st, int B, int P, uint32_t* slow,
                                                         uint32_t* scr) {
  constexpr uint32_t PH = LEVEL == 1 ? PH_SCR1 : PH_SCR2;
  constexpr int NB = LEVEL == 1 ? kBins : 1024, MATCH = LEVEL == 1 ? 21 : 10, BSH = LEVEL == 1 ? 10 : 0;
  constexpr int BITS = LEVEL == 1 ? 11 : 10;
  __shared__ uint32_t lh[kMaxTgt * NB];
  __shared__ uint32_t wsum[kSlowBlock / 64], rb[kMaxTgt], rr[kMaxTgt], pre[kMaxTgt];
  __shared__ int go, nslot, last;
  __shared__ SelState s;
  const int b = blockIdx.x / P, part = blockIdx.x - (blockIdx.x / P) * P;
  if (b >= B) return;
  if (threadIdx.x == 0) go = st[b].phase == PH ? 1 : 0;
  __syncthreads();
  if (!go) return;
  if (threadIdx.x == 0) {
    s = st[b];
    nslot = scratch_slots(s, pre);
  }
  __syncthreads();
  const int ns = nslot;
  for (int i = threadIdx.x; i < ns * NB; i += kSlowBlock) lh[i] = 0;
  __syncthreads();
  const int v0 = (int)((int64_t)g.H * part / P), v1 = (int)((int64_t)g.H * (part + 1) / P);
  for_rows(g, b, v0, v1, [&](float val) {
    if (!isfinite(val)) return;
    const uint32_t k = f2key(val);
    for (int q = 0; q < ns; ++q)
      if ((k >> MATCH) == pre[q]) atomicAdd(&lh[q * NB + ((k >> BSH) & (NB - 1))], 1u);
  });
  __syncthreads();
  uint32_t* gh = scr + (size_t)b * kScrWords + (LEVEL == 1 ? kScrL1 : kScrL2);
  for (int i = threadIdx.x; i < ns * NB; i += kSlowBlock)
    if (lh[i]) atomicAdd(&gh[i], lh[i]);
  if (!arrive_last(&slow[8 * (size_t)b], P, &last)) return;
  const int open = scratch_resolve(s, gh, NB, BITS, pre, ns, LEVEL == 2, lh, wsum, rb, rr);
  if (LEVEL == 1)
    for (int i = threadIdx.x; i < kMaxTgt * 1024; i += kSlowBlock) scr[(size_t)b * kScrWords + kScrL2 + i] = 0;
  if (threadIdx.x == 0) {
    if (LEVEL == 1 && open) s.phase = PH_SCR2;
    else finish_targets(s, true);
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
  int proj;                      // 0 pinhole (app.py:216-238), 1 equirectangular (panoramas)
  const double* trig;            // equirectangular: [W] (sin, cos) of longitude, then [H] (sin, cos) of latitude
  int W;
};

__device__ __forceinline__ void project(double d, int v, int u, const Cam& c, float& x, float& y, float& z) {
  const double zd = d * c.scale;                       // app.py:233
  if (c.proj == 1) {
    // equirectangular panorama (not in the reference): the depth is the range along the ray
    // of longitude lon(u) = (u + 0.5) 2pi / W - pi, latitude lat(v) = pi / 2 - (v + 0.5) pi / H;
    // x right, y down, z forward (the pinhole axes at the panorama centre)
    const double slon = c.trig[2 * u], clon = c.trig[2 * u + 1];
    const double slat = c.trig[2 * c.W + 2 * v], clat = c.trig[2 * c.W + 2 * v + 1];
    const double rh = zd * clat;
    x = (float)(rh * slon);
    y = (float)(-(zd * slat));
    z = (float)(rh * clon);
    return;
  }
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

// Fast unprojection (no smoothing, N % 4 == 0, ceil(W/step) % 4 == 0, 3 channels):
// every load is unconditional (indices clamped, only the stores are predicated) so
// the compiler never parks a wave on a divergent vmcnt(0); the RGB of both point
// groups a thread owns is in flight before any arithmetic; cv2 taps are recomputed
// in registers (no table loads).
// bbox / stats of one image to float64 (the k_finalize work for image b)
__device__ __forceinline__ void write_final(const SelState& s, const uint32_t* bbox_key, int b, double* bbox,
                                            double* stats) {
  if (bbox)
    for (int k = 0; k < 6; ++k) bbox[b * 6 + k] = (double)key2f(bbox_key[k]);
  if (stats) {
    stats[b * 4 + 0] = s.p2;
    stats[b * 4 + 1] = s.p98;
    stats[b * 4 + 2] = (double)s.mode;
    stats[b * 4 + 3] = s.has_med ? (double)s.med : (double)__uint_as_float(0x7fc00000u);
  }
}

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
    stage_floats(rows, g.depth + ((size_t)b * g.dh + lo) * g.dw, (hi - lo + 1) * g.dw);
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

// Wave-uniform copies (SGPRs) of values every lane loaded from the same address: the branches
// on them become scalar and the fp64 constants stay out of VGPRs.
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ float uni(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }
__device__ __forceinline__ double uni(double x) {
  const uint64_t u = __double_as_longlong(x);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Row-sweep unprojection (fast path with a resized map): workgroup = image b x point rows
// [r0, r1) x one column tile of 4 * tpr points (tpr = threads per row, a multiple of 64, so a
// wave stays inside one row; kBlock / tpr rows per pass); thread t owns points 4c..4c+3
// (c = t % tpr) of the tile in rows r0 + t / tpr + k * (kBlock / tpr), so its x taps,
// (u - cx) and column offsets are computed once.  The model rows the
// block spans are staged in LDS and interpolated horizontally once (cv2's first pass, the
// right-border single tap copied exactly) into per-thread 16-B slots; a point then costs one
// 16-B LDS read per model row pair, the vertical blend, the nanmedian fill, the normalisation
// (uniform branch) and the projection.  RGB of the next row is in flight while a row is
// computed; each wave's 256 points leave through LDS as contiguous 1 KB / 256 B stores.
// Same arithmetic, in the same order, as k_unproject_fast / k_unproject (bit-identical).
constexpr int kRowsPT = 8;   // k_unproject_rows: point rows per thread and workgroup (rows_plan)

template <int STEP>
__global__ __launch_bounds__(kBlock) void k_unproject_rows(Geo g, const SelState* st, const uint8_t* img, int B,
                                                           Sweep sw, int invert, Cam cam, float* xyz, uint8_t* rgb,
                                                           SelState* stw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_u[];
  __shared__ uint32_t red[6][4];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int b, blk;
  map_rows(blockIdx.x, B, sw.nrb * sw.ntiles, b, blk);
  b = uni(b);
  const int rb = uni(blk / sw.ntiles), ct = uni(blk - (blk / sw.ntiles) * sw.ntiles);
  const SelState* S = st + b;
  Norm nm;
  nm.mode = uni(S->mode);
  nm.invert = invert;
  nm.p2 = uni(S->p2);
  nm.p98 = uni(S->p98);
  nm.den64 = uni(S->den64);
  nm.rden64 = uni(S->rden64);
  nm.lo32 = uni(S->lo32);
  nm.hi32 = uni(S->hi32);
  nm.den32 = uni(S->den32);
  const bool fill = uni((int)S->has_med) != 0;
  const float med = uni(S->med);
  const int Hn = cam.N / cam.Wn;
  const int r0 = sw.row0 + rb * sw.R;
  const int r1 = min(min(Hn, sw.row_end), r0 + sw.R);
  const int tpr = sw.tpr, rpp = kBlock / tpr;
  const int c0 = ct * 4 * tpr;
  const int ncol = min(4 * tpr, cam.Wn - c0);
  const int lo = ytap(g, r0 * STEP).i0;
  const int nrows = ytap(g, (r1 - 1) * STEP).i1 - lo + 1;
  // LDS: [horizontally interpolated rows: lds_rows x kBlock float4] then, in turn, the raw model
  // rows (until the horizontal pass is done) and each wave's store staging (rows_plan)
  float4* hrow = reinterpret_cast<float4*>(smem_u);   // [row][thread]
  float* raw = reinterpret_cast<float*>(hrow + sw.lds_rows * kBlock);
  float4* sx = reinterpret_cast<float4*>(raw) + wid * 192;                          // 3 KB per wave
  uint32_t* sc = reinterpret_cast<uint32_t*>(reinterpret_cast<float4*>(raw) + 4 * 192) + wid * 192;

  const int tcol = (int)threadIdx.x % tpr, trow = (int)threadIdx.x / tpr;
  const int t4 = 4 * tcol;
  const bool act = trow < rpp && t4 < ncol;
  const int ub = c0 + (act ? t4 : 0);                  // first point column of this thread
  const int rfirst = trow < rpp ? r0 + trow : r1;   // waves past rpp * tpr threads: idle
  const int nrt = rfirst < r1 ? (r1 - rfirst + rpp - 1) / rpp : 0;   // rows of this thread (<= kRowsPT)
  const size_t img_base = (size_t)b * g.H * g.W;
  // the BGR bytes of this thread's 4 points of a row as dwords: STEP 1 the 12 contiguous bytes;
  // STEP 2 the 24 bytes of image columns 2 ub .. 2 ub + 7 (point j at byte 6 j); STEP 4 one dword
  // per point (point j at byte 12 j) -- r04: the byte loads of STEP 2 / 4 (12 per row) and their
  // one-row prefetch left the medium-density kernel at 0.36 of HBM
  constexpr int NQ = STEP == 1 ? 3 : STEP == 2 ? 6 : 4;
  auto load_rgb = [&](int row, uint32_t (&q)[NQ]) {
    const int v = row * STEP;
    const uint32_t* p32 = reinterpret_cast<const uint32_t*>(img + (img_base + (size_t)v * g.W + (size_t)ub * STEP) * 3);
    if (STEP == 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) q[j] = p32[3 * j];
    } else {
#pragma unroll
      for (int d = 0; d < NQ; ++d) q[d] = p32[d];
    }
  };
  // the RGB of all of this thread's rows is requested first, so the HBM latency of the cold
  // image overlaps the model-row staging and the horizontal pass
  constexpr int PF = kRowsPT;
  uint32_t qa[PF][NQ];
#pragma unroll
  for (int k = 0; k < PF; ++k)
    if (k < nrt) load_rgb(rfirst + k * rpp, qa[k]);
  stage_floats(raw, g.depth + ((size_t)b * g.dh + lo) * g.dw, nrows * g.dw);
  __syncthreads();
  int ui[4];
  double du[4];
  Tap tx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ui[j] = (ub + j) * STEP;
    du[j] = (double)ui[j] - cam.cx;
    tx[j] = xtap(g, ui[j]);
  }
  // cv2's horizontal pass over the staged rows, this thread's four columns
  for (int r = 0; r < nrows; ++r) {
    const float* rr = raw + r * g.dw;
    float h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a0 = rr[tx[j].i0];
      h[j] = tx[j].i1 < 0 ? a0 : a0 * tx[j].w0 + rr[tx[j].i1] * tx[j].w1;
    }
    hrow[r * kBlock + threadIdx.x] = make_float4(h[0], h[1], h[2], h[3]);
  }
  __syncthreads();   // the raw rows are dead: their LDS becomes the store staging

  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int k = 0; k < kRowsPT; ++k) {
    if (k >= nrt) break;
    const int row = rfirst + k * rpp;
    const int v = row * STEP;
    const Tap ty = ytap(g, v);
    const float4 h0 = hrow[(ty.i0 - lo) * kBlock + threadIdx.x];
    const float4 h1 = hrow[(ty.i1 - lo) * kBlock + threadIdx.x];
    const float hv0[4] = {h0.x, h0.y, h0.z, h0.w}, hv1[4] = {h1.x, h1.y, h1.z, h1.w};
    const double dv = (double)v - cam.cy;
    uint32_t pc[4][3];   // [point][r,g,b] (source is BGR)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        if (STEP == 4) {
          pc[j][c] = (qa[k][j] >> (8 * (2 - c))) & 0xffu;
        } else {
          const int byte = 3 * STEP * j + (2 - c);
          pc[j][c] = (qa[k][byte >> 2] >> (8 * (byte & 3))) & 0xffu;
        }
      }
    float px[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float val = hv0[j] * ty.w0 + hv1[j] * ty.w1;
      if (fill && !isfinite(val)) val = med;
      const double d = normalize(val, nm);
      if (cam.proj == 1) {
        project(d, v, ui[j], cam, px[j][0], px[j][1], px[j][2]);
      } else {                                             // project(), pinhole, (u - cx) hoisted
        const double zd = d * cam.scale;
        const double zz = zd != 0.0 ? zd : 1e-6;
        px[j][0] = (float)div_rn(du[j] * zz, cam.f, cam.rf);
        px[j][1] = (float)div_rn(dv * zz, cam.f, cam.rf);
        px[j][2] = (float)zd;
      }
    }
    if (act) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 3; ++c) { mn[c] = fminf(mn[c], px[j][c]); mx[c] = fmaxf(mx[c], px[j][c]); }
    }
    // the wave's 256 consecutive points through LDS: contiguous 1 KB (xyz) / 256 B (rgb) stores
    float4* wx = sx;
    uint32_t* wc = sc;
    wx[lane * 3 + 0] = make_float4(px[0][0], px[0][1], px[0][2], px[1][0]);
    wx[lane * 3 + 1] = make_float4(px[1][1], px[1][2], px[2][0], px[2][1]);
    wx[lane * 3 + 2] = make_float4(px[2][2], px[3][0], px[3][1], px[3][2]);
    wc[lane * 3 + 0] = pc[0][0] | (pc[0][1] << 8) | (pc[0][2] << 16) | (pc[1][0] << 24);
    wc[lane * 3 + 1] = pc[1][1] | (pc[1][2] << 8) | (pc[2][0] << 16) | (pc[2][1] << 24);
    wc[lane * 3 + 2] = pc[2][2] | (pc[3][0] << 8) | (pc[3][1] << 16) | (pc[3][2] << 24);
    __builtin_amdgcn_wave_barrier();
    const int wp = (tcol >> 6) * 256;                          // first point of this wave in the tile
    const size_t o = (size_t)b * cam.N + (size_t)row * cam.Wn + c0 + wp;
    float4* dx = reinterpret_cast<float4*>(xyz + o * 3);
    uint32_t* dc = reinterpret_cast<uint32_t*>(rgb + o * 3);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int f = k * 64 + lane;
      if (wp + (f / 3) * 4 < ncol) {      // streamed once: non-temporal (sw.nt) or default policy
        const float4 vx = wx[f];
        if (sw.nt) {
          __builtin_nontemporal_store(vx.x, &dx[f].x);
          __builtin_nontemporal_store(vx.y, &dx[f].y);
          __builtin_nontemporal_store(vx.z, &dx[f].z);
          __builtin_nontemporal_store(vx.w, &dx[f].w);
          __builtin_nontemporal_store(wc[f], &dc[f]);
        } else {
          dx[f] = vx;
          dc[f] = wc[f];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  uint32_t kk[6];
  for (int c = 0; c < 3; ++c) {
    const bool any = mn[c] <= mx[c];
    kk[2 * c] = any ? f2key(mn[c]) : 0xffffffffu;
    kk[2 * c + 1] = any ? f2key(mx[c]) : 0u;
  }
  for (int c = 0; c < 6; ++c) {
    uint32_t x = (c & 1) ? wave_max_u32(kk[c]) : wave_min_u32(kk[c]);
    if (lane == 0) red[c][wid] = x;
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

// Smooth path (app.py:209-214): materialise the normalised field, blur, unproject.  The field
// is addressed as the whole image; a band run (C4) fills only image rows [r0, r1): its band
// plus the blur's halo, recomputed from the model-resolution depth every rank holds, so
// smoothing needs no exchange beyond the selection's.
__global__ void k_norm_field(Geo g, const SelState* st, int B, int invert, double* field, int r0, int r1) {
  const size_t n = (size_t)g.H * g.W;
  const size_t nr = (size_t)(r1 - r0) * g.W;
  const size_t total = nr * B;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / nr);
    const int p = (int)(i - (size_t)b * nr);
    const int v = r0 + p / g.W, u = p % g.W;
    const SelState* S = st + b;
    float val = sample(g, b, v, u);
    if (S->has_med && !isfinite(val)) val = S->med;
    field[(size_t)b * n + (size_t)v * g.W + u] = normalize(val, load_norm(S, invert));
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
// mode 0, float32 with float32 taps otherwise).  Output rows [r0, r1) of every image.
template <bool kRows>
__global__ void k_blur(const double* src, double* dst, const SelState* st, int B, int H, int W, BlurTaps taps,
                       int r0, int r1) {
  const size_t n = (size_t)H * W;
  const size_t nr = (size_t)(r1 - r0) * W;
  const size_t total = nr * B;
  const int r = taps.k / 2;
  for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < total; j += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(j / nr);
    const int p = (int)(j - (size_t)b * nr);
    const int v = r0 + p / W, u = p % W;
    const size_t i = (size_t)b * n + (size_t)v * W + u;
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

static int reflect101_host(int i, int n) {
  if (n == 1) return 0;
  while ((unsigned)i >= (unsigned)n) i = i < 0 ? -i : 2 * (n - 1) - i;
  return i;
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
  write_final(st[b], st[b].bbox_key, b, bbox, stats);
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
  sw.ntiles = 1;
  // allocate only the window R output rows can span (not the whole budget): occupancy
  if (cap_rows) cap_rows = std::min(cap_rows, (int)std::floor((double)(sw.R - 1) * step * dh / H) + 3);
  sw.lds_rows = cap_rows;
  return sw;
}

static size_t sweep_lds(const Sweep& sw, int dw) { return sw.lds_rows ? (size_t)sw.lds_rows * dw * sizeof(float) : 0; }

// k_unproject_rows knobs (I2PC_UNP_ROWS / _NT / _RPT, or i2pc_set_tuning "unp_rows" / "unp_nt" / "unp_rpt")
static int env_int(const char* name, int dflt) { const char* e = getenv(name); return e ? atoi(e) : dflt; }
static thread_local int g_unp_rows = env_int("I2PC_UNP_ROWS", 1);
static thread_local int g_unp_nt = env_int("I2PC_UNP_NT", 1);
static thread_local int g_unp_rpt = env_int("I2PC_UNP_RPT", kRowsPT);

// k_unproject_rows geometry: column tiles of 4 * tpr points (tpr a multiple of 64, <= kBlock),
// 8192 points per workgroup where the rows allow, LDS = staged model rows + one 16-B slot per
// thread and model row (<= 64 KiB; false: use k_unproject_fast).  I2PC_UNP_ROWS=0 disables it.
static bool rows_plan(int Hn, int step, int dh, int dw, int H, int Wn, int prow0, int prow1, Sweep& sr, size_t& lds) {
  const int enabled = g_unp_rows, nt = g_unp_nt, rpt = std::max(1, std::min(kRowsPT, g_unp_rpt));
  if (!enabled) return false;
  const int tpr = std::min(kBlock, (((std::min(Wn, 4 * kBlock) + 3) / 4 + 63) / 64) * 64);
  const int rpp = kBlock / tpr;
  int target = std::max(rpp, std::min(rpt * rpp, (8192 / (4 * tpr)) / rpp * rpp));
  for (; target >= 1; target = target > rpp ? target / 2 : target - rpp) {
    sr = plan_sweep(Hn, step, dh, dw, H, false, target, prow0, prow1);
    if (sr.lds_rows <= 0) return false;
    lds = (size_t)sr.lds_rows * kBlock * 16 +
          std::max(((size_t)sr.lds_rows * dw * sizeof(float) + 15) / 16 * 16, (size_t)(kBlock / 64) * 192 * 20);
    if (lds <= 64 * 1024) break;
  }
  if (target < 1 || lds > 64 * 1024) return false;
  sr.tpr = tpr;
  sr.nt = nt;
  sr.ntiles = (Wn + 4 * tpr - 1) / (4 * tpr);
  return true;
}

// Tile-parallel mode: the level-0 counters a sweep accumulates, out of / back into the
// per-image state, as int64 [4][B] = {nan counts, non-finite counts, min key, max key}
// (sum, sum, min, max across the bands).
__global__ void k_band_export(const SelState* st, int B, int64_t* ex) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    ex[b] = (int64_t)st[b].nan_count | ((int64_t)st[b].ninf_neg << 32);   // two sums in one row
    ex[B + b] = st[b].nonfinite_count;
    ex[2 * B + b] = st[b].kmin;
    ex[3 * B + b] = st[b].kmax;
  }
}
__global__ void k_band_import(SelState* st, int B, const int64_t* ex) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    st[b].nan_count = (uint32_t)(ex[b] & 0xffffffffll);
    st[b].ninf_neg = (uint32_t)(ex[b] >> 32);
    st[b].nonfinite_count = (uint32_t)ex[B + b];
    st[b].kmin = (uint32_t)ex[2 * B + b];
    st[b].kmax = (uint32_t)ex[3 * B + b];
  }
}

// Window-selection band runs (C4).  After k_sweep_w over its band, a rank holds its band's
// window keys (local candidate lists), below-window counts, spike counts and non-finite
// counts.  1) k_bandw_hist: per window a kBins-bin histogram of the local keys over the
// window's key range (the same range on every rank: the windows come from the whole image's
// sample) and the counters as int64 [4][kBandEx] (rows 0-1 SUM, row 2 MIN, row 3 MAX) -> one
// all-reduce.  2) k_bandw_pickc: from the SUMMED counts every rank derives the same targets and,
// for a target in a window's compacted part, its fine bin and its rank inside the bin; the local
// keys of that bin (count, min, max, up to kPick keys) go to the target's slot -> one all-gather.
// 3) k_bandw_final: each target's bin keys of every band merged, the exact key selected.
// A bin holding more than kPick keys in one band (and more than one distinct key), or a target
// outside every window, sets `err`: every rank then selects the whole image from scratch in
// k_sel_slow (identical decisions everywhere: the inputs are identical on every rank).
__device__ __forceinline__ void window_keys(const SelState& s, int w, uint32_t& k0, uint32_t& k1) {
  k0 = f2key(s.wvlo[w]);
  k1 = f2key(s.wvhi[w]);
  if (k1 < k0) k1 = k0;
}

constexpr int kBandSplit = 32;   // workgroups per window of the band histogram / compaction passes

__global__ __launch_bounds__(kBlock) void k_bandw_hist(const SelState* st, const uint32_t* cand, uint32_t cap,
                                                       uint32_t* hist, int64_t* ex, const uint32_t* wpart,
                                                       uint32_t* send) {
  __shared__ uint32_t lh[kBins];
  __shared__ uint32_t below[3];
  const int w = blockIdx.x % 3, j = blockIdx.x / 3;
  const SelState& s = st[0];
  if (blockIdx.x == 0) {
    sum_below(wpart, 0, below);
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int64_t* e = ex;
    e[0] = s.nonfinite_count; e[1] = s.nan_count; e[2] = s.ninf_neg; e[3] = s.ninf_pos;
    for (int q = 0; q < 3; ++q) {
      e[4 + q] = below[q];
      e[8 + q] = s.wcntF[q];
      e[11 + q] = s.wcntL[q];
      e[16 + q] = s.wminF[q];
      e[19 + q] = s.wminL[q];
      e[24 + q] = s.wmaxF[q];
      e[27 + q] = s.wmaxL[q];
    }
    // the bands' compacted counts (SUM) and whether any band's list overflowed (MAX): every rank
    // must take the same decision
    e[7] = s.ccount[0]; e[14] = s.ccount[1]; e[15] = s.ccount[2];
    e[22] = e[23] = 0xffffffffll;
    e[30] = (s.ccount[0] > cap || s.ccount[1] > cap || s.ccount[2] > cap) ? 1 : 0;
    e[31] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x < kMaxTgt) {   // target slot headers for k_bandw_pickc's atomics
    uint32_t* h = send + (size_t)threadIdx.x * kPickWords;
    h[0] = 0u;
    h[1] = 0xffffffffu;
    h[2] = 0u;
  }
  if (w >= (int)s.nwin) return;
  const uint32_t c = min(s.ccount[w], cap);
  const uint32_t i0 = (uint32_t)((uint64_t)c * j / kBandSplit), i1 = (uint32_t)((uint64_t)c * (j + 1) / kBandSplit);
  if (i0 == i1) return;
  for (int i = threadIdx.x; i < kBins; i += kBlock) lh[i] = 0;
  __syncthreads();
  uint32_t k0, k1;
  window_keys(s, w, k0, k1);
  const uint32_t mult = bin_mult(k0, k1);
  const uint32_t* keys = cand + (size_t)w * cap;
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kBlock) atomicAdd(&lh[bin_of(keys[i], k0, mult)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < kBins; i += kBlock)      // (hist zeroed by k_prepare)
    if (lh[i]) atomicAdd(&hist[(size_t)w * kBins + i], lh[i]);
}

// k_bandw_pickc: kBandSplit workgroups per window w.  Each places the targets from the summed
// counts (the same on every workgroup and rank) and finds its window's target fine bins; the
// first workgroup of the window records them in the state, and every workgroup appends the
// keys of those bins from its slice of the band's window keys to the target slots.
__global__ __launch_bounds__(kBlock) void k_bandw_pickc(SelState* st, const uint32_t* cand, uint32_t cap,
                                                        const uint32_t* hist, const int64_t* ex, uint32_t* send) {
  __shared__ SelState s;
  __shared__ uint32_t qr[kMaxTgt], rbin[kMaxTgt], rrem[kMaxTgt], wsum[kBlock / 64];
  __shared__ uint32_t sl[kMaxTgt], sz[kMaxTgt];
  __shared__ int tq[kMaxTgt], slot[kMaxTgt], nc, fail, nslot;
  __shared__ uint32_t ctot[3];
  const int w = blockIdx.x % 3, jw = blockIdx.x / 3;
  const bool rec = jw == 0;                // this workgroup records the window's targets
  SelState* S = st;
  if (threadIdx.x == 0) {
    s = st[0];
    const int64_t* e = ex;
    s.nonfinite_count = (uint32_t)e[0]; s.nan_count = (uint32_t)e[1];
    s.ninf_neg = (uint32_t)e[2]; s.ninf_pos = (uint32_t)e[3];
    for (int q = 0; q < 3; ++q) {
      s.wbelow[q] = (uint32_t)e[4 + q];
      s.wcntF[q] = (uint32_t)e[8 + q];
      s.wcntL[q] = (uint32_t)e[11 + q];
      s.wminF[q] = (uint32_t)e[16 + q];
      s.wminL[q] = (uint32_t)e[19 + q];
      s.wmaxF[q] = (uint32_t)e[24 + q];
      s.wmaxL[q] = (uint32_t)e[27 + q];
    }
    ctot[0] = (uint32_t)e[7]; ctot[1] = (uint32_t)e[14]; ctot[2] = (uint32_t)e[15];
    fail = e[30] ? 1 : 0;                // some band's list overflowed: its histogram is short
    nc = 0;
    nslot = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0 && !fail) {
    bool done = false;
    if (s.nonfinite_count == 0) {
      pct_ranks(s.n, s.rank);
      s.ntgt = 4;
      for (int t = 0; t < 4; ++t) { s.tlo[t] = 0; s.thi[t] = 0xffffffffu; }
    } else if (s.nan_count == s.n) {     // all-NaN: nanmedian is NaN, every value stays NaN
      if (w == 0 && rec) {
        S->has_med = 1;
        S->mode = 2;
        S->p2 = S->p98 = (double)__uint_as_float(0x7fc00000u);
        S->phase = PH_DONE;
      }
      done = true;
    } else {
      fill_targets(s, true);
    }
    if (!done) {
      if (w == 0 && rec) {
        S->ntgt = s.ntgt;
        S->fill = s.fill;
        S->med_ranks = s.med_ranks;
        S->nonfinite_count = s.nonfinite_count;
        S->nan_count = s.nan_count;
        for (int t = 0; t < (int)s.ntgt; ++t)     // (the others belong to their window's workgroup)
          if (s.tlo[t] == s.thi[t]) { S->tlo[t] = s.tlo[t]; S->thi[t] = s.thi[t]; S->tslot[t] = kNoSlot; }
      }
      const uint32_t nwin = s.nwin;
      for (int t = 0; t < (int)s.ntgt; ++t) {
        if (s.tlo[t] == s.thi[t]) continue;
        const uint64_t r = s.rank[t];
        int in = -1;
        for (uint32_t k = 0; k < nwin; ++k) {
          const uint64_t lo = s.wbelow[k];
          const uint64_t c = (uint64_t)((s.wspike[k] & 1u) ? s.wcntF[k] : 0u) + ctot[k] +
                             ((s.wspike[k] & 2u) ? s.wcntL[k] : 0u);
          if (r >= lo && r < lo + c) in = (int)k;
        }
        if (in < 0) { fail = 1; continue; }
        if (in != w) continue;
        const uint32_t cF = (s.wspike[w] & 1u) ? s.wcntF[w] : 0u;
        const uint64_t rp = r - s.wbelow[w];
        if (rp < cF) {
          if (s.wminF[w] != s.wmaxF[w]) fail = 1;
          else if (rec) { S->tlo[t] = S->thi[t] = s.wminF[w]; S->tslot[t] = kNoSlot; }
        } else if (rp < (uint64_t)cF + ctot[w]) {
          qr[nc] = (uint32_t)(rp - cF);
          tq[nc++] = t;
        } else {
          if (s.wminL[w] != s.wmaxL[w]) fail = 1;
          else if (rec) { S->tlo[t] = S->thi[t] = s.wminL[w]; S->tslot[t] = kNoSlot; }
        }
      }
    }
  }
  __syncthreads();
  if (fail) {
    if (rec && threadIdx.x == 0) atomicOr(&S->err, 1u);
    return;
  }
  if (nc == 0) return;
  find_bins(hist + (size_t)w * kBins, kBins, qr, nc, wsum, rbin, rrem);
  if (threadIdx.x == 0) {
    uint32_t k0, k1;
    window_keys(s, w, k0, k1);
    const uint32_t mult = bin_mult(k0, k1);
    for (int j = 0; j < nc; ++j) {
      uint32_t a, z;
      bin_interval(rbin[j], k0, mult, 0u, 0xffffffffu, a, z);
      int own = -1;                      // targets sharing a bin share the first one's slot
      for (int q = 0; q < nslot; ++q)
        if (sl[q] == a && sz[q] == z) own = q;
      if (own < 0) {
        own = nslot++;
        sl[own] = a; sz[own] = z;
        slot[own] = tq[j];
      }
      if (rec) {
        const int t = tq[j];
        S->tlo[t] = a;
        S->thi[t] = z;
        S->rank[t] = rrem[j];            // rank inside the fine bin
        S->tslot[t] = (uint32_t)slot[own];
        S->twin[t] = (uint32_t)w;
      }
    }
  }
  __syncthreads();
  // this workgroup's slice of the band's window keys -> the slots (headers zeroed by k_bandw_hist)
  const int ns = nslot;
  const uint32_t c = min(s.ccount[w], cap);
  const uint32_t i0 = (uint32_t)((uint64_t)c * jw / kBandSplit), i1 = (uint32_t)((uint64_t)c * (jw + 1) / kBandSplit);
  const uint32_t* keys = cand + (size_t)w * cap;
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kBlock) {
    const uint32_t k = keys[i];
    for (int q = 0; q < ns; ++q) {
      if (k >= sl[q] && k <= sz[q]) {
        uint32_t* h = send + (size_t)slot[q] * kPickWords;
        const uint32_t pos = atomicAdd(&h[0], 1u);
        atomicMin(&h[1], k);
        atomicMax(&h[2], k);
        if (pos < (uint32_t)kPick) h[3 + pos] = k;
      }
    }
  }
}

// Every band's keys of each target slot merged (in LDS, or `scratch` past kBins keys), then the
// exact key of each target sharing the slot (rank inside the bin) selected: a workgroup per slot.
__global__ __launch_bounds__(kBlock) void k_bandw_final(SelState* st, const uint32_t* recv, int nranks,
                                                        uint32_t* scratch, uint32_t scratch_cap) {
  __shared__ uint32_t lh[kBins];
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ uint32_t rbin[kMaxTgt], rrem[kMaxTgt], tl[kMaxTgt], tz[kMaxTgt], tr[kMaxTgt], out[kMaxTgt];
  __shared__ uint32_t ranks[kMaxTgt], offs[kMaxBandRanks + 1];
  __shared__ int who[kMaxTgt], ng, bad;
  __shared__ uint32_t tot, gmn, gmx;
  SelState* S = st;
  if (S->phase != PH_INIT || S->err) return;
  const int ntgt = (int)S->ntgt;
  // one workgroup per target slot (slot t0 = the first target of its fine bin)
  const int t0 = blockIdx.x;
  if (t0 >= ntgt || S->tslot[t0] != (uint32_t)t0) return;      // not a slot owner (or resolved)
  const uint32_t per = scratch_cap / kMaxTgt;                  // each slot's keys in their own scratch range
  const uint32_t base = per * (uint32_t)t0;
  {
    if (threadIdx.x == 0) {
      ng = 0;
      for (int t = t0; t < ntgt; ++t)
        if (S->tslot[t] == (uint32_t)t0) { who[ng] = t; ranks[ng++] = S->rank[t]; }
      uint32_t acc = 0, a = 0xffffffffu, z = 0u;
      bad = 0;
      for (int r = 0; r < nranks; ++r) {
        const uint32_t* h = recv + (size_t)r * kBandWords + (size_t)t0 * kPickWords;
        offs[r] = acc;
        if (h[0]) { a = min(a, h[1]); z = max(z, h[2]); }
        if (h[0] > (uint32_t)kPick) bad = 1;
        acc += min(h[0], (uint32_t)kPick);
      }
      offs[nranks] = acc;
      tot = acc;
      gmn = a;
      gmx = z;
      if (bad && a == z) {              // one distinct key: every target of the slot is it
        for (int q = 0; q < ng; ++q) { S->tlo[who[q]] = S->thi[who[q]] = a; }
        ng = 0;
        bad = 0;
      }
      if (!bad && ng > 0 && acc > (uint32_t)kBins && acc > per) bad = 1;
      if (bad) S->err = 1u;
    }
    __syncthreads();
    if (bad) return;
    if (ng == 0) return;
    if (tot <= (uint32_t)kBins) {
      // the usual case (tens of keys per fine bin and band): the bin's keys in LDS, each key's
      // rank range counted against all of them
      for (int r = 0; r < nranks; ++r) {
        const uint32_t o = offs[r], n = offs[r + 1] - o;
        const uint32_t* src = recv + (size_t)r * kBandWords + (size_t)t0 * kPickWords + 3;
        for (uint32_t i = threadIdx.x; i < n; i += kBlock) lh[o + i] = src[i];
      }
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < tot; i += kBlock) {
        const uint32_t k = lh[i];
        uint32_t less = 0, leq = 0;
        for (uint32_t q = 0; q < tot; ++q) {
          const uint32_t v = lh[q];
          less += v < k ? 1u : 0u;
          leq += v <= k ? 1u : 0u;
        }
        for (int q = 0; q < ng; ++q)
          if (less <= ranks[q] && ranks[q] < leq) S->tlo[who[q]] = S->thi[who[q]] = k;   // (equal keys: same value)
      }
      return;
    }
    uint32_t* keys = scratch + base;
    for (int r = 0; r < nranks; ++r) {
      const uint32_t o = offs[r], n = offs[r + 1] - o;
      const uint32_t* src = recv + (size_t)r * kBandWords + (size_t)t0 * kPickWords + 3;
      for (uint32_t i = threadIdx.x; i < n; i += kBlock) keys[o + i] = src[i];
    }
    __syncthreads();
    cand_select(keys, tot, gmn, gmx < gmn ? gmn : gmx, ranks, ng, out, lh, wsum, rbin, rrem, tl, tz, tr);
    if (threadIdx.x < ng) S->tlo[who[threadIdx.x]] = S->thi[who[threadIdx.x]] = out[threadIdx.x];
  }
}

struct Exchange {
  i2pc_exchange_fn fn;
  void* user;
  int64_t* ex;     // device int64 [4][max(B, kBandEx)]
  i2pc_gather_fn gather;   // window-selection band runs: the candidate all-gather (else NULL)
  int nranks;
  uint32_t* send;          // [kBandWords]
  uint32_t* recv;          // [nranks][kBandWords]
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

// Selection sweep geometry: kTileW-column tiles, rows per workgroup from I2PC_SEL_PTS
// points (default 8192) and the LDS the interpolated model rows of R output rows take.
static Sweep plan_select(int H, int W, int dh, int dw, bool same, int row0, int row1) {
  static const int sel_pts = [] { const char* e = getenv("I2PC_SEL_PTS"); return e ? atoi(e) : 8192; }();
  Sweep sw{};
  const int tw = std::min(W, kTileW);
  int R = std::max(1, std::min(32, (sel_pts + tw - 1) / tw));   // <= 32 rows: 16-bit LDS counts
  auto rows_for = [&](int r) { return std::min(dh, (int)std::floor((double)(r - 1) * dh / H) + 3); };
  auto bytes = [&](int r, bool raw) { return (size_t)rows_for(r) * (kTileW + (raw ? dw : 0)) * sizeof(float); };
  sw.raw = 1;
  if (!same) {
    while (R > 1 && bytes(R, true) > (size_t)kHrowBudget) R /= 2;
    if (bytes(R, true) > (size_t)kHrowBudget) sw.raw = 0;   // very wide model rows: interpolate from global
  }
  sw.R = R;
  sw.row0 = row0;
  sw.row_end = row1;
  sw.nrb = std::max(1, (row1 - row0 + R - 1) / R);
  sw.ntiles = (W + kTileW - 1) / kTileW;
  sw.lds_rows = same ? 0 : rows_for(R);
  return sw;
}

template <int LEVEL>
static int select_level(const Geo& g, SelState* st, uint32_t* hist, uint32_t* cand, uint32_t cap, int B,
                        const Sweep& sw, hipStream_t s, const Exchange* x) {
  // level 0 histograms one slot (8 KB of LDS); levels 1-2 up to kSlots target intervals
  const size_t lds = sizeof(uint32_t) * kSlots * kSlotWords +
                     (size_t)sw.lds_rows * (kTileW + (sw.raw ? g.dw : 0)) * sizeof(float);
  const dim3 grid(B * sw.nrb * sw.ntiles), block(kBlock);
  if (g.same)
    hipLaunchKernelGGL((k_sweep<LEVEL, true>), grid, block, lds, s, g, st, hist, cand, cap, B, sw);
  else
    hipLaunchKernelGGL((k_sweep<LEVEL, false>), grid, block, lds, s, g, st, hist, cand, cap, B, sw);
  int rc = exchange<LEVEL>(x, hist, st, B, s);
  if (rc) return rc;
  // tile-parallel runs only histogram: the histograms are what the bands exchange
  hipLaunchKernelGGL((k_resolve<LEVEL>), dim3(B), dim3(kBlock), 0, s, st, hist, cand, cap, B, x ? 0 : 1);
  return I2PC_OK;
}

// "sel_windows" (I2PC_SEL_WIN): 1 = the window-only batch selection (k_sweep_w / k_resolve_w),
// 0 = the histogram levels (the band path's); both exact.
static thread_local int g_sel_windows = [] { const char* e = getenv("I2PC_SEL_WIN"); return e ? atoi(e) : 1; }();
// "sel_scratch" (I2PC_SEL_SCRATCH, tests / measurement only): every image of a window-path selection
// goes to the selection from scratch (as if a window had missed)
static thread_local int g_sel_scratch = [] { const char* e = getenv("I2PC_SEL_SCRATCH"); return e ? atoi(e) : 0; }();
__global__ void k_force_scratch(SelState* st, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B && st[b].phase == PH_INIT) st[b].err = 1u;
}
// output rows per k_sweep_w workgroup ("sel_rows", I2PC_SEL_ROWS)
static thread_local int g_sel_rows = [] {
  const char* e = getenv("I2PC_SEL_ROWS");
  const int v = e ? atoi(e) : 16;
  return v > 0 && v <= kMaxSelRows ? v : 16;
}();

// k_sel_slow's workgroups per image: ~256 K pixels each (a 1024^2 image: 4), <= 2048 workgroups in all
static int slow_parts(int H, int W, int B) {
  const int64_t want = std::max<int64_t>(1, (int64_t)H * W / 262144);
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, std::max(1, 2048 / std::max(B, 1))));
}

// the selection's finish: k_sel_slow (finish / range / from-scratch level 0) and the from-scratch
// radix levels 1 and 2 (no-ops unless an image needs them)
static void launch_slow(const Geo& g, SelState* st, int B, uint32_t* slow, uint32_t* scr, int swept, hipStream_t s) {
  const int P = slow_parts(g.H, g.W, B);
  hipLaunchKernelGGL(k_sel_slow, dim3(B * P), dim3(kSlowBlock), 0, s, g, st, B, P, slow, swept, scr);
  hipLaunchKernelGGL(k_scratch<1>, dim3(B * P), dim3(kSlowBlock), 0, s, g, st, B, P, slow, scr);
  hipLaunchKernelGGL(k_scratch<2>, dim3(B * P), dim3(kSlowBlock), 0, s, g, st, B, P, slow, scr);
}

static int launch_select(const Geo& g, SelState* st, uint32_t* hist, uint32_t* cand, const uint32_t* rpart,
                         uint32_t* mhist, uint32_t* wpart, uint32_t* slow, uint32_t* scr, uint32_t cap, int B,
                         const Sweep& sw, hipStream_t s, const Exchange* x = nullptr, int nrc = 0) {
  if (nrc <= 0) nrc = range_chunks(B);
  // full-resolution sample of ~64 K points per image for the level-0 estimate
  const SamplePlan sp = sample_plan(g.H, g.W, B);
  // windows: the batch path, and band runs that can all-gather their candidate lists
  const bool win = x ? x->gather != nullptr : g_sel_windows != 0;
  hipLaunchKernelGGL(k_model_hist, dim3(B * sp.nch), dim3(kHistBlock), 0, s, g, B, st, mhist, rpart, sp.stride, sp.nch,
                     nrc);
  hipLaunchKernelGGL(k_window, dim3(B), dim3(kBlock), 0, s, st, mhist, cap, B, win ? 1 : 0, sp.ns, sp.nch);
  if (win) {
    // batch path: one window-only sweep + resolve; k_sel_slow finishes (or, for the rare image
    // a window missed, selects from scratch).  Sweep workgroup = kSelRows output rows x a
    // kTileW-column tile (register-streamed model rows, no LDS row window).
    Sweep sww{};
    sww.R = g_sel_rows;
    sww.row0 = sw.row0;
    sww.row_end = sw.row_end;
    sww.nrb = std::max(1, (sw.row_end - sw.row0 + sww.R - 1) / sww.R);
    sww.ntiles = (g.W + kTileW - 1) / kTileW;
    const dim3 grid(B * sww.nrb * sww.ntiles), block(kBlock);
    if (g.same)
      hipLaunchKernelGGL((k_sweep_w<true>), grid, block, 0, s, g, st, cand, cap, B, sww, wpart);
    else
      hipLaunchKernelGGL((k_sweep_w<false>), grid, block, 0, s, g, st, cand, cap, B, sww, wpart);
    if (x) {
      // band run (B = 1): fine histograms + counters all-reduced, each target's bin keys
      // all-gathered, every rank selects the same keys (2 collectives, ~40 KB per rank)
      hipLaunchKernelGGL(k_bandw_hist, dim3(3 * kBandSplit), dim3(kBlock), 0, s, st, cand, cap, hist, x->ex, wpart,
                         x->send);
      if (x->fn(x->user, hist, 3 * kBins, x->ex, kBandEx, s) != 0)
        return set_error(I2PC_ELAUNCH, "exchange callback failed (window histograms)");
      hipLaunchKernelGGL(k_bandw_pickc, dim3(3 * kBandSplit), dim3(kBlock), 0, s, st, cand, cap, hist, x->ex, x->send);
      if (x->gather(x->user, x->send, x->recv, kBandWords, s) != 0)
        return set_error(I2PC_ELAUNCH, "gather callback failed (target bins)");
      hipLaunchKernelGGL(k_bandw_final, dim3(kMaxTgt), dim3(kBlock), 0, s, st, x->recv, x->nranks, cand, kSlots * cap);
      if (g_sel_scratch) hipLaunchKernelGGL(k_force_scratch, dim3((B + 63) / 64), dim3(64), 0, s, st, B);
      launch_slow(g, st, B, slow, scr, sw.row0 == 0 && sw.row_end == g.H ? 1 : 0, s);
      return check_launch("select");
    }
    hipLaunchKernelGGL(k_resolve_w, dim3(B * 3), dim3(kBlock), 0, s, st, cand, cap, B, wpart);
    if (g_sel_scratch) hipLaunchKernelGGL(k_force_scratch, dim3((B + 63) / 64), dim3(64), 0, s, st, B);
    launch_slow(g, st, B, slow, scr, sw.row0 == 0 && sw.row_end == g.H ? 1 : 0, s);
    return check_launch("select");
  }
  int rc;
  if ((rc = select_level<0>(g, st, hist, cand, cap, B, sw, s, x))) return rc;
  if ((rc = select_level<1>(g, st, hist, cand, cap, B, sw, s, x))) return rc;
  if ((rc = select_level<2>(g, st, hist, cand, cap, B, sw, s, x))) return rc;
  if ((rc = select_level<3>(g, st, hist, cand, cap, B, sw, s, x))) return rc;
  launch_slow(g, st, B, slow, scr, 0, s);
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

// Forked selection chains (batch path): per host thread and device, side streams and the
// fork / join events (thread-local, so concurrent callers on other threads never share them).
// "sel_parts" (I2PC_SEL_PARTS): sub-batches of the selection chain; 0 = automatic = 1.
// Measured r03 (B = 32 x 1024^2, whole call): 1 part 254 us, 2 parts 271, 3 parts 289, 4 parts
// 311 -- the halves' launches do not overlap enough to pay for the split sweeps, so it stays off.
constexpr int kMaxParts = 4;
struct AuxStreams {
  bool ok = false;
  int dev = -1;
  hipStream_t s[kMaxParts - 1] = {};
  hipEvent_t fork = nullptr, join[kMaxParts - 1] = {};
  // released when the owning host thread exits (thread_local below; the main thread's run before
  // the static destructors, so the HIP runtime is still up)
  ~AuxStreams() {
    if (dev < 0) return;
    int cur = -1;
    const bool swap = hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess;
    for (int i = 0; i < kMaxParts - 1; ++i) {
      if (s[i]) (void)hipStreamDestroy(s[i]);
      if (join[i]) (void)hipEventDestroy(join[i]);
    }
    if (fork) (void)hipEventDestroy(fork);
    if (swap) (void)hipSetDevice(cur);
  }
};
static thread_local int g_sel_parts = [] { const char* e = getenv("I2PC_SEL_PARTS"); return e ? atoi(e) : 0; }();
// "sel_lband" (I2PC_SEL_LBAND): a single image resolves its windows through the band kernels with a
// local (identity) exchange -- fine histogram and target-bin compaction spread over 3 x kBandSplit
// workgroups -- instead of k_resolve_w's one workgroup per window, whose key lists grow with the
// image (the window half-width follows the sample's rank noise).  -1 = automatic (from
// kLocalBandPixels pixels: measured equal at 1024^2, 120 -> 102 us at 2048^2, 301 -> 248 us at
// 8192 x 4096), 0 = off, 1 = always (B = 1).
static thread_local int g_sel_lband = [] { const char* e = getenv("I2PC_SEL_LBAND"); return e ? atoi(e) : -1; }();
constexpr int64_t kLocalBandPixels = 2 << 20;
static int local_exchange(void*, uint32_t*, int64_t, int64_t*, int, void*) { return 0; }   // one band: sums in place
static int local_gather(void*, const uint32_t*, uint32_t*, int64_t, void*) { return 0; }    // recv aliases send
static int select_parts(int batch) {
  if (!g_sel_windows) return 1;
  const int p = g_sel_parts > 0 ? std::min(g_sel_parts, kMaxParts) : 1;
  return std::max(1, std::min(p, batch));
}
static AuxStreams& aux_streams(int need) {
  static thread_local AuxStreams ax[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) { static thread_local AuxStreams bad; return bad; }
  AuxStreams& a = ax[dev];
  if (!a.ok) {
    a.ok = hipEventCreateWithFlags(&a.fork, hipEventDisableTiming) == hipSuccess;
    for (int i = 0; i < kMaxParts - 1 && a.ok; ++i)
      a.ok = hipStreamCreateWithFlags(&a.s[i], hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&a.join[i], hipEventDisableTiming) == hipSuccess;
    a.dev = dev;
  }
  (void)need;
  return a;
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
  I2PC_REQUIRE(params->projection == 0 || params->projection == 1, "projection must be 0 (pinhole) or 1 (equirectangular)");
  I2PC_REQUIRE((int64_t)img_h * img_w < (1ll << 31), "image too large");
  const int blur_k = params->smooth_ksize < 3 ? 3 : params->smooth_ksize / 2 * 2 + 1;   // app.py:211
  if (params->smooth)
    I2PC_REQUIRE(blur_k <= kMaxBlur, "smooth_ksize -> kernel %d: at most %d taps", blur_k, kMaxBlur);
  const int granks = xch && xch->gather ? xch->nranks : 0;
  const Layout L = layout(batch, img_h, img_w, params->smooth, granks);
  const bool lband = !xch && batch == 1 && g_sel_windows &&
                     (g_sel_lband > 0 || (g_sel_lband < 0 && (int64_t)img_h * img_w >= kLocalBandPixels));
  if (workspace_bytes < L.total) return set_error(I2PC_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, L.total);
  hipStream_t s = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  SelState* st = reinterpret_cast<SelState*>(ws + L.state);
  uint32_t* hist = reinterpret_cast<uint32_t*>(ws + L.hist);
  Tap* xt = reinterpret_cast<Tap*>(ws + L.xtab);
  Tap* yt = reinterpret_cast<Tap*>(ws + L.ytab);

  const int n = img_h * img_w;
  uint32_t* rpart = reinterpret_cast<uint32_t*>(ws + L.rpart);
  double* trig = params->projection == 1 ? reinterpret_cast<double*>(ws + L.trig) : nullptr;
  hipLaunchKernelGGL(k_prepare, dim3(batch * range_chunks(batch)), dim3(kBlock), 0, s, depth, batch, dep_h * dep_w, n,
                     st, (xch || lband || !g_sel_windows) ? hist : nullptr, rpart, xt, yt, dep_h, dep_w, img_h, img_w,
                     cv_scale(dep_w, img_w), cv_scale(dep_h, img_h), trig, reinterpret_cast<uint32_t*>(ws + L.mhist),
                     range_chunks(batch), reinterpret_cast<uint32_t*>(ws + L.wpart), reinterpret_cast<uint32_t*>(ws + L.slow),
                     reinterpret_cast<uint32_t*>(ws + L.scr));

  Geo g{depth, dep_h, dep_w, img_h, img_w, xt, yt, (dep_h == img_h && dep_w == img_w) ? 1 : 0,
        cv_scale(dep_w, img_w), cv_scale(dep_h, img_h)};
  // selection sweeps: I2PC_SEL_PTS points per workgroup (default 8192: 8 rows of a 1024-wide
  // tile; measured r02, B = 32 x 1024^2 whole call: 4096 pts 334 us, 8192 299 us, 16384 = 8192
  // (the LDS budget caps the rows at 8))
  const Sweep ssel = plan_select(img_h, img_w, dep_h, dep_w, g.same != 0, row0, row1);
  Exchange xb = xch ? *xch : Exchange{nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr};
  xb.ex = reinterpret_cast<int64_t*>(ws + L.ex);
  xb.send = reinterpret_cast<uint32_t*>(ws + L.gsend);
  xb.recv = reinterpret_cast<uint32_t*>(ws + L.grecv);
  if (lband) {
    xb.fn = local_exchange;
    xb.gather = local_gather;
    xb.nranks = 1;
    xb.recv = xb.send;
  }
  uint32_t* cand = reinterpret_cast<uint32_t*>(ws + L.cand);
  uint32_t* mhist = reinterpret_cast<uint32_t*>(ws + L.mhist);
  uint32_t* wpart = reinterpret_cast<uint32_t*>(ws + L.wpart);
  uint32_t* slow = reinterpret_cast<uint32_t*>(ws + L.slow);
  uint32_t* scr = reinterpret_cast<uint32_t*>(ws + L.scr);
  const int nrc = range_chunks(batch);
  int rc;
  const int parts = xch ? 1 : select_parts(batch);
  if (parts > 1) {
    // the selection chain is mostly latency-bound small launches: run it as `parts` sub-batches
    // on forked streams so their launches overlap, then join for one unprojection launch
    AuxStreams& ax = aux_streams(parts - 1);
    if (!ax.ok) return set_error(I2PC_ELAUNCH, "cannot create the selection side streams");
    if (hipEventRecord(ax.fork, s) != hipSuccess) return set_error(I2PC_ELAUNCH, "hipEventRecord failed");
    for (int q = 0; q < parts; ++q) {
      const int b0 = batch * q / parts, b1 = batch * (q + 1) / parts;
      hipStream_t sq = q == 0 ? s : ax.s[q - 1];
      if (q > 0 && hipStreamWaitEvent(sq, ax.fork, 0) != hipSuccess) return set_error(I2PC_ELAUNCH, "hipStreamWaitEvent failed");
      Geo gq = g;
      gq.depth = g.depth + (size_t)b0 * dep_h * dep_w;
      rc = launch_select(gq, st + b0, hist + (size_t)b0 * kSlots * kBins, cand + (size_t)b0 * kSlots * L.cap,
                         rpart + (size_t)b0 * nrc * 2, mhist + (size_t)b0 * kBins, wpart + (size_t)b0 * kBelowSlots * 4,
                         slow + (size_t)b0 * 8, scr + (size_t)b0 * kScrWords, L.cap, b1 - b0, ssel, sq, nullptr, nrc);
      if (rc) return rc;
      if (q > 0) {
        if (hipEventRecord(ax.join[q - 1], sq) != hipSuccess || hipStreamWaitEvent(s, ax.join[q - 1], 0) != hipSuccess)
          return set_error(I2PC_ELAUNCH, "stream join failed");
      }
    }
  } else {
    rc = launch_select(g, st, hist, cand, rpart, mhist, wpart, slow, scr, L.cap, batch, ssel, s,
                       (xch || lband) ? &xb : nullptr, nrc);
    if (rc) return rc;
  }

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
  cam.proj = params->projection;
  cam.trig = trig;
  cam.W = img_w;
  cam.Wn = (img_w + step - 1) / step;
  const int Hn = (img_h + step - 1) / step;
  cam.N = cam.Wn * Hn;
  const int unp_rows = std::max(1, std::min(kMaxRows, (4 * 1024 + cam.Wn - 1) / cam.Wn));
  const int prow0 = row0 / step, prow1 = (row1 + step - 1) / step;   // point rows of the band
  const Sweep sunp = plan_sweep(Hn, step, dep_h, dep_w, img_h, g.same != 0, unp_rows, prow0, prow1);
  const size_t unp_lds = sweep_lds(sunp, dep_w);
  const double* field = nullptr;
  const bool fast = !params->smooth && channels == 3 && cam.N % 4 == 0 && cam.Wn % 4 == 0;
  Sweep sr{};
  size_t lr = 0;
  if (params->smooth) {
    double* f0 = reinterpret_cast<double*>(ws + L.field);
    double* f1 = reinterpret_cast<double*>(ws + L.tmp);
    const int nb = 2048;
    // image rows the vertical pass reads for the band's output rows (reflect-101 included):
    // the band plus a k/2 halo, or reflected rows near the image's top and bottom
    const int hr = blur_k / 2;
    int f_lo = row0, f_hi = row1;
    for (int v = row0; v < row1; ++v) {
      if (v >= row0 + hr && v < row1 - hr) { v = row1 - hr - 1; continue; }   // interior rows add nothing
      for (int t = -hr; t <= hr; ++t) {
        const int rr = reflect101_host(v + t, img_h);
        f_lo = std::min(f_lo, rr);
        f_hi = std::max(f_hi, rr + 1);
      }
    }
    hipLaunchKernelGGL(k_norm_field, dim3(nb), dim3(256), 0, s, g, st, batch, params->invert, f0, f_lo, f_hi);
    const BlurTaps taps = gaussian_taps(blur_k);
    hipLaunchKernelGGL((k_blur<true>), dim3(nb), dim3(256), 0, s, f0, f1, st, batch, img_h, img_w, taps, f_lo, f_hi);
    hipLaunchKernelGGL((k_blur<false>), dim3(nb), dim3(256), 0, s, f1, f0, st, batch, img_h, img_w, taps, row0, row1);
    field = f0;
    hipLaunchKernelGGL((k_unproject<true>), dim3(batch * sunp.nrb), dim3(kBlock), 0, s, g, st, field, image,
                       channels, batch, sunp, params->invert, cam, xyz, rgb, st);
  } else if (fast && !g.same && rows_plan(Hn, step, dep_h, dep_w, img_h, cam.Wn, prow0, prow1, sr, lr)) {
    prof_mark(0, s);
    const dim3 grid(batch * sr.nrb * sr.ntiles), block(kBlock);
    if (step == 1)
      hipLaunchKernelGGL((k_unproject_rows<1>), grid, block, lr, s, g, st, image, batch, sr, params->invert, cam, xyz, rgb, st);
    else if (step == 2)
      hipLaunchKernelGGL((k_unproject_rows<2>), grid, block, lr, s, g, st, image, batch, sr, params->invert, cam, xyz, rgb, st);
    else
      hipLaunchKernelGGL((k_unproject_rows<4>), grid, block, lr, s, g, st, image, batch, sr, params->invert, cam, xyz, rgb, st);
    prof_mark(1, s);
  } else if (fast) {
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

static int run_band(const float* depth, int dep_h, int dep_w, const uint8_t* image_band, int channels,
                    int img_h, int img_w, int row0, int row1, const i2pc_unproject_params* params,
                    float* xyz_band, uint8_t* rgb_band, double* bbox, double* stats,
                    void* workspace, size_t workspace_bytes, i2pc_exchange_fn exchange_fn,
                    i2pc_gather_fn gather_fn, int nranks, void* user, void* stream);

extern "C" size_t i2pc_unproject_band_workspace_bytes(int img_h, int img_w, int smooth, int nranks) {
  if (img_h <= 0 || img_w <= 0 || nranks <= 0 || nranks > kMaxBandRanks) return 0;
  return layout(1, img_h, img_w, smooth, nranks).total;
}

extern "C" int i2pc_unproject_band(const float* depth, int dep_h, int dep_w, const uint8_t* image_band, int channels,
                                   int img_h, int img_w, int row0, int row1, const i2pc_unproject_params* params,
                                   float* xyz_band, uint8_t* rgb_band, double* bbox, double* stats,
                                   void* workspace, size_t workspace_bytes, i2pc_exchange_fn exchange_fn,
                                   void* user, void* stream) {
  clear_error();
  return run_band(depth, dep_h, dep_w, image_band, channels, img_h, img_w, row0, row1, params, xyz_band, rgb_band,
                  bbox, stats, workspace, workspace_bytes, exchange_fn, nullptr, 0, user, stream);
}

extern "C" int i2pc_unproject_band_w(const float* depth, int dep_h, int dep_w, const uint8_t* image_band,
                                     int channels, int img_h, int img_w, int row0, int row1,
                                     const i2pc_unproject_params* params, float* xyz_band, uint8_t* rgb_band,
                                     double* bbox, double* stats, void* workspace, size_t workspace_bytes,
                                     int nranks, i2pc_exchange_fn exchange_fn, i2pc_gather_fn gather_fn, void* user,
                                     void* stream) {
  clear_error();
  I2PC_REQUIRE(exchange_fn && gather_fn, "the window band mode needs both the exchange and the gather");
  I2PC_REQUIRE(nranks > 0 && nranks <= kMaxBandRanks, "nranks %d outside [1, %d]", nranks, kMaxBandRanks);
  return run_band(depth, dep_h, dep_w, image_band, channels, img_h, img_w, row0, row1, params, xyz_band, rgb_band,
                  bbox, stats, workspace, workspace_bytes, exchange_fn, gather_fn, nranks, user, stream);
}

static int run_band(const float* depth, int dep_h, int dep_w, const uint8_t* image_band, int channels,
                    int img_h, int img_w, int row0, int row1, const i2pc_unproject_params* params,
                    float* xyz_band, uint8_t* rgb_band, double* bbox, double* stats,
                    void* workspace, size_t workspace_bytes, i2pc_exchange_fn exchange_fn,
                    i2pc_gather_fn gather_fn, int nranks, void* user, void* stream) {
  I2PC_REQUIRE(params != nullptr, "params is NULL");
  I2PC_REQUIRE(image_band && xyz_band && rgb_band, "NULL device pointer");
  I2PC_REQUIRE(img_h > 0 && img_w > 0 && channels >= 1 && channels <= 4, "bad image shape");
  const int step = params->step;
  I2PC_REQUIRE(step == 1 || step == 2 || step == 4, "step must be 1, 2 or 4 (low/medium/high)");
  I2PC_REQUIRE(0 <= row0 && row0 < row1 && row1 <= img_h, "band rows [%d, %d) outside [0, %d)", row0, row1, img_h);
  I2PC_REQUIRE(row0 % step == 0 && (row1 % step == 0 || row1 == img_h),
               "band rows must start (and end, unless at the bottom) on a multiple of the step %d", step);
  // smooth_depth: the band's field plus the blur's halo rows are recomputed locally (the
  // model-resolution depth and, after the exchange, the stats are whole on every rank)
  // the kernels address the full image: shift the band buffers back to row 0
  const int Wn = (img_w + step - 1) / step;
  const uint8_t* image = image_band - (ptrdiff_t)row0 * img_w * channels;
  float* xyz = xyz_band - (ptrdiff_t)(row0 / step) * Wn * 3;
  uint8_t* rgb = rgb_band - (ptrdiff_t)(row0 / step) * Wn * 3;
  const Exchange x{exchange_fn, user, nullptr, gather_fn, nranks, nullptr, nullptr};
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
  const int n = h * w;
  uint32_t* rpart = reinterpret_cast<uint32_t*>(ws + L.rpart);
  hipLaunchKernelGGL(k_prepare, dim3(batch * range_chunks(batch)), dim3(kBlock), 0, s, depth, batch, n, n, st,
                     g_sel_windows ? nullptr : hist, rpart, xt, yt, h, w, h, w, 1.0, 1.0, nullptr,
                     reinterpret_cast<uint32_t*>(ws + L.mhist), range_chunks(batch), reinterpret_cast<uint32_t*>(ws + L.wpart),
                     reinterpret_cast<uint32_t*>(ws + L.slow), reinterpret_cast<uint32_t*>(ws + L.scr));
  Geo g{depth, h, w, h, w, xt, yt, 1, 1.0, 1.0};
  const Sweep ssel = plan_select(h, w, h, w, true, 0, h);
  int rc = launch_select(g, st, hist, reinterpret_cast<uint32_t*>(ws + L.cand), rpart,
                         reinterpret_cast<uint32_t*>(ws + L.mhist), reinterpret_cast<uint32_t*>(ws + L.wpart),
                         reinterpret_cast<uint32_t*>(ws + L.slow), reinterpret_cast<uint32_t*>(ws + L.scr), L.cap, batch,
                         ssel, s);
  if (rc) return rc;
  const int64_t total = (int64_t)batch * n;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_preview, dim3(blocks), dim3(256), 0, s, depth, st, batch, n, invert ? 1 : 0, lut_bgr, out_bgr);
  if (stats) hipLaunchKernelGGL(k_finalize, dim3((batch + 63) / 64), dim3(64), 0, s, st, batch, nullptr, stats);
  return check_launch("depth_preview");
}

bool i2pc_unproject_tune(const char* name, int value) {
  if (std::strcmp(name, "unp_rows") == 0) { i2pc::unproj::g_unp_rows = value; return true; }
  if (std::strcmp(name, "unp_nt") == 0) { i2pc::unproj::g_unp_nt = value; return true; }
  if (std::strcmp(name, "unp_rpt") == 0) { i2pc::unproj::g_unp_rpt = value; return true; }
  if (std::strcmp(name, "sel_windows") == 0) { i2pc::unproj::g_sel_windows = value; return true; }
  if (std::strcmp(name, "sel_scratch") == 0) { i2pc::unproj::g_sel_scratch = value; return true; }
  if (std::strcmp(name, "sel_parts") == 0) { g_sel_parts = value; return true; }
  if (std::strcmp(name, "sel_lband") == 0) { g_sel_lband = value; return true; }
  if (std::strcmp(name, "sel_rows") == 0) {
    i2pc::unproj::g_sel_rows = value > 0 && value <= i2pc::unproj::kMaxSelRows ? value : 16;
    return true;
  }
  return false;
}

// Network input pipeline on the GPU (gfx950): BGR uint8 -> RGB -> Pillow-exact
// separable bicubic resample (8-bit fixed point, uint8 intermediate) -> rescale
// 1/255 (float64 -> float32) -> (x - mean) / std (float32), written either as
// float32 NCHW pixel_values or directly as bf16 patch rows for the patch-embed GEMM.
//
// Replaces backend/app.py:103 (cvtColor) + :109 (DPTImageProcessorPil:
// transformers image_processing_pil_dpt.py:192-267, image_transforms.py:89-122,
// 313-440) and the patchify of DPTViTPatchEmbeddings (modeling_dpt.py:60-69).
// Coefficients follow Pillow's libImaging/Resample.c (precompute_coeffs /
// normalize_coeffs_8bpc, PRECISION_BITS = 22) and are computed once per size on
// the host (i2pc_preprocess_plan_create), so the device path is pure integer
// arithmetic and bit-exact.
//
// One workgroup = one image x a band of R output rows x a tile of output columns:
// the horizontal pass resamples exactly the input rows (and the input column
// window) that tile needs into LDS (uint8), the vertical pass reads them back;
// nothing but the input and the output touch HBM.  Any width works: wide
// keep-aspect outputs and inputs wider than one LDS stage split into column tiles.
#include "common.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#pragma clang fp contract(off)

namespace i2pc {
namespace pre {

constexpr int PB = 32 - 8 - 2;     // PRECISION_BITS
// LDS per workgroup: the uint8 band of horizontally resampled rows plus the staged input
// rows; 56 + 24 KB keeps two 256-thread workgroups per CU (160 KB).
constexpr int kLdsBudget = 56 * 1024;
constexpr int kStageBytes = 24 * 1024;

struct Axis {
  int out, ksize;
  std::vector<int> xmin, cnt;
  std::vector<int> k;   // [out][ksize] fixed point
};

static double bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc (box = [0, in_size)).
static Axis coeffs(int in_size, int out_size) {
  Axis ax;
  ax.out = out_size;
  const float in0 = 0.f, in1 = (float)in_size;
  double scale = (double)(in1 - in0) / out_size;
  double filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 2.0 * filterscale;
  ax.ksize = (int)std::ceil(support) * 2 + 1;
  ax.xmin.resize(out_size);
  ax.cnt.resize(out_size);
  ax.k.assign((size_t)out_size * ax.ksize, 0);
  std::vector<double> kk(ax.ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    for (int x = 0; x < xmax; ++x) {
      const double w = bicubic((x + xmin - center + 0.5) * ss);
      kk[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) kk[x] /= ww;
    for (int x = 0; x < xmax; ++x) {
      const double v = kk[x] * (1 << PB);
      ax.k[(size_t)xx * ax.ksize + x] = kk[x] < 0 ? (int)(-0.5 + v) : (int)(0.5 + v);
    }
    ax.xmin[xx] = xmin;
    ax.cnt[xx] = xmax;
  }
  return ax;
}

static Axis identity(int n) {
  Axis ax;
  ax.out = n;
  ax.ksize = 1;
  ax.xmin.resize(n);
  ax.cnt.assign(n, 1);
  ax.k.assign(n, 1 << PB);
  for (int i = 0; i < n; ++i) ax.xmin[i] = i;
  return ax;
}

// A workgroup owns one image x a band of R output rows x a tile of CW output columns.
// Wide outputs (keep-aspect panoramas) and wide inputs split into column tiles, each
// staging only the input column window [col_a0, col_a0 + col_wb) bytes its taps read.
struct DevPlan {
  int in_h, in_w, out_h, out_w, kx, ky, R, tiles, CW, ctiles, patch, pld, lds_bytes;
  int crows, stage_off;   // input rows staged per chunk, LDS offset of the staging area
  float mean[3], stdv[3];
  const int* hx_min; const int* hx_cnt; const int* hx_k;
  const int* vy_min; const int* vy_cnt; const int* vy_k;
  const int* tile_lo; const int* tile_n;
  const int* col_a0; const int* col_wb;
  const uint32_t* lut;    // [3][256]: channel c's output for uint8 u -- fp32 bits (layout 0), then bf16 (layout 1)
};

}  // namespace pre
}  // namespace i2pc

struct i2pc_preprocess_plan {
  i2pc::pre::DevPlan p;
  void* dev;
};

namespace i2pc {
namespace pre {

// Coefficients are < 2^23 in magnitude (22-bit fixed point of weights below 2): sign-extended from 24
// bits the compiler knows it, and the taps become v_mad_i32_i24 (full rate) -- without it every tap
// was a v_mad_u64_u32 (a quarter-rate 64-bit multiply), which bound the kernel
__device__ __forceinline__ int k24(int k) { return (k << 8) >> 8; }

__device__ __forceinline__ uint8_t clip8(int ss) {
  if (ss >= (1 << PB << 8)) return 255;
  if (ss <= 0) return 0;
  return (uint8_t)(ss >> PB);
}

__global__ __launch_bounds__(256) void k_preprocess(DevPlan P, const uint8_t* __restrict__ bgr, int layout, void* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tmp[];   // [rows][CW][3] uint8 (BGR order)
  // the rescale + normalise of a uint8 value depends on (channel, value) only: a 3 x 256 table (fp32 bits,
  // or bf16 for the patch rows) built on the host with the same arithmetic replaces, per output value,
  // an f64 multiply and a correctly rounded fp32 division (which made the vertical pass VALU-heavy)
  __shared__ uint32_t lut[3 * 256];
  for (int i = threadIdx.x; i < 3 * 256; i += blockDim.x) lut[i] = P.lut[(layout == 0 ? 0 : 3 * 256) + i];
  const int per_img = P.tiles * P.ctiles;
  const int b = blockIdx.x / per_img;
  const int rem = blockIdx.x - b * per_img;
  const int tile = rem / P.ctiles;
  const int ct = rem - tile * P.ctiles;
  const int ylo = P.tile_lo[tile];
  const int nrows = P.tile_n[tile];
  const uint8_t* img = bgr + (int64_t)b * P.in_h * P.in_w * 3;
  const int x0 = ct * P.CW;
  const int CWt = min(P.CW, P.out_w - x0);          // output columns of this tile
  const int row_bytes = P.in_w * 3;
  const int a0 = P.col_a0[ct], wb = P.col_wb[ct];   // staged input window (bytes) of each row
  uint8_t* stg = tmp + P.stage_off;
  const bool vec = ((row_bytes | a0 | wb) & 15) == 0;
  // horizontal pass: input rows [ylo, ylo + nrows), window [a0, a0 + wb) -> LDS, P.crows
  // input rows at a time staged with coalesced 16-B loads (the taps then read LDS, not 3
  // scattered global bytes per tap)
  for (int c0 = 0; c0 < nrows; c0 += P.crows) {
    const int cr = min(P.crows, nrows - c0);
    const uint8_t* src = img + (int64_t)(ylo + c0) * row_bytes + a0;
    __syncthreads();                       // the previous chunk's taps are read
    if (vec) {
      // up to 8 loads per thread in flight before their LDS stores (a load -> store loop
      // serialised one memory latency per iteration)
      const int u = wb >> 4;
      const int n = cr * u;
      constexpr int U = 8;
      for (int i0 = threadIdx.x; i0 < n; i0 += U * blockDim.x) {
        uint4 q[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {   // unconditional (index clamped): no per-load branch + wait
          const int i = min(i0 + k * (int)blockDim.x, n - 1);
          const int r = i / u, c = i - r * u;
          q[k] = reinterpret_cast<const uint4*>(src + (int64_t)r * row_bytes)[c];
        }
#pragma unroll
        for (int k = 0; k < U; ++k)     // clamped too (past n: the last element's own value again)
          reinterpret_cast<uint4*>(stg)[min(i0 + k * (int)blockDim.x, n - 1)] = q[k];
      }
    } else {
      for (int i = threadIdx.x; i < cr * wb; i += blockDim.x) {
        const int r = i / wb, c = i - r * wb;
        stg[i] = src[(int64_t)r * row_bytes + c];
      }
    }
    __syncthreads();
    const int hwork = cr * CWt;
    for (int i = threadIdx.x; i < hwork; i += blockDim.x) {
      const int rl = i / CWt;
      const int xl = i - rl * CWt;
      const int xx = x0 + xl;
      const uint8_t* row = stg + rl * wb - a0;
      const int xmin = P.hx_min[xx], cnt = P.hx_cnt[xx];
      const int* k = P.hx_k + xx * P.kx;
      int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
      for (int x = 0; x < cnt; ++x) {
        const uint8_t* px = row + (xmin + x) * 3;
        const int kv = k24(k[x]);
        s0 += px[0] * kv;
        s1 += px[1] * kv;
        s2 += px[2] * kv;
      }
      uint8_t* t = tmp + ((c0 + rl) * CWt + xl) * 3;
      t[0] = clip8(s0);
      t[1] = clip8(s1);
      t[2] = clip8(s2);
    }
  }
  __syncthreads();
  // vertical pass + rescale/normalise + layout
  const int OW = P.out_w;
  const int y0 = tile * P.R;
  const int rows_out = min(P.R, P.out_h - y0);
  const int vwork = rows_out * CWt;
  const int np_x = OW / max(P.patch, 1);
  const int npatch = (P.out_h / max(P.patch, 1)) * np_x;
  for (int i = threadIdx.x; i < vwork; i += blockDim.x) {
    const int ry = i / CWt;
    const int xl = i - ry * CWt;
    const int xx = x0 + xl;
    const int yy = y0 + ry;
    const int ymin = P.vy_min[yy] - ylo, cnt = P.vy_cnt[yy];
    const int* k = P.vy_k + yy * P.ky;
    int s[3] = {1 << (PB - 1), 1 << (PB - 1), 1 << (PB - 1)};
    for (int y = 0; y < cnt; ++y) {
      const uint8_t* t = tmp + ((ymin + y) * CWt + xl) * 3;
      const int kv = k24(k[y]);
      s[0] += t[0] * kv;
      s[1] += t[1] * kv;
      s[2] += t[2] * kv;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {       // c = RGB channel; BGR source index 2 - c
      const uint32_t v = lut[c * 256 + clip8(s[2 - c])];
      if (layout == 0) {
        static_cast<uint32_t*>(out)[(((int64_t)b * 3 + c) * P.out_h + yy) * OW + xx] = v;
      } else {
        const int p = P.patch;
        const int prow = b * npatch + (yy / p) * np_x + xx / p;
        const int col = c * p * p + (yy % p) * p + (xx % p);
        static_cast<uint16_t*>(out)[(int64_t)prow * P.pld + col] = (uint16_t)v;
      }
    }
  }
}

}  // namespace pre
}  // namespace i2pc

using namespace i2pc;
using namespace i2pc::pre;

extern "C" int i2pc_preprocess_plan_create(int in_h, int in_w, int out_h, int out_w, const float* mean,
                                           const float* stdv, int patch, i2pc_preprocess_plan** plan) {
  clear_error();
  I2PC_REQUIRE(plan && mean && stdv, "NULL argument");
  I2PC_REQUIRE(in_h > 0 && in_w > 0 && out_h > 0 && out_w > 0, "empty size");
  I2PC_REQUIRE(patch >= 0, "patch must be >= 0");
  if (patch > 0) I2PC_REQUIRE(out_h % patch == 0 && out_w % patch == 0, "output %dx%d not a multiple of patch %d", out_h, out_w, patch);
  Axis hx = out_w != in_w ? coeffs(in_w, out_w) : identity(in_w);
  Axis vy = out_h != in_h ? coeffs(in_h, out_h) : identity(in_h);
  const double scale = (double)in_h / out_h;
  const int row_bytes = in_w * 3;
  const bool vec = (row_bytes & 15) == 0;
  // column tiles: the widest that lets the vertical taps of >= 1 output row fit the band
  // budget and lets one input row's window fit the stage
  auto window = [&](int x0, int x1, int& a0, int& wb) {
    int lo = in_w, hi = 0;
    for (int x = x0; x < x1; ++x) { lo = std::min(lo, hx.xmin[x]); hi = std::max(hi, hx.xmin[x] + hx.cnt[x]); }
    a0 = lo * 3;
    int a1 = hi * 3;
    if (vec) { a0 &= ~15; a1 = std::min(row_bytes, (a1 + 15) & ~15); }
    wb = a1 - a0;
  };
  int CW = out_w;
  std::vector<int> ca0, cwb;
  for (;;) {
    bool ok = (vy.ksize + 2) * CW * 3 <= kLdsBudget;
    if (ok) {
      const int ct = (out_w + CW - 1) / CW;
      ca0.assign(ct, 0);
      cwb.assign(ct, 0);
      for (int c = 0; c < ct && ok; ++c) {
        window(c * CW, std::min(out_w, (c + 1) * CW), ca0[c], cwb[c]);
        ok = cwb[c] <= kStageBytes;
      }
      if (ok) break;
    }
    I2PC_REQUIRE(CW > 1, "no column tile fits the LDS budget (in %dx%d -> out %dx%d)", in_h, in_w, out_h, out_w);
    CW = (CW + 1) / 2;
  }
  const int ctiles = (out_w + CW - 1) / CW;
  int max_wb = 0;
  for (int c = 0; c < ctiles; ++c) max_wb = std::max(max_wb, cwb[c]);
  // output rows per workgroup so that the uint8 intermediate fits the band budget
  const int band_row = CW * 3;
  int R = 1;
  for (int r = 64; r >= 1; r /= 2) {
    // rows needed by r output rows <= (r - 1) * scale + ksize + 2
    const double need = (r - 1) * scale + vy.ksize + 2;
    if (need * band_row <= kLdsBudget) { R = r; break; }
  }
  const int tiles = (out_h + R - 1) / R;
  std::vector<int> tlo(tiles), tn(tiles);
  int max_rows = 0;
  for (int t = 0; t < tiles; ++t) {
    const int y0 = t * R, y1 = std::min(out_h, y0 + R);
    int lo = 1 << 30, hi = 0;
    for (int y = y0; y < y1; ++y) { lo = std::min(lo, vy.xmin[y]); hi = std::max(hi, vy.xmin[y] + vy.cnt[y]); }
    tlo[t] = lo;
    tn[t] = hi - lo;
    max_rows = std::max(max_rows, hi - lo);
  }
  I2PC_REQUIRE(max_rows * band_row <= kLdsBudget, "LDS band too large (%d rows x %d B)", max_rows, band_row);
  {
    const size_t lds = align_up((size_t)max_rows * band_row, 16) +
                       align_up((size_t)std::max(1, kStageBytes / max_wb) * max_wb, 16);
    I2PC_REQUIRE(lds + 3 * 256 * 4 <= 160 * 1024, "preprocess plan needs %zu B of LDS", lds);
  }
  // every check is done: allocate.  One device buffer:
  // hx_min | hx_cnt | hx_k | vy_min | vy_cnt | vy_k | tile_lo | tile_n | col_a0 | col_wb
  // output table: (float)((double)u / 255 in float64) then (f - mean) / std in float32 (the device formula
  // of r04, image_transforms.py rescale + normalize), as fp32 bits and as RNE bf16
  std::vector<int> lut(2 * 3 * 256);
  for (int c = 0; c < 3; ++c)
    for (int u = 0; u < 256; ++u) {
      const float f = (float)((double)u * (1.0 / 255.0));
      const float v = (f - mean[c]) / stdv[c];
      uint32_t bits;
      std::memcpy(&bits, &v, 4);
      lut[c * 256 + u] = (int)bits;
      const uint32_t rne = bits + 0x7FFFu + ((bits >> 16) & 1u);   // finite values only
      lut[3 * 256 + c * 256 + u] = (int)(rne >> 16);
    }
  std::vector<int> blob;
  auto put = [&](const std::vector<int>& v) { size_t off = blob.size(); blob.insert(blob.end(), v.begin(), v.end()); return off; };
  const size_t o0 = put(hx.xmin), o1 = put(hx.cnt), o2 = put(hx.k), o3 = put(vy.xmin), o4 = put(vy.cnt), o5 = put(vy.k),
               o6 = put(tlo), o7 = put(tn), o8 = put(ca0), o9 = put(cwb), o10 = put(lut);
  void* dev = nullptr;
  if (hipMalloc(&dev, blob.size() * sizeof(int)) != hipSuccess) return set_error(I2PC_ELAUNCH, "hipMalloc failed");
  if (hipMemcpy(dev, blob.data(), blob.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(dev);
    return set_error(I2PC_ELAUNCH, "hipMemcpy failed");
  }
  auto* pl = new i2pc_preprocess_plan();
  pl->dev = dev;
  DevPlan& P = pl->p;
  P.in_h = in_h; P.in_w = in_w; P.out_h = out_h; P.out_w = out_w;
  P.kx = hx.ksize; P.ky = vy.ksize; P.R = R; P.tiles = tiles; P.CW = CW; P.ctiles = ctiles; P.patch = patch;
  P.pld = (3 * patch * patch + 63) / 64 * 64;   // patch-row pitch: the GEMM K axis, padded to 64
  P.stage_off = (int)align_up((size_t)max_rows * band_row, 16);
  P.crows = std::max(1, kStageBytes / max_wb);
  P.lds_bytes = P.stage_off + (int)align_up((size_t)P.crows * max_wb, 16);
  for (int c = 0; c < 3; ++c) { P.mean[c] = mean[c]; P.stdv[c] = stdv[c]; }
  const int* base = static_cast<const int*>(dev);
  P.hx_min = base + o0; P.hx_cnt = base + o1; P.hx_k = base + o2;
  P.vy_min = base + o3; P.vy_cnt = base + o4; P.vy_k = base + o5;
  P.tile_lo = base + o6; P.tile_n = base + o7;
  P.col_a0 = base + o8; P.col_wb = base + o9;
  P.lut = reinterpret_cast<const uint32_t*>(base + o10);
  *plan = pl;
  return I2PC_OK;
}

extern "C" void i2pc_preprocess_plan_destroy(i2pc_preprocess_plan* plan) {
  if (!plan) return;
  (void)hipFree(plan->dev);
  delete plan;
}

extern "C" int i2pc_preprocess(const i2pc_preprocess_plan* plan, const uint8_t* bgr, int batch, int layout,
                               void* out, void* stream) {
  clear_error();
  I2PC_REQUIRE(plan && bgr && out && batch > 0, "bad arguments");
  I2PC_REQUIRE(layout == 0 || (layout == 1 && plan->p.patch > 0), "layout must be 0 (fp32 NCHW) or 1 (bf16 patch rows, plan with patch > 0)");
  const DevPlan& P = plan->p;
  if (P.lds_bytes > 64 * 1024) {
    static bool attr = false;
    if (!attr) {
      // (the kernel's static LDS -- the 3 x 256 output table -- counts against the 160 KB too)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_preprocess), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024 - 3 * 256 * 4);
      attr = true;
    }
  }
  hipLaunchKernelGGL(k_preprocess, dim3(batch * P.tiles * P.ctiles), dim3(256), P.lds_bytes, as_stream(stream), P, bgr, layout, out);
  return check_launch("preprocess");
}

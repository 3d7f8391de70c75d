// Statistical outlier removal (refine_point_cloud, backend/app.py:252-269) on MI355X.
//
// The reference hands the float64 copy of the cloud to Open3D (open3d>=0.17.0,
// backend/requirements.txt:14) PointCloud::RemoveStatisticalOutliers(20, 2.0):
//   avg[i] = mean of sqrt(d2) over the k = min(nb_neighbors, n) nearest points of the
//            cloud (point i itself included, d2 = 0); d2 = (dx*dx + dy*dy) + dz*dz in
//            float64 (nanoflann's L2 metric), summed in ascending order;
//   mean   = sum(avg[i] > 0) / n;   std = sqrt(sum_{avg>0} (avg - mean)^2 / (n - 1));
//   keep i iff 0 < avg[i] < mean + std_ratio * std (ascending indices).
// The kNN is exact on a uniform grid that is built and sized on the device (no host
// synchronisation, so the call is graph-capturable):
//   k_bbox -> k_grid (one thread: the smallest cell size giving at most `cap` cells)
//   -> k_cell (cell of each point + counts) -> exclusive scan -> k_scatter (points
//   counting-sorted by cell as float4 {x, y, z, index}) -> k_knn (one thread per sorted
//   point; Chebyshev shells of cells around its own, whose x-runs are contiguous in the
//   sorted array; stops once k candidates are held and the k-th distance lies inside the
//   scanned cube) -> deterministic two-pass mean / std -> flags -> scan -> compaction.
// Candidate loads are L2 hits (a wave's queries share cells); the kernel is latency-
// and FP64-issue-bound, not HBM-bound.
#include "common.h"

#include <algorithm>
#include <cmath>

namespace i2pc {
namespace sor {

constexpr int kBlock = 256;
constexpr int kScanTile = 4 * kBlock;   // elements per scan block
constexpr int kRedBlocks = 512;         // fixed partition -> deterministic sums

struct Grid {
  double ox, oy, oz, h, margin;
  float fox, foy, foz, inv_h;
  int nx, ny, nz, bad;
};

struct State {
  uint32_t key[6];    // input bbox, ordered float keys: min x, max x, min y, max y, min z, max z
  uint32_t kkey[6];   // bbox of the kept points
  double mean, thr;
};

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o));
  return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
  return x;
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o);
    if (lane >= o) x += y;
  }
  return x;
}

// Wave then block min/max of the ordered keys; one atomic per block and component (a
// per-wave atomic on the same six addresses serialised into ~1 ms per pass).
__device__ __forceinline__ void block_bbox_atomics(const uint32_t* mn, const uint32_t* mx, uint32_t* keys) {
  __shared__ uint32_t red[6][kBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const uint32_t a = wave_min(mn[c]), b = wave_max(mx[c]);
    if (lane == 0) {
      red[2 * c][wid] = a;
      red[2 * c + 1][wid] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int c = threadIdx.x;
    uint32_t x = red[c][0];
    for (int w = 1; w < kBlock / 64; ++w) x = (c & 1) ? max(x, red[c][w]) : min(x, red[c][w]);
    if (c & 1) {
      if (x) atomicMax(&keys[c], x);
    } else if (x != 0xffffffffu) {
      atomicMin(&keys[c], x);
    }
  }
}

__global__ void k_init(State* st, int64_t* count) {
  const int t = threadIdx.x;
  if (t < 6) {
    st->key[t] = (t & 1) ? 0u : 0xffffffffu;
    st->kkey[t] = (t & 1) ? 0u : 0xffffffffu;
  }
  if (t == 0 && count) *count = 0;
}

__global__ __launch_bounds__(kBlock) void k_bbox(const float* __restrict__ xyz, int64_t n, State* st) {
  uint32_t mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const uint32_t k = f2key(xyz[i * 3 + c]);
      mn[c] = min(mn[c], k);
      mx[c] = max(mx[c], k);
    }
  }
  block_bbox_atomics(mn, mx, st->key);
}

// One thread: the smallest h (bisection) whose grid prod(floor(e/h)+1) has <= cap cells.
__global__ void k_grid(const State* st, Grid* g, uint32_t cap) {
  if (threadIdx.x != 0) return;
  float lo[3];
  double e[3], emax = 0.0;
  bool ok = true;
  for (int c = 0; c < 3; ++c) {
    lo[c] = key2f(st->key[2 * c]);
    const float hi = key2f(st->key[2 * c + 1]);
    ok = ok && isfinite(lo[c]) && isfinite(hi);
    e[c] = (double)hi - (double)lo[c];
    emax = fmax(emax, e[c]);
  }
  double h = 1.0;
  if (ok && emax > 0.0) {
    double a = emax / (double)cap, b = emax * 1.0000001;     // cells(a) > cap >= 8 >= cells(b)
    for (int it = 0; it < 64; ++it) {
      const double m = 0.5 * (a + b);
      double cells = 1.0;
      for (int c = 0; c < 3; ++c) cells *= floor(e[c] / m) + 1.0;
      if (cells <= (double)cap) b = m;
      else a = m;
    }
    h = b;
  }
  int d[3];
  for (int c = 0; c < 3; ++c) d[c] = ok ? (int)fmin(floor(e[c] / h) + 1.0, 16777216.0) : 1;
  g->fox = ok ? lo[0] : 0.f;
  g->foy = ok ? lo[1] : 0.f;
  g->foz = ok ? lo[2] : 0.f;
  g->ox = g->fox;
  g->oy = g->foy;
  g->oz = g->foz;
  g->h = h;
  g->inv_h = (float)(1.0 / h);
  g->nx = d[0];
  g->ny = d[1];
  g->nz = d[2];
  g->bad = ok ? 0 : 1;
  // the float cell assignment (p - o) * inv_h is off the exact face by < ~3 ulp of the
  // extent: the stopping bound gives that much away
  g->margin = 1e-6 * (emax + h);
}

__device__ __forceinline__ void cell_of(const Grid& g, float x, float y, float z, int& cx, int& cy, int& cz) {
  cx = min(max((int)((x - g.fox) * g.inv_h), 0), g.nx - 1);
  cy = min(max((int)((y - g.foy) * g.inv_h), 0), g.ny - 1);
  cz = min(max((int)((z - g.foz) * g.inv_h), 0), g.nz - 1);
}

__global__ __launch_bounds__(kBlock) void k_cell(const float* __restrict__ xyz, int64_t n, const Grid* gp,
                                                 uint32_t* __restrict__ cell, uint32_t* counts) {
  const Grid g = *gp;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    int cx, cy, cz;
    cell_of(g, xyz[i * 3], xyz[i * 3 + 1], xyz[i * 3 + 2], cx, cy, cz);
    const uint32_t c = ((uint32_t)cz * (uint32_t)g.ny + (uint32_t)cy) * (uint32_t)g.nx + (uint32_t)cx;
    cell[i] = c;
    atomicAdd(&counts[c], 1u);
  }
}

__global__ __launch_bounds__(kBlock) void k_scatter(const float* __restrict__ xyz, int64_t n,
                                                    const uint32_t* __restrict__ cell,
                                                    const uint32_t* __restrict__ start, uint32_t* fill,
                                                    float4* __restrict__ pts) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const uint32_t c = cell[i];
    const uint32_t pos = start[c] + atomicAdd(&fill[c], 1u);
    pts[pos] = make_float4(xyz[i * 3], xyz[i * 3 + 1], xyz[i * 3 + 2], __int_as_float((int)i));
  }
}

// Exact k nearest (k <= KC) of every point; avg[original index] = mean distance.
template <int KC>
__global__ __launch_bounds__(kBlock) void k_knn(const float4* __restrict__ pts, int n, const Grid* gp,
                                                const uint32_t* __restrict__ start, int k,
                                                double* __restrict__ avg) {
#pragma clang fp contract(off)
  const int t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= n) return;
  const Grid g = *gp;
  const float4 q = pts[t];
  const int qi = __float_as_int(q.w);
  if (g.bad) {
    avg[qi] = __builtin_nan("");
    return;
  }
  int cx, cy, cz;
  cell_of(g, q.x, q.y, q.z, cx, cy, cz);
  const double qx = q.x, qy = q.y, qz = q.z;
  double best[KC];
#pragma unroll
  for (int m = 0; m < KC; ++m) best[m] = INFINITY;
  double dk = INFINITY;       // best[k - 1]
  int held = 0;
  bool zero = false;          // k candidates at distance 0: nothing can be closer
  for (int r = 0;; ++r) {
    const int x0 = cx - r, x1 = cx + r, y0 = cy - r, y1 = cy + r, z0 = cz - r, z1 = cz + r;
    const int xa = max(x0, 0), xb = min(x1, g.nx - 1);
    for (int z = max(z0, 0); z <= min(z1, g.nz - 1) && !zero; ++z) {
      for (int y = max(y0, 0); y <= min(y1, g.ny - 1) && !zero; ++y) {
        const uint32_t row = ((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx;
        const bool face = (z == z0 || z == z1 || y == y0 || y == y1);
        // a face row of the shell is one contiguous run of cells; an inner row only its two ends
        for (int part = 0; part < 2 && !zero; ++part) {
          int xs, xe;
          if (face) {
            if (part) break;
            xs = xa;
            xe = xb;
          } else {
            const int x = part ? x1 : x0;
            if (x < 0 || x >= g.nx) continue;
            xs = xe = x;
          }
          const int s = (int)start[row + xs], e = (int)start[row + xe + 1];
          for (int j0 = s; j0 < e && !zero; j0 += 4) {
            float4 pf[4];              // four candidate loads in flight per lane
#pragma unroll
            for (int u = 0; u < 4; ++u) pf[u] = pts[min(j0 + u, e - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
            if (j0 + u >= e || zero) break;
            const float4 p = pf[u];
            const double dx = qx - (double)p.x, dy = qy - (double)p.y, dz = qz - (double)p.z;
            const double d2 = (dx * dx + dy * dy) + dz * dz;
            ++held;
            if (d2 < dk) {
              double v = d2;        // sorted insert, the largest falls off the end
#pragma unroll
              for (int m = 0; m < KC; ++m) {
                const double lo = fmin(best[m], v);
                v = fmax(best[m], v);
                best[m] = lo;
              }
              double b = best[0];
#pragma unroll
              for (int m = 1; m < KC; ++m)
                if (m == k - 1) b = best[m];
              dk = b;
              if (dk == 0.0) zero = true;
            }
            }
          }
        }
      }
    }
    if (zero) break;
    if (x0 <= 0 && x1 >= g.nx - 1 && y0 <= 0 && y1 >= g.ny - 1 && z0 <= 0 && z1 >= g.nz - 1) break;  // all scanned
    if (held >= k) {
      // every unscanned point lies beyond one face of the cube [c - r, c + r]
      double bound = INFINITY;
      if (x0 > 0) bound = fmin(bound, qx - (g.ox + (double)x0 * g.h));
      if (x1 < g.nx - 1) bound = fmin(bound, (g.ox + (double)(x1 + 1) * g.h) - qx);
      if (y0 > 0) bound = fmin(bound, qy - (g.oy + (double)y0 * g.h));
      if (y1 < g.ny - 1) bound = fmin(bound, (g.oy + (double)(y1 + 1) * g.h) - qy);
      if (z0 > 0) bound = fmin(bound, qz - (g.oz + (double)z0 * g.h));
      if (z1 < g.nz - 1) bound = fmin(bound, (g.oz + (double)(z1 + 1) * g.h) - qz);
      bound -= g.margin;
      if (bound > 0.0 && dk <= bound * bound) break;
    }
  }
  double s = 0.0;
#pragma unroll
  for (int m = 0; m < KC; ++m)
    if (m < k) s += sqrt(best[m]);
  avg[qi] = s / (double)k;
}

// Fixed-partition partial sums (pass 0: avg > 0; pass 1: (avg - mean)^2 over avg > 0).
__global__ __launch_bounds__(kBlock) void k_sum(const double* __restrict__ avg, int64_t n, const State* st,
                                                int pass, double* part) {
#pragma clang fp contract(off)
  __shared__ double red[kBlock];
  const double mean = pass ? st->mean : 0.0;
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const double x = avg[i];
    if (x > 0) s += pass ? (x - mean) * (x - mean) : x;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void k_sum_final(const double* part, int nb, int64_t n, double ratio, int pass, State* st) {
#pragma clang fp contract(off)
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[b];
  if (pass == 0) {
    st->mean = s / (double)n;
  } else {
    const double sd = sqrt(s / (double)(n - 1));   // n == 1: 0/0 -> NaN -> nothing kept, as Open3D
    st->thr = st->mean + ratio * sd;
  }
}

__global__ __launch_bounds__(kBlock) void k_flags(const double* __restrict__ avg, int64_t n, const State* st,
                                                  uint32_t* __restrict__ flag) {
  const double thr = st->thr;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const double a = avg[i];
    flag[i] = (a > 0.0 && a < thr) ? 1u : 0u;
  }
}

__global__ __launch_bounds__(kBlock) void k_compact(const float* __restrict__ xyz, const uint8_t* __restrict__ rgb,
                                                    int64_t n, const uint32_t* __restrict__ flag,
                                                    const uint32_t* __restrict__ pos, State* st,
                                                    float* __restrict__ oxyz, uint8_t* __restrict__ orgb,
                                                    int64_t* __restrict__ oidx, int64_t* count) {
  uint32_t mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const uint32_t f = flag[i];
    if (i == n - 1) *count = (int64_t)pos[i] + f;
    if (!f) continue;
    const int64_t j = pos[i];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = xyz[i * 3 + c];
      if (oxyz) oxyz[j * 3 + c] = v;
      if (orgb) orgb[j * 3 + c] = rgb[i * 3 + c];
      const uint32_t k = f2key(v);
      mn[c] = min(mn[c], k);
      mx[c] = max(mx[c], k);
    }
    if (oidx) oidx[j] = i;
  }
  block_bbox_atomics(mn, mx, st->kkey);
}

__global__ void k_finish(const State* st, double* bbox) {
  const int t = threadIdx.x;
  if (t >= 6) return;
  const bool none = st->kkey[0] == 0xffffffffu;
  bbox[t] = none ? __builtin_nan("") : (double)key2f(st->kkey[t]);
}

// --- exclusive scan of u32 (three launches: tiles, tile sums, add) ---
__global__ __launch_bounds__(kBlock) void k_scan_tiles(const uint32_t* __restrict__ in, int64_t n,
                                                       uint32_t* __restrict__ out, uint32_t* __restrict__ tsum) {
  __shared__ uint32_t ws[kBlock / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * 4;
  uint32_t v[4], s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = base + j < n ? in[base + j] : 0u;
    s += v[j];
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(s, lane);
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  uint32_t off = 0;
  for (int w = 0; w < wid; ++w) off += ws[w];
  uint32_t run = off + inc - s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
  if (threadIdx.x == kBlock - 1) tsum[blockIdx.x] = off + inc;
}

__global__ __launch_bounds__(1024) void k_scan_sums(uint32_t* tsum, int nt) {
  __shared__ uint32_t ws[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int c0 = 0; c0 < nt; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    const uint32_t x = i < nt ? tsum[i] : 0u;
    const uint32_t inc = wave_incl_scan(x, lane);
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    uint32_t off = carry;
    for (int w = 0; w < wid; ++w) off += ws[w];
    if (i < nt) tsum[i] = off + inc - x;
    __syncthreads();
    if (threadIdx.x == 1023) carry = off + inc;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void k_scan_add(uint32_t* __restrict__ out, int64_t n,
                                                     const uint32_t* __restrict__ tsum) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  const uint32_t a = tsum[blockIdx.x];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = base + threadIdx.x + j * kBlock;
    if (i < n) out[i] += a;
  }
}

static void scan_u32(const uint32_t* in, int64_t n, uint32_t* out, uint32_t* tsum, hipStream_t s) {
  const int nt = (int)((n + kScanTile - 1) / kScanTile);
  hipLaunchKernelGGL(k_scan_tiles, dim3(nt), dim3(kBlock), 0, s, in, n, out, tsum);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, s, tsum, nt);
  hipLaunchKernelGGL(k_scan_add, dim3(nt), dim3(kBlock), 0, s, out, n, tsum);
}

struct Layout {
  size_t grid, state, cell, counts, start, pts, avg, flag, pos, tsum, part, total;
  uint32_t cap;
};

static Layout layout(int64_t n) {
  Layout L{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align_up(o + bytes, 256);
    return at;
  };
  static const int cells_per_point = [] { const char* e = getenv("I2PC_SOR_CELLS"); return e ? atoi(e) : 4; }();
  L.cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(cells_per_point * n, 8), 1 << 24);
  const int64_t nc = (int64_t)L.cap + 1;
  L.grid = take(sizeof(Grid));
  L.state = take(sizeof(State));
  L.cell = take(4 * (size_t)n);
  L.counts = take(4 * (size_t)nc);
  L.start = take(4 * (size_t)nc);
  L.pts = take(16 * (size_t)n);
  L.avg = take(8 * (size_t)n);
  L.flag = take(4 * (size_t)n);
  L.pos = take(4 * (size_t)n);
  const int64_t nt = (std::max<int64_t>(nc, n) + kScanTile - 1) / kScanTile;
  L.tsum = take(4 * (size_t)nt);
  L.part = take(8 * (size_t)kRedBlocks);
  L.total = o;
  return L;
}

static int grid_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, 1024)); }

}  // namespace sor
}  // namespace i2pc

using namespace i2pc;

extern "C" size_t i2pc_sor_workspace_bytes(int64_t n) {
  if (n <= 0) return 256;
  return sor::layout(n).total;
}

extern "C" int i2pc_sor(const float* xyz, const uint8_t* rgb, int64_t n, int nb_neighbors, double std_ratio,
                        float* out_xyz, uint8_t* out_rgb, int64_t* out_index, int64_t* count, double* bbox,
                        double* avg_dist, void* workspace, size_t workspace_bytes, void* stream) {
  using namespace sor;
  clear_error();
  I2PC_REQUIRE(nb_neighbors >= 1 && std_ratio > 0,
               "Illegal input parameters, the number of neighbors and standard deviation ratio must be positive.");
  if (nb_neighbors > 32) return set_error(I2PC_EUNSUPPORTED, "sor: nb_neighbors %d > 32 is not implemented", nb_neighbors);
  I2PC_REQUIRE(n >= 0 && n < (1ll << 31), "sor: n = %lld out of range", (long long)n);
  I2PC_REQUIRE(count != nullptr && workspace != nullptr, "sor: count / workspace is NULL");
  I2PC_REQUIRE(n == 0 || xyz != nullptr, "sor: xyz is NULL");
  I2PC_REQUIRE(out_rgb == nullptr || rgb != nullptr, "sor: out_rgb needs rgb");
  hipStream_t s = as_stream(stream);
  const Layout L = layout(std::max<int64_t>(n, 1));
  if (n > 0 && workspace_bytes < L.total)
    return set_error(I2PC_EWORKSPACE, "sor: workspace %zu < %zu bytes", workspace_bytes, L.total);
  char* ws = static_cast<char*>(workspace);
  State* st = reinterpret_cast<State*>(ws + L.state);
  hipLaunchKernelGGL(k_init, dim3(1), dim3(64), 0, s, st, count);
  if (n == 0) {
    if (bbox) hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, s, st, bbox);
    return check_launch("sor");
  }
  Grid* g = reinterpret_cast<Grid*>(ws + L.grid);
  uint32_t* cell = reinterpret_cast<uint32_t*>(ws + L.cell);
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws + L.counts);
  uint32_t* start = reinterpret_cast<uint32_t*>(ws + L.start);
  float4* pts = reinterpret_cast<float4*>(ws + L.pts);
  double* avg = avg_dist ? avg_dist : reinterpret_cast<double*>(ws + L.avg);
  uint32_t* flag = reinterpret_cast<uint32_t*>(ws + L.flag);
  uint32_t* pos = reinterpret_cast<uint32_t*>(ws + L.pos);
  uint32_t* tsum = reinterpret_cast<uint32_t*>(ws + L.tsum);
  double* part = reinterpret_cast<double*>(ws + L.part);
  const int64_t nc = (int64_t)L.cap + 1;
  const int gb = grid_blocks(n);

  if (hipMemsetAsync(counts, 0, 4 * (size_t)nc, s) != hipSuccess) return set_error(I2PC_ELAUNCH, "sor: memset failed");
  hipLaunchKernelGGL(k_bbox, dim3(gb), dim3(kBlock), 0, s, xyz, n, st);
  hipLaunchKernelGGL(k_grid, dim3(1), dim3(64), 0, s, st, g, L.cap);
  hipLaunchKernelGGL(k_cell, dim3(gb), dim3(kBlock), 0, s, xyz, n, g, cell, counts);
  scan_u32(counts, nc, start, tsum, s);
  if (hipMemsetAsync(counts, 0, 4 * (size_t)nc, s) != hipSuccess) return set_error(I2PC_ELAUNCH, "sor: memset failed");
  hipLaunchKernelGGL(k_scatter, dim3(gb), dim3(kBlock), 0, s, xyz, n, cell, start, counts, pts);
  const int k = (int)std::min<int64_t>(nb_neighbors, n);
  const dim3 kg((unsigned)((n + kBlock - 1) / kBlock));
  if (k <= 8)
    hipLaunchKernelGGL(k_knn<8>, kg, dim3(kBlock), 0, s, pts, (int)n, g, start, k, avg);
  else if (k <= 20)
    hipLaunchKernelGGL(k_knn<20>, kg, dim3(kBlock), 0, s, pts, (int)n, g, start, k, avg);
  else
    hipLaunchKernelGGL(k_knn<32>, kg, dim3(kBlock), 0, s, pts, (int)n, g, start, k, avg);
  const int rb = (int)std::min<int64_t>(kRedBlocks, (n + kBlock - 1) / kBlock);
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(k_sum, dim3(rb), dim3(kBlock), 0, s, avg, n, st, pass, part);
    hipLaunchKernelGGL(k_sum_final, dim3(1), dim3(64), 0, s, part, rb, n, std_ratio, pass, st);
  }
  hipLaunchKernelGGL(k_flags, dim3(gb), dim3(kBlock), 0, s, avg, n, st, flag);
  scan_u32(flag, n, pos, tsum, s);
  hipLaunchKernelGGL(k_compact, dim3(gb), dim3(kBlock), 0, s, xyz, rgb, n, flag, pos, st, out_xyz, out_rgb,
                     out_index, count);
  if (bbox) hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, s, st, bbox);
  return check_launch("sor");
}

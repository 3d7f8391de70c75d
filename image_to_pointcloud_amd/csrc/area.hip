// Area-averaging downscale of uint8 images: cv2.resize(image, (new_w, new_h),
// interpolation=cv2.INTER_AREA), which process_image_pipeline applies to inputs above
// MAX_IMAGE_DIM = 3072 px (backend/app.py:436-445).  OpenCV is not in this image, so the
// arithmetic restates OpenCV's published algorithm (imgproc/src/resize.cpp) -- parity
// unpinned against cv2 itself, pinned against oracle/area_ref.py:
//  * scale = 1 / (dst / src) per axis (double); integer scales in both axes take the
//    "area fast" box average: int sum * (1.f / area) rounded half-to-even, except 2 x 2,
//    whose vector path is (sum + 2) >> 2;
//  * otherwise each output pixel is sum_y beta_y * (sum_x alpha_x * S[y][x]) in float in
//    OpenCV's accumulation order, with the cell weights of computeResizeAreaTab (partial
//    border cells kept when they exceed 1e-3), rounded half-to-even and saturated.
// One thread per output pixel and channel group; the source window is at most
// ceil(scale) + 1 pixels per axis and is L2/L1 resident.
#include "common.h"

#include <cmath>

namespace i2pc {
namespace area {

#pragma clang fp contract(off)

struct Cells {
  int s0, n;            // first source index, number of cells
  float first, mid, last;   // weight of cell 0, cells 1..n-2, cell n-1
};

// computeResizeAreaTab for destination index d
__device__ __forceinline__ Cells cells(int d, int ssize, double scale) {
  const double f1 = d * scale, f2 = f1 + scale;
  const double cw = fmin(scale, (double)ssize - f1);
  int s1 = (int)ceil(f1), s2 = (int)floor(f2);
  s2 = min(s2, ssize - 1);
  s1 = min(s1, s2);
  const bool left = s1 - f1 > 1e-3, right = f2 - s2 > 1e-3;
  Cells c;
  c.s0 = left ? s1 - 1 : s1;
  c.n = (left ? 1 : 0) + (s2 - s1) + (right ? 1 : 0);
  const float full = (float)(1.0 / cw);
  c.mid = full;
  c.first = left ? (float)((s1 - f1) / cw) : full;
  c.last = right ? (float)(fmin(fmin(f2 - s2, 1.0), cw) / cw) : full;
  if (c.n == 1) c.first = left ? c.first : c.last;
  return c;
}

__device__ __forceinline__ float weight(const Cells& c, int i) {
  return i == 0 ? c.first : (i == c.n - 1 ? c.last : c.mid);
}

__device__ __forceinline__ uint8_t sat_round(float v) {
  const float r = rintf(v);                 // cvRound: half to even
  return (uint8_t)fminf(fmaxf(r, 0.f), 255.f);
}

template <int C>
__global__ __launch_bounds__(256) void k_area(const uint8_t* __restrict__ src, int B, int h, int w, uint8_t* __restrict__ dst,
                                              int H, int W, double sy, double sx, int fast, int iy, int ix) {
  const int64_t total = (int64_t)B * H * W;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(p % W);
    const int64_t r = p / W;
    const int oy = (int)(r % H);
    const int b = (int)(r / H);
    const uint8_t* S = src + (int64_t)b * h * w * C;
    uint8_t out[C];
    if (fast) {
      int sum[C];
#pragma unroll
      for (int c = 0; c < C; ++c) sum[c] = 0;
      for (int y = 0; y < iy; ++y)
        for (int x = 0; x < ix; ++x) {
          const uint8_t* q = S + ((int64_t)(oy * iy + y) * w + (ox * ix + x)) * C;
#pragma unroll
          for (int c = 0; c < C; ++c) sum[c] += q[c];
        }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if (iy == 2 && ix == 2) out[c] = (uint8_t)((sum[c] + 2) >> 2);
        else out[c] = sat_round((float)sum[c] * (1.f / (float)(iy * ix)));
      }
    } else {
      const Cells cy = cells(oy, h, sy), cx = cells(ox, w, sx);
      float acc[C];
      for (int j = 0; j < cy.n; ++j) {
        const float beta = weight(cy, j);
        const uint8_t* row = S + (int64_t)(cy.s0 + j) * w * C;
        float buf[C];
#pragma unroll
        for (int c = 0; c < C; ++c) buf[c] = 0.f;
        for (int i = 0; i < cx.n; ++i) {
          const float alpha = weight(cx, i);
          const uint8_t* q = row + (int64_t)(cx.s0 + i) * C;
#pragma unroll
          for (int c = 0; c < C; ++c) buf[c] = buf[c] + (float)q[c] * alpha;
        }
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = j == 0 ? beta * buf[c] : acc[c] + beta * buf[c];
      }
#pragma unroll
      for (int c = 0; c < C; ++c) out[c] = sat_round(acc[c]);
    }
    uint8_t* d = dst + p * C;
#pragma unroll
    for (int c = 0; c < C; ++c) d[c] = out[c];
  }
}

}  // namespace area
}  // namespace i2pc

using namespace i2pc;

extern "C" int i2pc_resize_area(const uint8_t* src, int batch, int h, int w, int channels, uint8_t* dst, int out_h,
                                int out_w, void* stream) {
  clear_error();
  I2PC_REQUIRE(src && dst, "resize_area: NULL pointer");
  I2PC_REQUIRE(batch > 0 && h > 0 && w > 0 && out_h > 0 && out_w > 0, "resize_area: empty shape");
  I2PC_REQUIRE(channels >= 1 && channels <= 4, "resize_area: channels must be 1..4");
  if (out_h > h || out_w > w)
    return set_error(I2PC_EUNSUPPORTED, "resize_area: only downscaling is implemented (%dx%d -> %dx%d)", w, h, out_w, out_h);
  const double sx = 1.0 / ((double)out_w / w), sy = 1.0 / ((double)out_h / h);
  const int ix = (int)lrint(sx), iy = (int)lrint(sy);
  const int fast = std::fabs(sx - ix) < 2.220446049250313e-16 && std::fabs(sy - iy) < 2.220446049250313e-16;
  const int64_t total = (int64_t)batch * out_h * out_w;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 16384);
  hipStream_t s = as_stream(stream);
  switch (channels) {
    case 1: hipLaunchKernelGGL(area::k_area<1>, dim3(blocks), dim3(256), 0, s, src, batch, h, w, dst, out_h, out_w, sy, sx, fast, iy, ix); break;
    case 2: hipLaunchKernelGGL(area::k_area<2>, dim3(blocks), dim3(256), 0, s, src, batch, h, w, dst, out_h, out_w, sy, sx, fast, iy, ix); break;
    case 3: hipLaunchKernelGGL(area::k_area<3>, dim3(blocks), dim3(256), 0, s, src, batch, h, w, dst, out_h, out_w, sy, sx, fast, iy, ix); break;
    default: hipLaunchKernelGGL(area::k_area<4>, dim3(blocks), dim3(256), 0, s, src, batch, h, w, dst, out_h, out_w, sy, sx, fast, iy, ix); break;
  }
  return check_launch("resize_area");
}

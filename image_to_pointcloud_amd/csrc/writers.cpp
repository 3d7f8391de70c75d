// Point-cloud artefact writers (host side of the C ABI): the file formats the
// reference's save_point_cloud produces (backend/app.py:310-389), written from
// host buffers (the caller copies xyz/rgb off the device once, pinned).
//
//   XYZ  app.py:380-389   "%.6f %.6f %.6f %d %d %d\n" per point (Python's 'f'
//                         formatting and glibc's are both correctly rounded);
//                         lines are formatted by several threads into
//                         per-thread buffers and written in order.
//   PLY  app.py:333-345   Open3D write_point_cloud defaults: binary little
//                         endian, double x/y/z, uchar red/green/blue where the
//                         colour went float32(c / 255) -> double -> * 255 ->
//                         clamp -> truncating uchar store (rply).  Open3D is
//                         absent here: layout restated, parity unpinned.
//   LAS  app.py:347-378   LAS 1.2, point format 2 (26-byte records), scale 0.01,
//                         offset = per-axis min, X = round((x - offset) / scale),
//                         RGB = c * 256.  laspy is absent: restated, parity unpinned.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

using namespace i2pc;

namespace {

struct File {
  FILE* f = nullptr;
  explicit File(const char* path) : f(std::fopen(path, "wb")) {}
  ~File() {
    if (f) std::fclose(f);
  }
  bool write(const void* p, size_t n) { return n == 0 || std::fwrite(p, 1, n, f) == n; }
};

template <class T>
void put(std::vector<char>& b, T v) {
  const char* p = reinterpret_cast<const char*>(&v);
  b.insert(b.end(), p, p + sizeof(T));
}

}  // namespace

extern "C" int i2pc_write_xyz(const char* path, const float* xyz, const uint8_t* rgb, int64_t n, int threads) {
  clear_error();
  I2PC_REQUIRE(path && (n == 0 || xyz), "write_xyz: NULL argument");
  I2PC_REQUIRE(n >= 0, "write_xyz: negative count");
  File out(path);
  if (!out.f) return set_error(I2PC_EINVAL, "write_xyz: cannot open %s", path);
  const int T = std::max(1, std::min(threads > 0 ? threads : 1, 64));
  constexpr int64_t kChunk = 1 << 16;                 // points per formatting task
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  for (int64_t c0 = 0; c0 < nchunks; c0 += T) {
    const int64_t cend = std::min<int64_t>(nchunks, c0 + T);
    std::vector<std::string> buf(cend - c0);
    auto work = [&](int64_t c) {
      std::string& s = buf[c - c0];
      const int64_t i0 = c * kChunk, i1 = std::min(n, i0 + kChunk);
      s.reserve((size_t)(i1 - i0) * 48);
      char line[160];
      for (int64_t i = i0; i < i1; ++i) {
        const int r = rgb ? rgb[i * 3] : 128, g = rgb ? rgb[i * 3 + 1] : 128, b = rgb ? rgb[i * 3 + 2] : 128;
        const int k = std::snprintf(line, sizeof(line), "%.6f %.6f %.6f %d %d %d\n", (double)xyz[i * 3],
                                    (double)xyz[i * 3 + 1], (double)xyz[i * 3 + 2], r, g, b);
        s.append(line, (size_t)k);
      }
    };
    std::vector<std::thread> pool;
    for (int64_t c = c0 + 1; c < cend; ++c) pool.emplace_back(work, c);
    work(c0);
    for (auto& t : pool) t.join();
    for (auto& s : buf)
      if (!out.write(s.data(), s.size())) return set_error(I2PC_EINVAL, "write_xyz: write failed");
  }
  return I2PC_OK;
}

extern "C" int i2pc_write_ply(const char* path, const float* xyz, const uint8_t* rgb, int64_t n) {
  clear_error();
  I2PC_REQUIRE(path && (n == 0 || xyz), "write_ply: NULL argument");
  I2PC_REQUIRE(n >= 0, "write_ply: negative count");
  File out(path);
  if (!out.f) return set_error(I2PC_EINVAL, "write_ply: cannot open %s", path);
  std::string h = "ply\nformat binary_little_endian 1.0\ncomment Created by Open3D\nelement vertex " +
                  std::to_string(n) + "\nproperty double x\nproperty double y\nproperty double z\n";
  if (rgb) h += "property uchar red\nproperty uchar green\nproperty uchar blue\n";
  h += "end_header\n";
  if (!out.write(h.data(), h.size())) return set_error(I2PC_EINVAL, "write_ply: write failed");
  const size_t rec = 24 + (rgb ? 3 : 0);
  std::vector<char> b;
  constexpr int64_t kChunk = 1 << 16;
  b.reserve(rec * kChunk);
  for (int64_t i0 = 0; i0 < n; i0 += kChunk) {
    b.clear();
    const int64_t i1 = std::min(n, i0 + kChunk);
    for (int64_t i = i0; i < i1; ++i) {
      for (int c = 0; c < 3; ++c) put<double>(b, (double)xyz[i * 3 + c]);
      if (rgb)
        for (int c = 0; c < 3; ++c) {
          const float unit = (float)rgb[i * 3 + c] / 255.0f;       // colors / 255.0 in float32 (NEP 50)
          const double v = std::min(255.0, std::max(0.0, (double)unit * 255.0));
          put<uint8_t>(b, (uint8_t)v);
        }
    }
    if (!out.write(b.data(), b.size())) return set_error(I2PC_EINVAL, "write_ply: write failed");
  }
  return I2PC_OK;
}

extern "C" int i2pc_write_las(const char* path, const float* xyz, const uint8_t* rgb, int64_t n, double scale) {
  clear_error();
  I2PC_REQUIRE(path && xyz, "write_las: NULL argument");
  I2PC_REQUIRE(n > 0, "write_las: no points to write");        // app.py:360-361
  I2PC_REQUIRE(n <= 0xffffffffll, "write_las: LAS 1.2 holds at most 2^32-1 points");
  I2PC_REQUIRE(scale > 0, "write_las: scale must be positive");
  double mn[3], mx[3];
  for (int c = 0; c < 3; ++c) { mn[c] = INFINITY; mx[c] = -INFINITY; }
  for (int64_t i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) {
      const double v = xyz[i * 3 + c];
      mn[c] = std::min(mn[c], v);
      mx[c] = std::max(mx[c], v);
    }
  const double* off = mn;                                           // app.py:354
  auto q = [&](double v, int c) { return (int32_t)std::nearbyint((v - off[c]) / scale); };
  // header min/max are the stored (quantised) extents
  double qmn[3], qmx[3];
  for (int c = 0; c < 3; ++c) {
    qmn[c] = q(mn[c], c) * scale + off[c];
    qmx[c] = q(mx[c], c) * scale + off[c];
  }
  std::vector<char> h;
  h.reserve(227);
  h.insert(h.end(), {'L', 'A', 'S', 'F'});
  put<uint16_t>(h, 0);          // file source id
  put<uint16_t>(h, 0);          // global encoding
  for (int i = 0; i < 16; ++i) put<uint8_t>(h, 0);   // project GUID
  put<uint8_t>(h, 1);           // version 1.2
  put<uint8_t>(h, 2);
  char sys[32] = "OTHER", gen[32] = "image_to_pointcloud_amd";
  h.insert(h.end(), sys, sys + 32);
  h.insert(h.end(), gen, gen + 32);
  const std::time_t now = std::time(nullptr);
  std::tm tm{};
  gmtime_r(&now, &tm);
  put<uint16_t>(h, (uint16_t)(tm.tm_yday + 1));
  put<uint16_t>(h, (uint16_t)(tm.tm_year + 1900));
  put<uint16_t>(h, 227);        // header size
  put<uint32_t>(h, 227);        // offset to point data
  put<uint32_t>(h, 0);          // number of VLRs
  put<uint8_t>(h, 2);           // point data format 2
  put<uint16_t>(h, 26);         // point record length
  put<uint32_t>(h, (uint32_t)n);
  for (int i = 0; i < 5; ++i) put<uint32_t>(h, 0);   // points by return (laspy: return_number left 0)
  for (int c = 0; c < 3; ++c) put<double>(h, scale);
  for (int c = 0; c < 3; ++c) put<double>(h, off[c]);
  for (int c = 0; c < 3; ++c) {
    put<double>(h, qmx[c]);
    put<double>(h, qmn[c]);
  }
  if (h.size() != 227) return set_error(I2PC_EINVAL, "write_las: header size %zu", h.size());
  File out(path);
  if (!out.f) return set_error(I2PC_EINVAL, "write_las: cannot open %s", path);
  if (!out.write(h.data(), h.size())) return set_error(I2PC_EINVAL, "write_las: write failed");
  std::vector<char> b;
  constexpr int64_t kChunk = 1 << 16;
  b.reserve(26 * kChunk);
  for (int64_t i0 = 0; i0 < n; i0 += kChunk) {
    b.clear();
    const int64_t i1 = std::min(n, i0 + kChunk);
    for (int64_t i = i0; i < i1; ++i) {
      for (int c = 0; c < 3; ++c) put<int32_t>(b, q(xyz[i * 3 + c], c));
      put<uint16_t>(b, 0);      // intensity
      put<uint8_t>(b, 0);       // return number / number of returns / flags (left 0, as laspy does)
      put<uint8_t>(b, 0);       // classification
      put<int8_t>(b, 0);        // scan angle rank
      put<uint8_t>(b, 0);       // user data
      put<uint16_t>(b, 0);      // point source id
      for (int c = 0; c < 3; ++c) put<uint16_t>(b, (uint16_t)((rgb ? rgb[i * 3 + c] : 128) * 256));
    }
    if (!out.write(b.data(), b.size())) return set_error(I2PC_EINVAL, "write_las: write failed");
  }
  return I2PC_OK;
}

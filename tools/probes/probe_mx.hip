// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3) operand and scale lane maps on gfx950.
// What csrc/gemm.hip's fp8 engine relies on (measured r02, "MX LAYOUT OK"):
//   byte j of lane l's 8 A VGPRs pairs with byte j of lane l' in the same 16-lane group
//   g = l >> 4 (A row l & 15, B column l' & 15), and the MFMA's k index of that pair is
//   kh(g, j) = j < 16 ? 16 g + j : 64 + 16 g + (j - 16);
//   D: lane l, reg r = D[row = 4 * (l >> 4) + r][col = l & 15];
//   scale_a (opsel 0): byte 0 of lane l's VGPR = E8M0 scale of A row (l & 15) over
//   kh in [32 (l >> 4), 32 (l >> 4) + 32); scale_b likewise for B column (l & 15).
// So a lane of group g loads 16-B chunks g and 4 + g of a 128-k row and passes the scale of
// 32-k block g: memory k order = kh, scale block b = memory k [32 b, 32 b + 32).
//   hipcc --offload-arch=gfx950 -O2 tools/probes/probe_mx.hip -o /tmp/probe_mx && /tmp/probe_mx
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// e4m3fn encodings of 0.5, 1 .. 16 (exact)
__host__ __device__ inline uint8_t e4m3_int(int v) {
  if (v == 0) return 0;
  int e = 31 - __builtin_clz(v);          // floor log2
  int m = (v << 3 >> e) & 7;              // 3 mantissa bits (v <= 16 -> exact)
  return (uint8_t)(((e + 7) << 3) | m);
}

// mode 0: A one-hot at (L, J) = 1, B(l', j') = code
__global__ void k_probe(const uint8_t* bvals, int sa_lane, int sb_lane, float* out) {
  const int l = threadIdx.x;
  for (int pos = 0; pos < 64 * 32; ++pos) {
    const int L = pos >> 5, J = pos & 31;
    uint8_t a[32], b[32];
    for (int j = 0; j < 32; ++j) {
      a[j] = (l == L && j == J) ? e4m3_int(1) : 0;
      b[j] = bvals[l * 32 + j];
    }
    i32x8 av, bv;
    __builtin_memcpy(&av, a, 32);
    __builtin_memcpy(&bv, b, 32);
    const int sa = (l == sa_lane) ? 128 : 127;
    const int sb = (l == sb_lane) ? 129 : 127;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sa, 0, sb);
    for (int r = 0; r < 4; ++r) out[(size_t)pos * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
  }
}

int main() {
  // B code: value = 1 + (j % 16) for the k-low code, second run 1 + (l >> 4) * 2 + (j >> 4)
  std::vector<uint8_t> b1(64 * 32), b2(64 * 32);
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 32; ++j) {
      b1[l * 32 + j] = e4m3_int(1 + (j % 16));
      b2[l * 32 + j] = e4m3_int(1 + (l >> 4) * 2 + (j >> 4));
    }
  uint8_t* db; float* dout;
  hipMalloc(&db, 64 * 32);
  hipMalloc(&dout, sizeof(float) * 2048 * 256);
  std::vector<float> o1(2048 * 256), o2(2048 * 256), o3(2048 * 256);
  hipMemcpy(db, b1.data(), 64 * 32, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, db, -1, -1, dout);
  hipMemcpy(o1.data(), dout, sizeof(float) * 2048 * 256, hipMemcpyDeviceToHost);
  hipMemcpy(db, b2.data(), 64 * 32, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, db, -1, -1, dout);
  hipMemcpy(o2.data(), dout, sizeof(float) * 2048 * 256, hipMemcpyDeviceToHost);
  // scales: lane 21 of A (row 5, k-block 1) x2, lane 37 of B (col 5, k-block 2) x4
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, db, 21, 37, dout);
  hipMemcpy(o3.data(), dout, sizeof(float) * 2048 * 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int pos = 0; pos < 2048; ++pos) {
    const int L = pos >> 5, J = pos & 31;
    const int row = L & 15, k = 32 * (L >> 4) + J;
    for (int m = 0; m < 16; ++m)
      for (int n = 0; n < 16; ++n) {
        const float v1 = o1[pos * 256 + m * 16 + n], v2 = o2[pos * 256 + m * 16 + n], v3 = o3[pos * 256 + m * 16 + n];
        // expected: row m == row; B element k at column n: lane (k >> 5) * 16 + n, byte k & 31
        const float e1 = m == row ? (float)(1 + ((k & 31) % 16)) : 0.f;
        const float e2 = m == row ? (float)(1 + (k >> 5) * 2 + ((k & 31) >> 4)) : 0.f;
        float sc = 1.f;
        const int g = L >> 4, kh = J < 16 ? 16 * g + J : 64 + 16 * g + (J - 16);
        if (row == 5 && (kh >> 5) == 1) sc *= 2.f;       // A lane 21: row 5, block 1
        if (n == 5 && (kh >> 5) == 2) sc *= 4.f;         // B lane 37: column 5, block 2
        const float e3 = e2 * sc;
        if (v1 != e1 || v2 != e2 || v3 != e3) {
          if (bad < 10) printf("mismatch A(l=%d,j=%d) D[%d][%d]: %g %g %g expected %g %g %g\n", L, J, m, n, v1, v2, v3, e1, e2, e3);
          ++bad;
        }
      }
  }
  // observed scale factors per k: A lane 21 (x2) seen at row 5 / col != 5, B lane 37 (x4) at col 5 / row != 5
  printf("A-scale k:");
  for (int pos = 0; pos < 2048; ++pos) {
    const int L = pos >> 5, J = pos & 31, row = L & 15, k = 32 * (L >> 4) + J;
    if (row != 5) continue;
    const float f = o3[pos * 256 + 5 * 16 + 0] / o2[pos * 256 + 5 * 16 + 0];
    if (f != 1.f) printf(" %d(x%g)", k, f);
  }
  printf("\nB-scale k (row 0):");
  for (int pos = 0; pos < 2048; ++pos) {
    const int L = pos >> 5, J = pos & 31, row = L & 15, k = 32 * (L >> 4) + J;
    if (row != 0) continue;
    const float f = o3[pos * 256 + 0 * 16 + 5] / o2[pos * 256 + 0 * 16 + 5];
    if (f != 1.f) printf(" %d(x%g)", k, f);
  }
  printf("\n");
  printf(bad ? "MX LAYOUT MISMATCH: %d\n" : "MX LAYOUT OK (%d mismatches)\n", bad);
  return bad != 0;
}

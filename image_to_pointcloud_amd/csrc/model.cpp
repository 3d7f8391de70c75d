// Native network executor: the whole depth stage of process_with_depth_anything
// (backend/app.py:99-122 -- BGR->RGB :103, the processor :109, the forward :111-116) behind the
// C ABI, with no Python.  i2pc_model_create reads a prepared-network file (model_file.py writes
// it from a loaded DepthAnythingModel: every weight already in the kernels' layout, the position
// table interpolated for the input size), uploads the weights and allocates every activation
// buffer once; i2pc_depth_forward then issues exactly the launches DepthAnythingModel.forward
// issues (LayerNorm folded through QKV / FC1, the shifted bf16 residual stream, the fused head),
// in the same order with the same descriptors, on the caller's stream -- no allocation, no host
// synchronisation, so a forward can be captured into a HIP graph.  The depth equals the Python
// path's bit for bit (tests/test_model_file_gpu.py).
#include "common.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace i2pc {
namespace model {

constexpr char kMagic[8] = {'I', '2', 'P', 'C', 'N', 'E', 'T', '1'};
// int header slots (model_file.py I_*)
enum {
  I_FAMILY = 0, I_VERSION = 1, I_IN_H = 2, I_IN_W = 3, I_OUT_H = 4, I_OUT_W = 5, I_GH = 6, I_GW = 7, I_PATCH = 8,
  I_HIDDEN = 9, I_LAYERS = 10, I_HEADS = 11, I_MLP = 12, I_FUSION = 13, I_HEAD_HIDDEN = 14, I_H1P = 15,
  I_NECK0 = 16, I_FAC0 = 20, I_OUT0 = 24, I_NTENSORS = 28, I_PITCH = 29
};
enum { F_EPS = 0, F_B_H3 = 1, F_MEAN0 = 2, F_STD0 = 5 };
constexpr int kFamilyDepthAnything = 1;
constexpr int kLnChunk = 32;   // depth_anything.LN_CHUNK

#pragma pack(push, 1)
struct Entry {
  char name[48];
  int32_t dtype, ndim;
  int64_t dims[4];
  int64_t offset, nbytes;
};
#pragma pack(pop)
static_assert(sizeof(Entry) == 48 + 8 + 32 + 16, "entry layout");

struct Map {   // an NHWC bf16 map
  void* p = nullptr;
  int b = 0, h = 0, w = 0, c = 0;
};

}  // namespace model
}  // namespace i2pc

struct i2pc_model {
  int32_t ints[32];
  float floats[16];
  int batch = 0;
  std::map<std::string, void*> w;          // device weights by name
  void* arena = nullptr;                    // weights
  std::vector<void*> bufs;                  // activations (freed at destroy)
  i2pc_preprocess_plan* plan = nullptr;
  void* ws = nullptr;                       // split-K workspace (the largest any call asks)
  size_t ws_bytes = 0;
  // activations
  void *patches = nullptr, *x = nullptr, *ln = nullptr, *qkv = nullptr, *att = nullptr, *mlp = nullptr;
  void *part = nullptr, *rs = nullptr, *sh0 = nullptr, *sh1 = nullptr;
  void* hs[4] = {nullptr, nullptr, nullptr, nullptr};
  i2pc::model::Map proj[4], rsz[4], feat[4];
  struct Fuse { i2pc::model::Map t, h, t2, h2, p, up; } fuse[4];
  i2pc::model::Map head_t;
};

namespace i2pc {
namespace model {

static void* get(i2pc_model* m, const std::string& name) {
  auto it = m->w.find(name);
  return it == m->w.end() ? nullptr : it->second;
}

static void* dalloc(i2pc_model* m, size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, std::max<size_t>(bytes, 256)) != hipSuccess) return nullptr;
  m->bufs.push_back(p);
  return p;
}

static bool alloc_map(i2pc_model* m, Map& mp, int b, int h, int w, int c) {
  mp.b = b; mp.h = h; mp.w = w; mp.c = c;
  mp.p = dalloc(m, (size_t)b * h * w * c * 2);
  return mp.p != nullptr;
}

// ---- the ops the forward uses: descriptors exactly as ops.py builds them
static i2pc_gemm_desc desc0() {
  i2pc_gemm_desc d;
  std::memset(&d, 0, sizeof d);
  return d;
}

// ops.conv2d: NHWC implicit GEMM (a plain GEMM for 1x1 / stride 1 / pad 0)
static i2pc_gemm_desc conv_desc(const Map& x, const void* w, const float* bias, int co, int k, int stride, int pad,
                                bool relu_in, int act, const void* res, const void* res2, const Map& out) {
  i2pc_gemm_desc d = desc0();
  d.a = x.p; d.lda = x.c; d.m = x.b * out.h * out.w; d.n = co; d.k = k * k * x.c;
  if (!(k == 1 && stride == 1 && pad == 0 && out.h == x.h && out.w == x.w)) {
    d.conv = 1; d.conv_batch = x.b; d.conv_h = x.h; d.conv_w = x.w; d.conv_c = x.c;
    d.conv_oh = out.h; d.conv_ow = out.w; d.conv_k = k; d.conv_stride = stride; d.conv_pad = pad;
  }
  d.conv_relu_in = relu_in ? 1 : 0;
  d.w = w; d.ldw = (int64_t)k * k * x.c;
  d.bias = bias;
  d.act = act;
  if (res) { d.res = res; d.res_f32 = 0; d.ldr = co; }
  if (res2) { d.res2 = res2; d.ldr2 = co; }
  d.c = out.p; d.c_f32 = 0; d.ldc = co;
  return d;
}

}  // namespace model
}  // namespace i2pc
int i2pc_gemm_check(const i2pc_gemm_desc* d, size_t* workspace_bytes);   // gemm.hip (no launch)
namespace i2pc {
namespace model {

// plan pass: every descriptor validated and planned as the launch would (an error here fails
// i2pc_model_create before any kernel runs), and the largest split-K workspace recorded; run pass: launch
static int gemm(i2pc_model* m, const i2pc_gemm_desc& d, bool plan, hipStream_t s) {
  if (plan) {
    size_t ws = 0;
    const int rc = i2pc_gemm_check(&d, &ws);
    if (rc != I2PC_OK) return rc;
    m->ws_bytes = std::max(m->ws_bytes, ws);
    return I2PC_OK;
  }
  return i2pc_gemm_ws(&d, m->ws, m->ws_bytes, s);
}

#define TRY(x)                      \
  do {                              \
    const int rc_ = (x);            \
    if (rc_ != I2PC_OK) return rc_; \
  } while (0)

// DepthAnythingModel.forward (depth_anything.py) on the defaults: LN_FOLD, BF16_STREAM, FUSED_HEAD
static int forward_da(i2pc_model* m, const uint8_t* bgr, float* depth, bool plan, hipStream_t s) {
  const int* I = m->ints;
  const int B = m->batch, D = I[I_HIDDEN], gh = I[I_GH], gw = I[I_GW], np_ = gh * gw, T = np_ + 1;
  const int M = B * T, F = I[I_FUSION], heads = I[I_HEADS], kp = I[I_PITCH];
  const float eps = m->floats[F_EPS];
  auto W = [&](const std::string& n) { return get(m, n); };
  auto Wf = [&](const std::string& n) { return static_cast<const float*>(get(m, n)); };
  if (!plan) TRY(i2pc_preprocess(m->plan, bgr, B, 1, m->patches, s));
  // patch embedding + position table, tokens 1.. of each image (out_map), then the CLS rows
  {
    i2pc_gemm_desc d = desc0();
    d.a = m->patches; d.lda = kp; d.m = B * np_; d.n = D; d.k = kp;
    d.w = W("pe.w"); d.ldw = kp; d.bias = Wf("pe.b");
    d.table = Wf("pos.table"); d.table_rows = np_;
    d.c = m->x; d.c_f32 = 1; d.ldc = D;
    d.out_group = np_; d.out_group_stride = T; d.out_offset = 1;
    TRY(gemm(m, d, plan, s));
  }
  if (!plan) TRY(i2pc_cls_pos(Wf("cls"), Wf("pos0"), B, T, D, static_cast<float*>(m->x), s));
  // encoder on the shifted bf16 residual stream (depth_anything._encoder_stream)
  const void* res = m->x;
  bool res_f32 = true;
  const float* rsh = nullptr;
  float* sh0 = static_cast<float*>(m->sh0);
  float* sh1 = static_cast<float*>(m->sh1);
  int hs_i = 0;
  for (int i = 0; i < I[I_LAYERS]; ++i) {
    const std::string L = "L" + std::to_string(i) + ".";
    i2pc_gemm_desc d = desc0();
    if (i == 0) {
      if (!plan)
        TRY(i2pc_layernorm_stats(static_cast<const float*>(m->x), D, Wf(L + "ln1_g"), Wf(L + "ln1_b"), eps, M, D, m->ln,
                                 D, sh0, s));
      d.a = m->ln; d.lda = D; d.m = M; d.n = 3 * D; d.k = D;
      d.w = W(L + "w_qkv"); d.ldw = D; d.bias = Wf(L + "b_qkv");
      d.c = m->qkv; d.ldc = 3 * D;
    } else {
      d.a = m->ln; d.lda = D; d.m = M; d.n = 3 * D; d.k = D;
      d.w = W(L + "w_qkv_f"); d.ldw = D; d.bias = Wf(L + "b_qkv_f");
      d.ln_rows = static_cast<const float*>(m->rs); d.col_sum = Wf(L + "s_qkv");
      d.c = m->qkv; d.ldc = 3 * D;
    }
    TRY(gemm(m, d, plan, s));
    if (!plan) TRY(i2pc_attention_q2(m->qkv, B, T, heads, m->att, s));   // Q folded (file version 2)
    // attention-out + residual -> the stream (bf16, relative to sh0) + 32-column partials
    d = desc0();
    d.a = m->att; d.lda = D; d.m = M; d.n = D; d.k = D;
    d.w = W(L + "w_o"); d.ldw = D; d.bias = Wf(L + "b_o");
    d.res = res; d.res_f32 = res_f32 ? 1 : 0; d.ldr = D;
    d.c = m->ln; d.c_f32 = 0; d.ldc = D;
    d.ln_part = static_cast<float*>(m->part); d.ln_chunk = kLnChunk; d.ln_shift = sh0;
    d.res_shift = rsh;
    TRY(gemm(m, d, plan, s));
    if (!plan)
      TRY(i2pc_ln_rowstats_w(static_cast<const float*>(m->part), M, D / kLnChunk, kLnChunk, eps,
                             static_cast<float*>(m->rs), sh0, sh1, s));
    d = desc0();                                           // FC1 + GELU, norm2 folded
    d.a = m->ln; d.lda = D; d.m = M; d.n = I[I_MLP]; d.k = D;
    d.w = W(L + "w_1_f"); d.ldw = D; d.bias = Wf(L + "b_1_f"); d.act = 1;
    d.ln_rows = static_cast<const float*>(m->rs); d.col_sum = Wf(L + "s_1");
    d.c = m->mlp; d.ldc = I[I_MLP];
    TRY(gemm(m, d, plan, s));
    d = desc0();                                           // FC2 + residual, in place on the stream
    d.a = m->mlp; d.lda = I[I_MLP]; d.m = M; d.n = D; d.k = I[I_MLP];
    d.w = W(L + "w_2"); d.ldw = I[I_MLP]; d.bias = Wf(L + "b_2");
    d.res = m->ln; d.res_f32 = 0; d.ldr = D; d.res_shift = sh0;
    d.c = m->ln; d.c_f32 = 0; d.ldc = D;
    d.ln_part = static_cast<float*>(m->part); d.ln_chunk = kLnChunk; d.ln_shift = sh1;
    TRY(gemm(m, d, plan, s));
    if (!plan)
      TRY(i2pc_ln_rowstats_w(static_cast<const float*>(m->part), M, D / kLnChunk, kLnChunk, eps,
                             static_cast<float*>(m->rs), sh1, sh0, s));
    res = m->ln;
    res_f32 = false;
    rsh = sh1;
    for (int k = 0; k < 4; ++k)
      if (I[I_OUT0 + k] == i + 1) {   // backbone LayerNorm of a kept hidden state
        if (!plan) TRY(i2pc_ln_apply(m->ln, D, static_cast<const float*>(m->rs), Wf("ln_g"), Wf("ln_b"), M, D,
                                     m->hs[hs_i], D, s));
        ++hs_i;
      }
  }
  // reassemble (drop CLS by the A row map) + neck convs
  for (int j = 0; j < 4; ++j) {
    const std::string S = "S" + std::to_string(j) + ".";
    const int c = I[I_NECK0 + j], fac = I[I_FAC0 + j];
    i2pc_gemm_desc d = desc0();
    d.a = m->hs[j]; d.lda = D; d.m = B * np_; d.n = c; d.k = D;
    d.a_group = np_; d.a_group_stride = T; d.a_offset = 1;
    d.w = W(S + "w_proj"); d.ldw = D; d.bias = Wf(S + "b_proj");
    d.c = m->proj[j].p; d.ldc = c;
    TRY(gemm(m, d, plan, s));
    const Map* r = &m->proj[j];
    if (fac > 1) {                                         // ConvTranspose(fac, stride fac)
      d = desc0();
      d.a = m->proj[j].p; d.lda = c; d.m = B * np_; d.n = fac * fac * c; d.k = c;
      d.w = W(S + "w_rs"); d.ldw = c; d.bias = Wf(S + "b_rs");
      d.c = m->rsz[j].p; d.c_f32 = 0; d.ldc = c;
      d.convt_s = fac; d.convt_h = gh; d.convt_w = gw; d.convt_c = c;
      TRY(gemm(m, d, plan, s));
      r = &m->rsz[j];
    } else if (fac < 0) {                                  // 3x3 stride -fac conv
      TRY(gemm(m, conv_desc(m->proj[j], W(S + "w_rs"), Wf(S + "b_rs"), c, 3, -fac, 1, false, 0, nullptr, nullptr,
                            m->rsz[j]), plan, s));
      r = &m->rsz[j];
    }
    TRY(gemm(m, conv_desc(*r, W(S + "w_neck"), nullptr, F, 3, 1, 1, false, 0, nullptr, nullptr, m->feat[j]), plan, s));
  }
  // fusion, coarse to fine (depth_anything._fuse)
  const Map* hidden = nullptr;
  for (int j = 0; j < 4; ++j) {
    const std::string Fj = "F" + std::to_string(j) + ".";
    const Map& feat = m->feat[3 - j];
    auto& fu = m->fuse[j];
    const Map* h = &feat;
    if (hidden) {
      TRY(gemm(m, conv_desc(feat, W(Fj + "r1c1.w"), Wf(Fj + "r1c1.b"), F, 3, 1, 1, true, 2, nullptr, nullptr, fu.t),
               plan, s));
      TRY(gemm(m, conv_desc(fu.t, W(Fj + "r1c2.w"), Wf(Fj + "r1c2.b"), F, 3, 1, 1, false, 0, feat.p, hidden->p, fu.h),
               plan, s));
      h = &fu.h;
    }
    TRY(gemm(m, conv_desc(*h, W(Fj + "r2c1.w"), Wf(Fj + "r2c1.b"), F, 3, 1, 1, true, 2, nullptr, nullptr, fu.t2),
             plan, s));
    TRY(gemm(m, conv_desc(fu.t2, W(Fj + "r2c2.w"), Wf(Fj + "r2c2.b"), F, 3, 1, 1, false, 0, h->p, nullptr, fu.h2),
             plan, s));
    i2pc_gemm_desc d = desc0();                            // 1x1 projection, then the resize
    d.a = fu.h2.p; d.lda = F; d.m = fu.h2.b * fu.h2.h * fu.h2.w; d.n = F; d.k = F;
    d.w = W(Fj + "w_proj"); d.ldw = F; d.bias = Wf(Fj + "b_proj");
    d.c = fu.p.p; d.ldc = F;
    TRY(gemm(m, d, plan, s));
    if (!plan)
      TRY(i2pc_resize_bilinear(fu.p.p, fu.p.b, fu.p.h, fu.p.w, F, fu.up.h, fu.up.w, 1, nullptr, fu.up.p, s));
    hidden = &fu.up;
  }
  // head: conv1, then the fused resize + conv2 + ReLU + conv3 + ReLU
  TRY(gemm(m, conv_desc(*hidden, W("H.w1"), Wf("H.b1"), I[I_H1P], 3, 1, 1, false, 0, nullptr, nullptr, m->head_t), plan,
           s));
  if (!plan)
    TRY(i2pc_head_upconv(m->head_t.p, B, m->head_t.h, m->head_t.w, m->head_t.c, (I[I_FUSION] / 2 + 31) / 32 * 32,
                         gh * I[I_PATCH], gw * I[I_PATCH],
                         W("H.w2"), Wf("H.b2"), Wf("H.w3"), m->floats[F_B_H3], depth, s));
  return I2PC_OK;
}

// Every tensor forward_da reads, with the dtype (0 fp32, 1 bf16) and element count the header's
// dimensions imply (model_file.py _tensors): a file whose table disagrees is rejected before any
// upload, so a truncated or mismatched file cannot reach a kernel.
struct Want { std::string name; int dtype; int64_t elems; };
static int expected_tensors(const int32_t* I, std::vector<Want>& want) {
  const int64_t D = I[I_HIDDEN], L = I[I_LAYERS], mlp = I[I_MLP], F = I[I_FUSION], h1p = I[I_H1P], kp = I[I_PITCH];
  const int64_t np_ = (int64_t)I[I_GH] * I[I_GW];
  want = {{"pe.w", 1, D * kp}, {"pe.b", 0, D}, {"cls", 0, D}, {"pos0", 0, D}, {"pos.table", 0, np_ * D}};
  for (int i = 0; i < L; ++i) {
    const std::string p = "L" + std::to_string(i) + ".";
    want.insert(want.end(), {{p + "ln1_g", 0, D}, {p + "ln1_b", 0, D}, {p + "w_qkv", 1, 3 * D * D}, {p + "b_qkv", 0, 3 * D},
                             {p + "w_qkv_f", 1, 3 * D * D}, {p + "b_qkv_f", 0, 3 * D}, {p + "s_qkv", 0, 3 * D},
                             {p + "w_o", 1, D * D}, {p + "b_o", 0, D}, {p + "w_1_f", 1, mlp * D}, {p + "b_1_f", 0, mlp},
                             {p + "s_1", 0, mlp}, {p + "w_2", 1, D * mlp}, {p + "b_2", 0, D}});
  }
  want.insert(want.end(), {{"ln_g", 0, D}, {"ln_b", 0, D}});
  for (int j = 0; j < 4; ++j) {
    const std::string p = "S" + std::to_string(j) + ".";
    const int64_t c = I[I_NECK0 + j], fac = I[I_FAC0 + j];
    want.insert(want.end(), {{p + "w_proj", 1, c * D}, {p + "b_proj", 0, c}, {p + "w_neck", 1, F * 9 * c}});
    if (fac > 1) want.insert(want.end(), {{p + "w_rs", 1, fac * fac * c * c}, {p + "b_rs", 0, fac * fac * c}});
    if (fac < 0) want.insert(want.end(), {{p + "w_rs", 1, c * 9 * c}, {p + "b_rs", 0, c}});
  }
  for (int j = 0; j < 4; ++j) {
    const std::string p = "F" + std::to_string(j) + ".";
    want.insert(want.end(), {{p + "w_proj", 1, F * F}, {p + "b_proj", 0, F}});
    for (const char* rc : {"r1c1", "r1c2", "r2c1", "r2c2"})
      want.insert(want.end(), {{p + rc + ".w", 1, F * 9 * F}, {p + rc + ".b", 0, F}});
  }
  want.insert(want.end(), {{"H.w1", 1, h1p * 9 * F}, {"H.b1", 0, h1p}, {"H.w2", 1, 32 * 9 * h1p}, {"H.b2", 0, 32},
                           {"H.w3", 0, 32}});
  return I2PC_OK;
}

static int validate(const int32_t* I, const std::vector<Entry>& tab) {
  // out_indices: four distinct layers, each of which the encoder loop meets once (else hs[] would
  // be left unwritten and the neck would read uninitialised hidden states)
  for (int k = 0; k < 4; ++k) {
    if (I[I_OUT0 + k] < 1 || I[I_OUT0 + k] > I[I_LAYERS])
      return set_error(I2PC_EINVAL, "model: out index %d = %d outside 1..%d", k, I[I_OUT0 + k], I[I_LAYERS]);
    for (int q = 0; q < k; ++q)
      if (I[I_OUT0 + q] == I[I_OUT0 + k]) return set_error(I2PC_EINVAL, "model: out indices repeat layer %d", I[I_OUT0 + k]);
  }
  for (int j = 0; j < 4; ++j)
    if (I[I_NECK0 + j] <= 0 || I[I_FAC0 + j] == 0 || I[I_FAC0 + j] > 16 || I[I_FAC0 + j] < -16)
      return set_error(I2PC_EINVAL, "model: reassemble stage %d (channels %d, factor %d)", j, I[I_NECK0 + j], I[I_FAC0 + j]);
  if (I[I_GH] <= 0 || I[I_GW] <= 0 || I[I_PITCH] < 3 * I[I_PATCH] * I[I_PATCH] || I[I_H1P] <= 0 || I[I_FUSION] <= 0 ||
      I[I_MLP] <= 0 || I[I_HIDDEN] <= 0 || I[I_LAYERS] <= 0 || I[I_LAYERS] > 1024 || I[I_PATCH] <= 0)
    return set_error(I2PC_EINVAL, "model: header dimensions out of range");
  std::map<std::string, const Entry*> by;
  for (const Entry& e : tab) by[std::string(e.name)] = &e;
  std::vector<Want> want;
  TRY(expected_tensors(I, want));
  for (const Want& w : want) {
    auto it = by.find(w.name);
    if (it == by.end()) return set_error(I2PC_EINVAL, "model: tensor %s missing", w.name.c_str());
    const Entry& e = *it->second;
    const int64_t esz = w.dtype ? 2 : 4;
    int64_t dims = 1;
    for (int k = 0; k < 4; ++k) dims *= k < e.ndim ? e.dims[k] : 1;
    if (e.dtype != w.dtype || e.ndim < 1 || e.ndim > 4 || e.nbytes != w.elems * esz || dims != w.elems)
      return set_error(I2PC_EINVAL, "model: tensor %s is %s x %lld elements (%lld bytes), the header implies %s x %lld",
                       w.name.c_str(), e.dtype == 1 ? "bf16" : e.dtype == 0 ? "fp32" : "?", (long long)dims,
                       (long long)e.nbytes, w.dtype ? "bf16" : "fp32", (long long)w.elems);
  }
  return I2PC_OK;
}

static int read_file(const char* path, std::vector<char>& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return set_error(I2PC_EINVAL, "model: cannot open %s", path);
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  buf.resize(n > 0 ? (size_t)n : 0);
  const size_t got = n > 0 ? std::fread(buf.data(), 1, (size_t)n, f) : 0;
  std::fclose(f);
  if (n <= 0 || got != (size_t)n) return set_error(I2PC_EINVAL, "model: cannot read %s", path);
  return I2PC_OK;
}

// the header and tensor table, checked against the file size
static int parse(const std::vector<char>& buf, int32_t* ints, float* floats, std::vector<Entry>& tab, size_t& data0) {
  const size_t hdr = 8 + 32 * 4 + 16 * 4;
  if (buf.size() < hdr || std::memcmp(buf.data(), kMagic, 8) != 0)
    return set_error(I2PC_EINVAL, "model: not an i2pc network file");
  std::memcpy(ints, buf.data() + 8, 32 * 4);
  std::memcpy(floats, buf.data() + 8 + 128, 16 * 4);
  // version 2: the Q rows of every QKV weight / bias carry the softmax scale * log2(e) (attention_q2)
  if (ints[I_VERSION] != 2) return set_error(I2PC_EUNSUPPORTED, "model: file version %d (this library reads 2)", ints[I_VERSION]);
  const int nt = ints[I_NTENSORS];
  if (nt <= 0 || nt > 100000 || buf.size() < hdr + (size_t)nt * sizeof(Entry))
    return set_error(I2PC_EINVAL, "model: bad tensor table");
  tab.resize(nt);
  std::memcpy(tab.data(), buf.data() + hdr, (size_t)nt * sizeof(Entry));
  data0 = hdr + (size_t)nt * sizeof(Entry);
  for (const Entry& e : tab) {
    if (e.name[47] != 0 || e.offset < 0 || e.nbytes < 0 || data0 + (size_t)e.offset + (size_t)e.nbytes > buf.size() ||
        e.offset % 256 != 0)
      return set_error(I2PC_EINVAL, "model: tensor %.47s out of the file", e.name);
  }
  return I2PC_OK;
}

}  // namespace model
}  // namespace i2pc

using namespace i2pc;
using namespace i2pc::model;

extern "C" int i2pc_model_file_info(const char* path, int32_t* ints32, float* floats16, int* ntensors) {
  clear_error();
  I2PC_REQUIRE(path && ints32 && floats16 && ntensors, "NULL pointer");
  std::vector<char> buf;
  TRY(read_file(path, buf));
  std::vector<Entry> tab;
  size_t data0 = 0;
  TRY(parse(buf, ints32, floats16, tab, data0));
  if (ints32[I_FAMILY] == kFamilyDepthAnything) TRY(validate(ints32, tab));
  *ntensors = (int)tab.size();
  return I2PC_OK;
}

static void destroy_impl(i2pc_model* m) {   // (keeps the thread's error message)
  if (!m) return;
  for (void* p : m->bufs) (void)hipFree(p);
  if (m->arena) (void)hipFree(m->arena);
  if (m->plan) i2pc_preprocess_plan_destroy(m->plan);
  delete m;
}

extern "C" int i2pc_model_destroy(i2pc_model* m) {
  clear_error();
  destroy_impl(m);
  return I2PC_OK;
}

extern "C" int i2pc_model_create(const char* path, int batch, int in_h, int in_w, i2pc_model** out) {
  clear_error();
  I2PC_REQUIRE(path && out, "NULL pointer");
  I2PC_REQUIRE(batch >= 1 && batch <= 4096, "model: batch %d", batch);
  *out = nullptr;
  std::vector<char> buf;
  TRY(read_file(path, buf));
  auto* m = new i2pc_model();
  std::vector<Entry> tab;
  size_t data0 = 0;
  int rc = parse(buf, m->ints, m->floats, tab, data0);
  const int* I = m->ints;
  auto bail = [&](int code) { destroy_impl(m); return code; };
  if (rc != I2PC_OK) return bail(rc);
  if (I[I_FAMILY] != kFamilyDepthAnything)
    return bail(set_error(I2PC_EUNSUPPORTED, "model: family %d (1 = Depth-Anything is the one the executor runs)", I[I_FAMILY]));
  if (I[I_IN_H] != in_h || I[I_IN_W] != in_w)
    return bail(set_error(I2PC_EINVAL, "model: the file is made for %dx%d input images, not %dx%d", I[I_IN_H], I[I_IN_W],
                          in_h, in_w));
  if ((rc = validate(I, tab)) != I2PC_OK) return bail(rc);
  const int D = I[I_HIDDEN], gh = I[I_GH], gw = I[I_GW], np_ = gh * gw, T = np_ + 1, F = I[I_FUSION];
  if (D <= 0 || D % 64 || I[I_MLP] % 64 || I[I_HEADS] * 64 != D || gh <= 0 || gw <= 0 || F % 64 || I[I_H1P] % 64 ||
      I[I_PITCH] % 64 || I[I_LAYERS] <= 0 || I[I_HEAD_HIDDEN] != 32 || D % kLnChunk)
    return bail(set_error(I2PC_EUNSUPPORTED, "model: configuration outside what the executor runs"));
  m->batch = batch;
  // weights: one arena, every tensor at its 256-byte file offset
  size_t total = 0;
  for (const Entry& e : tab) total = std::max(total, (size_t)(e.offset + e.nbytes));
  if (hipMalloc(&m->arena, std::max<size_t>(total, 256)) != hipSuccess)
    return bail(set_error(I2PC_ELAUNCH, "model: hipMalloc of %zu weight bytes failed", total));
  if (hipMemcpy(m->arena, buf.data() + data0, total, hipMemcpyHostToDevice) != hipSuccess)
    return bail(set_error(I2PC_ELAUNCH, "model: weight upload failed"));
  for (const Entry& e : tab) m->w[std::string(e.name)] = static_cast<char*>(m->arena) + e.offset;
  // preprocessing plan (Pillow-exact bicubic; bf16 patch rows)
  const float mean[3] = {m->floats[F_MEAN0], m->floats[F_MEAN0 + 1], m->floats[F_MEAN0 + 2]};
  const float stdv[3] = {m->floats[F_STD0], m->floats[F_STD0 + 1], m->floats[F_STD0 + 2]};
  if ((rc = i2pc_preprocess_plan_create(in_h, in_w, I[I_OUT_H], I[I_OUT_W], mean, stdv, I[I_PATCH], &m->plan)) != I2PC_OK)
    return bail(rc);
  // activations (depth_anything.buffers + the per-call maps of forward)
  const int64_t M = (int64_t)batch * T;
  const size_t prow = (size_t)batch * np_ * I[I_PITCH] * 2;
  m->patches = dalloc(m, prow);
  m->x = dalloc(m, M * D * 4);
  m->ln = dalloc(m, M * D * 2);
  m->qkv = dalloc(m, M * 3 * D * 2);
  m->att = dalloc(m, M * D * 2);
  m->mlp = dalloc(m, M * I[I_MLP] * 2);
  m->part = dalloc(m, M * (D / kLnChunk) * 8);
  m->rs = dalloc(m, M * 8);
  m->sh0 = dalloc(m, M * 4);
  m->sh1 = dalloc(m, M * 4);
  for (int k = 0; k < 4; ++k) m->hs[k] = dalloc(m, M * D * 2);
  bool ok = m->patches && m->x && m->ln && m->qkv && m->att && m->mlp && m->part && m->rs && m->sh0 && m->sh1 &&
            m->hs[0] && m->hs[1] && m->hs[2] && m->hs[3];
  // the pad columns of the patch rows stay zero (the preprocessing kernel writes 3*p*p of them)
  if (ok && hipMemset(m->patches, 0, prow) != hipSuccess) ok = false;
  int sizes[4][2];
  for (int j = 0; j < 4 && ok; ++j) {
    const int c = I[I_NECK0 + j], fac = I[I_FAC0 + j];
    if (c % 64 || fac == 0) return bail(set_error(I2PC_EUNSUPPORTED, "model: reassemble stage %d", j));
    ok = alloc_map(m, m->proj[j], batch, gh, gw, c);
    int h = gh, w = gw;
    if (fac > 1) { h = gh * fac; w = gw * fac; }
    if (fac < 0) { h = (gh + 2 - 3) / -fac + 1; w = (gw + 2 - 3) / -fac + 1; }
    if (fac != 1) ok = ok && alloc_map(m, m->rsz[j], batch, h, w, c);
    ok = ok && alloc_map(m, m->feat[j], batch, h, w, F);
    sizes[j][0] = h;
    sizes[j][1] = w;
  }
  for (int j = 0; j < 4 && ok; ++j) {
    const Map& feat = m->feat[3 - j];
    auto& fu = m->fuse[j];
    if (j > 0) {
      const Map& prev = m->fuse[j - 1].up;
      if (prev.h != feat.h || prev.w != feat.w)     // depth_anything._fuse's resize branch: not reached here
        return bail(set_error(I2PC_EUNSUPPORTED, "model: fusion stage %d shapes differ", j));
      ok = alloc_map(m, fu.t, batch, feat.h, feat.w, F) && alloc_map(m, fu.h, batch, feat.h, feat.w, F);
    }
    ok = ok && alloc_map(m, fu.t2, batch, feat.h, feat.w, F) && alloc_map(m, fu.h2, batch, feat.h, feat.w, F) &&
         alloc_map(m, fu.p, batch, feat.h, feat.w, F);
    const int uh = j + 1 < 4 ? sizes[3 - (j + 1)][0] : 2 * feat.h, uw = j + 1 < 4 ? sizes[3 - (j + 1)][1] : 2 * feat.w;
    ok = ok && alloc_map(m, fu.up, batch, uh, uw, F);
  }
  ok = ok && alloc_map(m, m->head_t, batch, m->fuse[3].up.h, m->fuse[3].up.w, I[I_H1P]);
  if (!ok) return bail(set_error(I2PC_ELAUNCH, "model: activation allocation failed"));
  // (every tensor the forward reads was checked by validate() above: name, dtype, byte count)
  // plan pass: the largest split-K workspace any call of the forward asks for
  if ((rc = forward_da(m, nullptr, nullptr, true, nullptr)) != I2PC_OK) return bail(rc);
  if (m->ws_bytes && !(m->ws = dalloc(m, m->ws_bytes))) return bail(set_error(I2PC_ELAUNCH, "model: workspace allocation failed"));
  *out = m;
  return I2PC_OK;
}

extern "C" int i2pc_model_io(const i2pc_model* m, int* batch, int* in_h, int* in_w, int* depth_h, int* depth_w) {
  clear_error();
  I2PC_REQUIRE(m, "NULL model");
  if (batch) *batch = m->batch;
  if (in_h) *in_h = m->ints[I_IN_H];
  if (in_w) *in_w = m->ints[I_IN_W];
  if (depth_h) *depth_h = m->ints[I_GH] * m->ints[I_PATCH];
  if (depth_w) *depth_w = m->ints[I_GW] * m->ints[I_PATCH];
  return I2PC_OK;
}

extern "C" int i2pc_depth_forward(i2pc_model* m, const uint8_t* bgr, float* depth, void* stream) {
  clear_error();
  I2PC_REQUIRE(m && bgr && depth, "NULL pointer");
  return forward_da(m, bgr, depth, false, as_stream(stream));
}

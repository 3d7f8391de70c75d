/*
 * i2pc.h -- C ABI of the MI355X-native image -> point-cloud hot path.
 *
 * The reference (Samsonboadi/Image_to_pointCloud @ 2025-09-05) has no native
 * code and no FFI: its hot path is the in-process Python calls
 *
 *   process_with_depth_anything(image, model_info) -> depth   backend/app.py:99-122
 *   depth_to_point_cloud(image, depth, density, invert,
 *                        depth_scale, smooth, smooth_ksize, fov)  backend/app.py:174-250
 *   generate_gis_metadata(points, request)["bounds"]            backend/app.py:391-400
 *
 * Every entry point below is what a binding for those calls needs (see
 * INTEGRATION.md for the ctypes stub a maintainer would add to app.py).
 * Conventions (all entry points):
 *   - all array pointers are DEVICE pointers (hipMalloc / torch CUDA tensors);
 *     inputs are never modified; outputs are caller-owned;
 *   - work is enqueued on `stream` (a hipStream_t; NULL = default stream) and
 *     is stream-ordered: no host synchronisation, no allocation, so every call
 *     can be captured into a hipGraph;
 *   - return 0 on success, a negative I2PC_E* code otherwise; the message of
 *     the last error on the calling thread is in i2pc_last_error();
 *   - re-entrant; one call may run per stream concurrently (kernel-selection knobs are
 *     per host thread, see i2pc_set_tuning).
 * No torch, no C++ types cross this boundary.
 */
#ifndef I2PC_H_
#define I2PC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define I2PC_OK 0
#define I2PC_EINVAL (-1)       /* bad argument (shape, pointer, enum) */
#define I2PC_EWORKSPACE (-2)   /* workspace too small */
#define I2PC_ELAUNCH (-3)      /* HIP launch error */
#define I2PC_EUNSUPPORTED (-4) /* shape/config the kernels do not cover */

/* Version of this ABI. */
int i2pc_abi_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* i2pc_last_error(void);

/* ------------------------------------------------------------------------
 * Unprojection: replaces depth_to_point_cloud (backend/app.py:174-250) plus the
 * bounds of generate_gis_metadata (backend/app.py:393-400), batched.
 * ------------------------------------------------------------------------ */
typedef struct i2pc_unproject_params {
  int32_t step;        /* density step: 4 low, 2 medium, 1 high (app.py:226) */
  int32_t invert;      /* invert_depth (app.py:205-206) */
  double depth_scale;  /* depth_scale (app.py:233) */
  double fov_deg;      /* fov; <= 0 or NaN selects f = 1.2*max(W,H) (app.py:219-223) */
  int32_t smooth;      /* smooth_depth (app.py:209-214) */
  int32_t smooth_ksize;/* GaussianBlur kernel: ksize//2*2+1, at least 3, at most 63 taps (app.py:211) */
  int32_t projection;  /* 0 pinhole (app.py:216-238); 1 equirectangular panorama (not in the
                          reference): depth = range along the ray of longitude (u+0.5)2pi/W - pi,
                          latitude pi/2 - (v+0.5)pi/H; x right, y down, z forward; fov ignored */
  int32_t reserved;    /* 0 */
} i2pc_unproject_params;

/* Bytes of device workspace i2pc_unproject needs. */
size_t i2pc_unproject_workspace_bytes(int batch, int img_h, int img_w, int smooth);

/*
 * depth  : float32 [batch, dep_h, dep_w]   model-resolution relative depth
 *          (resized to img_h x img_w with cv2 INTER_LINEAR semantics when the
 *          sizes differ -- app.py:186-188; never materialised at full res)
 * image  : uint8   [batch, img_h, img_w, channels]  BGR (cv2.imdecode order);
 *          channels >= 3 -> colour gathered as RGB, else grey 128 (app.py:240-244)
 * xyz    : float32 [batch, N, 3]   N = ceil(img_h/step) * ceil(img_w/step),
 *          point i <-> pixel (v,u) = ((i / ceil(W/step))*step, (i % ceil(W/step))*step)
 * rgb    : uint8   [batch, N, 3]   (the reference returns these as float32)
 * bbox   : float64 [batch, 6]      minX maxX minY maxY minZ maxZ of xyz
 * stats  : float64 [batch, 4]      p2, p98 (after the min/max fallback),
 *                                  branch (0 fp64 / 1 fp32 fallback / 2 constant),
 *                                  nanmedian fill value (NaN if none was needed)
 * Any of bbox/stats may be NULL.
 */
int i2pc_unproject(const float* depth, int dep_h, int dep_w,
                   const uint8_t* image, int channels,
                   int batch, int img_h, int img_w,
                   const i2pc_unproject_params* params,
                   float* xyz, uint8_t* rgb, double* bbox, double* stats,
                   void* workspace, size_t workspace_bytes, void* stream);

/* Tile-parallel unprojection of ONE image split into row bands across ranks (SURVEY
 * §8e, config C4: an 8192 x 4096 panorama across 8 GPUs).  Each rank calls this for its
 * band [row0, row1) of the image rows with the full model-resolution depth; the exact
 * global p2/p98 (and nanmedian) need the histograms of every band, so between each
 * selection sweep and its resolve the call hands its partial histograms to `exchange`,
 * which must all-reduce them in place across the ranks (ordered on `stream`):
 *   hist     : uint32 [hist_words] -> element-wise SUM over ranks
 *   counters : int64 [4][batch] or NULL -> rows 0-1 SUM, row 2 MIN, row 3 MAX
 *              (row 0 = NaN count | -Inf count << 32, row 1 = non-finite count,
 *               rows 2-3 = finite key range; passed at level 0 only)
 * and return 0 (non-zero aborts the call).  Every rank must make the same sequence of
 * calls (4 per image, one per selection level; band runs take the histogram levels).
 * image_band : uint8 [row1 - row0, img_w, channels]   the band's rows of the image
 * xyz_band   : float32 [Nb, 3], rgb_band uint8 [Nb, 3] with Nb = (ceil(row1/step) -
 *              row0/step) * ceil(img_w/step): the band's points, row-major, i.e. the
 *              slice [row0/step * ceil(img_w/step), ...) of the whole image's points
 * bbox       : float64 [6] of this band's points (the caller min/max-reduces them)
 * stats      : float64 [4] as i2pc_unproject (identical on every rank)
 * row0 must be a multiple of step, and row1 too unless row1 == img_h.  smooth: each rank
 * recomputes its band's normalised field plus the blur's k/2 halo rows (reflect-101 at the
 * image edges) from the whole model-resolution depth, so smoothed bands concatenate to the
 * whole image's smoothed points with no extra exchange.  workspace:
 * i2pc_unproject_workspace_bytes(1, img_h, img_w, smooth). */
typedef int (*i2pc_exchange_fn)(void* user, uint32_t* hist, int64_t hist_words, int64_t* counters, int batch,
                                void* stream);
int i2pc_unproject_band(const float* depth, int dep_h, int dep_w, const uint8_t* image_band, int channels,
                        int img_h, int img_w, int row0, int row1, const i2pc_unproject_params* params,
                        float* xyz_band, uint8_t* rgb_band, double* bbox, double* stats,
                        void* workspace, size_t workspace_bytes, i2pc_exchange_fn exchange, void* user,
                        void* stream);

/* Window-selection band mode: the same band call with ONE selection sweep instead of four.
 * Every rank derives the same value windows around p2 / p98 (and the median) from a sample of
 * the whole image, sweeps its band once (compacting its window keys locally), then
 *   exchange(user, hist, 6144, counters, 8, stream)  hist: 2048 fine bins per window of the
 *                                                band's window keys (SUM); counters int64 [4][8]:
 *                                                rows 0-1 SUM, row 2 MIN, row 3 MAX
 *   gather(user, send, recv, words, stream)      all-gather: every rank's `words` uint32 into
 *                                                recv [nranks][words] (any fixed rank order):
 *                                                per target the band's keys of its fine bin
 * and every rank selects the same exact keys (about 25 KB all-reduced + 41 KB gathered per
 * rank, whatever the image size).  A target the windows missed, or a fine bin holding more than
 * 1024 distinct-valued keys in one band, falls back to an exact whole-image selection on every
 * rank (same result, much slower).  workspace: i2pc_unproject_band_workspace_bytes(img_h, img_w,
 * smooth, nranks). */
typedef int (*i2pc_gather_fn)(void* user, const uint32_t* send, uint32_t* recv, int64_t words, void* stream);
size_t i2pc_unproject_band_workspace_bytes(int img_h, int img_w, int smooth, int nranks);
int i2pc_unproject_band_w(const float* depth, int dep_h, int dep_w, const uint8_t* image_band, int channels,
                          int img_h, int img_w, int row0, int row1, const i2pc_unproject_params* params,
                          float* xyz_band, uint8_t* rgb_band, double* bbox, double* stats,
                          void* workspace, size_t workspace_bytes, int nranks, i2pc_exchange_fn exchange,
                          i2pc_gather_fn gather, void* user, void* stream);

/* The window-selection band call with the exchange done on the device by RCCL (the counters'
 * all-reduces and the candidates' all-gather on `stream`), so the call is stream-ordered end to
 * end and can be captured into a HIP graph; workspace: i2pc_unproject_band_workspace_bytes(
 * img_h, img_w, smooth, nranks of the communicator).  `comm` comes from
 * i2pc_comm_create on every rank with the id rank 0 got from i2pc_comm_unique_id
 * (ncclGetUniqueId / ncclCommInitRank; 128 bytes, shipped by the caller); the current HIP
 * device must be the rank's GPU. */
typedef struct i2pc_comm i2pc_comm;
int i2pc_comm_unique_id(void* out, int nbytes);
int i2pc_comm_create(const void* unique_id, int nranks, int rank, i2pc_comm** comm);
void i2pc_comm_destroy(i2pc_comm* comm);
int i2pc_unproject_band_rccl(const float* depth, int dep_h, int dep_w, const uint8_t* image_band, int channels,
                             int img_h, int img_w, int row0, int row1, const i2pc_unproject_params* params,
                             float* xyz_band, uint8_t* rgb_band, double* bbox, double* stats, void* workspace,
                             size_t workspace_bytes, i2pc_comm* comm, void* stream);

/* Depth preview image (create_depth_preview, backend/app.py:124-172) for a batch of
 * model-resolution depth maps, before any resize: nanmedian fill, exact p2/p98 of
 * the map itself, clip/normalise/invert exactly as i2pc_unproject, then
 * (d*255).astype(uint8) and a colour table.
 * depth   : float32 [batch, h, w]
 * lut_bgr : uint8 [256][3] device colour table in B,G,R order (cv2.COLORMAP_PLASMA)
 * out_bgr : uint8 [batch, h, w, 3]   (what cv2.imencode('.png') receives)
 * stats   : float64 [batch, 4] as in i2pc_unproject, or NULL
 * workspace: i2pc_unproject_workspace_bytes(batch, h, w, 0) bytes. */
int i2pc_depth_preview(const float* depth, int batch, int h, int w, int invert, const uint8_t* lut_bgr,
                       uint8_t* out_bgr, double* stats, void* workspace, size_t workspace_bytes, void* stream);

/* Profiling hook (bench.py's roofline): while enabled, i2pc_unproject records two HIP
 * events on its stream around the unprojection kernel (the HBM-bound back-projection +
 * RGB gather + bbox launch, when the fast layout applies), and
 * i2pc_profile_unproject_ms() returns that kernel's duration of the last such call
 * (synchronising on the stop event), or -1 if none was recorded. Not thread-safe. */
int i2pc_profile_enable(int on);
float i2pc_profile_unproject_ms(void);

/* Measurement aid (no reference counterpart; bench.py's clock_ghz_run): `workgroups` 256-thread
 * workgroups (one per CU: 256) run `iters` x 4 dense bf16 32x32x16 MFMAs on random operands; for
 * workgroup g, out[2g] = shader-clock ticks (s_memtime) and out[2g + 1] = 100 MHz ticks
 * (s_memrealtime) of the chain, so the clock held under MFMA load is out[2g] / out[2g + 1] * 0.1 GHz.
 * out: device buffer of 2 * workgroups u64. */
int i2pc_clock_probe(int workgroups, int iters, unsigned long long* out, void* stream);

/* Gather every stride-th point (preview subsample, app.py:496-506):
 * out_xyz/out_rgb [count] with count = ceil(n / stride). */
int i2pc_gather_stride(const float* xyz, const uint8_t* rgb, int64_t n, int64_t stride,
                       float* out_xyz, float* out_rgb, void* stream);

/* Statistical outlier removal of one cloud: replaces refine_point_cloud
 * (backend/app.py:252-269), i.e. Open3D PointCloud::RemoveStatisticalOutliers
 * (nb_neighbors, std_ratio) of open3d>=0.17.0 (backend/requirements.txt:14):
 * avg[i] = mean distance to the min(nb_neighbors, n) nearest points (itself included,
 * float64), keep i iff 0 < avg[i] < mean + std_ratio * std (Bessel), ascending order.
 * Exact kNN on a device-sized uniform grid; stream-ordered, no host synchronisation.
 * xyz       : float32 [n, 3] (finite; a non-finite cloud keeps nothing)
 * rgb       : uint8 [n, 3] or NULL       out_rgb  : uint8 [n, 3] or NULL (needs rgb)
 * out_xyz   : float32 [n, 3] or NULL     out_index: int64 [n] or NULL (Open3D's `ind`)
 *             (the first *count rows of the outputs are the kept points, in index order)
 * count     : int64 [1] number kept      bbox     : float64 [6] of the kept points or NULL
 * avg_dist  : float64 [n] per-point mean neighbour distance, or NULL
 * nb_neighbors in [1, 32], std_ratio > 0 (Open3D rejects the rest);
 * workspace : i2pc_sor_workspace_bytes(n) bytes. */
size_t i2pc_sor_workspace_bytes(int64_t n);
int i2pc_sor(const float* xyz, const uint8_t* rgb, int64_t n, int nb_neighbors, double std_ratio,
             float* out_xyz, uint8_t* out_rgb, int64_t* out_index, int64_t* count, double* bbox,
             double* avg_dist, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Depth network building blocks (replace the PyTorch CPU conv / linear / SDPA /
 * LayerNorm arithmetic that process_with_depth_anything reaches through
 * transformers, backend/app.py:109-113).  bf16 operands, fp32 accumulation.
 * ------------------------------------------------------------------------ */

/* out[m][n] = epilogue( sum_k A[m][k] * W[n][k] ) on the MFMA cores.
 * A: bf16 rows (dense, row r(m) = (m / a_group)*a_group_stride + m % a_group + a_offset,
 *    a_group = 0 means r(m) = m + a_offset), or with conv = 1 the implicit im2col of an
 *    NHWC bf16 image [conv_batch, conv_h, conv_w, conv_c] for a conv_k x conv_k
 *    convolution (k order = (ky, kx, ci)), stride conv_stride, zero padding conv_pad,
 *    optional ReLU applied to the input (conv_relu_in; pre-activation residual units).
 * W: bf16 [n][k], row stride ldw.
 * Epilogue in fp32, in this order: + bias[n]; + row_bias[m / row_bias_group][n];
 *    + table[m % table_rows][n]; act (0 none, 1 GELU-erf, 2 ReLU); + res (fp32 or bf16,
 *    same indexing as the output); + res2 (bf16); store bf16 (c_f32 = 0) or fp32.
 * Output row o(m) = (m / out_group)*out_group_stride + m % out_group + out_offset
 *    (row stride ldc), or, with convt_s > 0, the ConvTranspose(kernel = stride = s)
 *    pixel shuffle: m = (b, iy, ix) over convt_h x convt_w, n = (dy*s + dx)*convt_c + co
 *    -> NHWC [b][iy*s+dy][ix*s+dx][co].
 * Requires k % 64 == 0, n % 32 == 0, conv_c % 64 == 0.  Other widths: zero-pad K (A's columns
 * and W's, or a conv's input channels) to a multiple of 64 and N (W's rows, bias, residuals) to a
 * multiple of 32, call on the padded shapes and keep the first n columns -- what the Python layer
 * (ops.linear / ops.conv2d) does for such checkpoints. */
typedef struct i2pc_gemm_desc {
  const void* a; int64_t lda; int32_t m, n, k;
  int32_t a_group, a_group_stride, a_offset;
  int32_t conv, conv_batch, conv_h, conv_w, conv_c, conv_oh, conv_ow, conv_k, conv_stride, conv_pad, conv_relu_in;
  const void* w; int64_t ldw;
  const float* bias;
  const float* row_bias; int32_t row_bias_group;
  const float* table; int32_t table_rows;
  int32_t act;
  const void* res; int32_t res_f32; int64_t ldr;
  const void* res2; int64_t ldr2;
  void* c; int32_t c_f32; int64_t ldc;
  int32_t out_group, out_group_stride, out_offset;
  int32_t convt_s, convt_h, convt_w, convt_c;
  /* LayerNorm folded through the GEMM (nn.LayerNorm before a linear layer, modeling_dpt.py:233-234,
   * 376-381; NULL = off).
   * Producer (fp32 output rows, e.g. the residual-add epilogue of attention-out / FC2): with
   *   ln_part set it also writes c_bf16 [m][ldc_bf16] = bf16(out) and, per output row and C-column
   *   chunk (C = ln_chunk: 0 or 64 -> 64, or 32), ln_part float2 [m][n / C] = (mean, sum of squared
   *   deviations from it) of that chunk of out.  With ln_shift (fp32 [m], e.g. the row means of the
   *   previous LayerNorm) both are taken of out - ln_shift[row] instead (the bf16 copy then keeps its
   *   precision for rows whose mean is large against their spread).  Needs n % C == 0, c_f32, no row
   *   remap / ConvTranspose store (EUNSUPPORTED where the chosen kernel cannot: i2pc_gemm_kernel_name
   *   says "invalid").  32-column chunks let narrow-tile plans produce (e.g. n = 384 on 384 x 192
   *   tiles, whose 96-column wave tiles hold no whole 64-column chunk).
   * Consumer (A = the producer's c_bf16, W = W * gamma[k] in bf16): with ln_rows set the epilogue
   *   computes act(rs.x * acc + rs.y * col_sum[n] + bias[n]) with rs = ln_rows float2 [m] =
   *   (rstd, -rstd * mean) (i2pc_ln_rowstats), col_sum fp32 [n] = sum_k of W's bf16 row, bias =
   *   b + W beta: the LayerNorm of A's rows applied after the product.  Dense A, bf16 output, no
   *   residuals / row bias / table (the persistent engine runs it).
   * bf16 residual stream (a producer with c_f32 = 0; c_bf16 NULL or == c): the output C itself is
   *   bf16(out - ln_shift[row]) -- the shifted residual stream the next consumer reads as A and the
   *   next producer reads as res -- and no fp32 copy is written.  A bf16 res is then taken as
   *   res[row][n] + res_shift[row] when res_shift (fp32 [m]) is set: the shift it was stored
   *   relative to (may differ from ln_shift, which tracks the latest LayerNorm mean).  The torch-bf16
   *   forward keeps its residual stream in bf16 too; the shift keeps each row's rounding at its
   *   spread rather than its mean. */
  const float* ln_rows; const float* col_sum;
  float* ln_part; void* c_bf16; int64_t ldc_bf16;
  const float* ln_shift;
  int32_t ln_chunk;
  const float* res_shift;
} i2pc_gemm_desc;

/* LayerNorm row statistics from i2pc_gemm's producer partials: rows_out float2 [rows] =
 * (rstd, -rstd * mean) of each row's `parts` 64-column chunks (part float2 [rows][parts]), the
 * chunks combined by Chan's formula; biased variance, rstd = 1 / sqrt(var + eps) (nn.LayerNorm).
 * shift_in (fp32 [rows] or NULL = 0): the producer's ln_shift -- the partials were taken of
 * out - shift_in, so `mean` above is the shifted mean; shift_out (or NULL) receives the rows' true
 * means, shift_in + mean (the next producer's shift; may alias shift_in).  parts <= 64. */
int i2pc_ln_rowstats(const float* part, int rows, int parts, float eps, float* rows_out, const float* shift_in,
                     float* shift_out, void* stream);
/* LayerNorm of bf16 rows from their statistics: y[r][c] = bf16(gamma[c] * (rs.x * x[r][c] + rs.y) +
 * beta[c]) with rows_stats float2 [rows] = (rstd, -rstd * mean) from i2pc_ln_rowstats of the producer
 * that wrote x (x may be the shifted bf16 residual stream: the statistics are of the same shifted
 * values).  E.g. Depth-Anything's backbone LayerNorm of a kept hidden state
 * (modeling_dinov2.py: `self.layernorm(hidden_state)` on out_features).  dim, ldx, ldy % 8 == 0. */
int i2pc_ln_apply(const void* x, int64_t ldx, const float* rows_stats, const float* gamma, const float* beta,
                  int rows, int dim, void* y, int64_t ldy, void* stream);
/* The same for chunk_cols-column chunks (32 or 64; i2pc_ln_rowstats = chunk_cols 64). */
int i2pc_ln_rowstats_w(const float* part, int rows, int parts, int chunk_cols, float eps, float* rows_out,
                       const float* shift_in, float* shift_out, void* stream);

int i2pc_gemm(const i2pc_gemm_desc* desc, void* stream);

/* i2pc_gemm with a caller-owned device workspace (16-byte aligned) for split-K: calls the
 * tile kernel would run on at most half the CUs with a long K (e.g. the 12x12 and 24x24 neck
 * convs, K = 9216) are split into K slices whose fp32 partial sums go to the workspace and
 * are then reduced in slice order with the same epilogue.  i2pc_gemm_workspace_bytes(desc)
 * is the size that call uses (0 = no split; a smaller or NULL workspace runs unsplit).
 * Automatic engine modes (0, 3) only; knob "gemm_splitk" (i2pc_set_tuning) turns it off. */
int i2pc_gemm_ws(const i2pc_gemm_desc* desc, void* workspace, size_t workspace_bytes, void* stream);
size_t i2pc_gemm_workspace_bytes(const i2pc_gemm_desc* desc);

/* MX fp8 GEMM / implicit-GEMM convolution (the DPT-Hybrid fp8 path, BASELINE configs[4]):
 * the same contract as i2pc_gemm with A and W in OCP e4m3fn (1 byte per element; lda, ldw
 * and ldc in ELEMENTS = bytes) and one E8M0 scale per 32 consecutive k:
 *   a_scale: uint32 [rows][lda_scale] -- dword kt of row m holds the scales of k-blocks
 *            4 kt .. 4 kt + 3 (byte b = block 4 kt + b), i.e. the bytes [rows][K / 32];
 *            for a conv, rows are input PIXELS (NHWC) and lda_scale = Cin / 128;
 *   w_scale: uint32 [n][ldw_scale], same layout over W's k;
 *   value(m, k) = e4m3(A[m][k]) * 2^(scale byte - 127).
 * Runs on v_mfma_scale_f32_16x16x128_f8f6f4 (fp32 accumulation).  Output: bf16 / fp32 as
 * i2pc_gemm, or (c_fp8 = 1) MX fp8 C [m][ldc] bytes + c_scale uint32 [m][ldc_scale] with
 * each 32-column block scaled so that max |v| / 2^e <= 448 (no saturation), e4m3 round to
 * nearest even.  Requires k % 128 == 0, n % 128 == 0 (256 for dense A / fp8 output),
 * conv_c % 128 == 0; no ConvTranspose store, no A row groups. */
typedef struct i2pc_gemm_fp8_desc {
  i2pc_gemm_desc g;
  const void* a_scale; int64_t lda_scale;
  const void* w_scale; int64_t ldw_scale;
  void* c_scale; int64_t ldc_scale;
  int32_t c_fp8;
} i2pc_gemm_fp8_desc;

int i2pc_gemm_fp8(const i2pc_gemm_fp8_desc* desc, void* stream);
const char* i2pc_gemm_fp8_kernel_name(const i2pc_gemm_fp8_desc* desc);

/* MX fp8 producers (operand format of i2pc_gemm_fp8).  quant_fp8: y[r] = fp8 of x[src(r)]
 * (x bf16 or fp32 [*][ldx], optional ReLU; src(r) = (r / g) * gs + r % g + o, g = 0: r + o --
 * e.g. skip the CLS row of every image); layernorm_fp8: nn.LayerNorm of fp32 rows written as
 * fp8 rows (dim % 256 == 0).  y: bytes [rows][ldy]; y_scale: uint32 [rows][ldy_scale]. */
int i2pc_quant_fp8(const void* x, int x_f32, int64_t ldx, int rows, int k, int relu, int row_group,
                   int row_group_stride, int row_offset, void* y, int64_t ldy, void* y_scale, int64_t ldy_scale,
                   void* stream);
int i2pc_layernorm_fp8(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps, int rows,
                       int dim, void* y, int64_t ldy, void* y_scale, int64_t ldy_scale, void* stream);

/* BiT-ResNet stem of DPT-Hybrid (transformers modeling_bit.py; bf16 NHWC maps).
 * bit_stem_im2col: fp32 NCHW pixel_values -> bf16 GEMM rows [b*out_h*out_w][k_pitch], k =
 *   (ky*ksize + kx)*3 + c (zero past ksize^2*3), input pixel (oy*2 - pad_top + ky, ox*2 -
 *   pad_left + kx), zero outside (DynamicPad2d "SAME", modeling_bit.py:148-196).
 * groupnorm_stats: stats fp32 [batch][groups][2] = (mean, 1 / sqrt(var + eps)), biased variance
 *   (nn.functional.group_norm): per-tile fp32 sums into `workspace`
 *   (>= i2pc_groupnorm_workspace_bytes), combined in fp64.
 * groupnorm_apply: y = relu?(gn(x) + shortcut); gn(x) = (x - mean) * rstd * gamma + beta;
 *   stats NULL = x raw; shortcut r NULL = none, r with r_stats NULL = raw bf16, else gn(r)
 *   with its own statistics.
 * maxpool3s2: 3x3 stride-2 max pool, zero padding pad_top/pad_left and past the bottom/right
 *   edge (BitMaxPool2d with DynamicPad2d, modeling_bit.py:199-223). */
int i2pc_bit_stem_im2col(const float* pixels, int batch, int h, int w, int out_h, int out_w, int pad_top,
                         int pad_left, int ksize, int k_pitch, void* out, void* stream);
size_t i2pc_groupnorm_workspace_bytes(int batch, int hw, int groups);
int i2pc_groupnorm_stats(const void* x, int batch, int hw, int c, int groups, float eps, float* stats,
                         void* workspace, size_t workspace_bytes, void* stream);
int i2pc_groupnorm_apply(const void* x, const float* stats, const float* gamma, const float* beta, const void* r,
                         const float* r_stats, const float* r_gamma, const float* r_beta, int batch, int hw, int c,
                         int groups, int relu, void* y, void* stream);
int i2pc_maxpool3s2(const void* x, int batch, int h, int w, int c, int out_h, int out_w, int pad_top, int pad_left,
                    void* y, void* stream);

/* Name of the kernel instance i2pc_gemm would launch for `desc` (profiling labels;
 * no device work).  Returns "invalid" for a descriptor i2pc_gemm would reject. */
const char* i2pc_gemm_kernel_name(const i2pc_gemm_desc* desc);

/* GEMM engine selection for calls made from the CALLING THREAD (thread-local: a setting on one
 * host thread never changes the kernels another thread's calls launch): 0 = automatic (the
 * persistent 256-column engine for calls with >= 3 tiles per CU whose epilogue it implements,
 * else the tile kernel), 1 = tile kernel only, 2 = persistent engine wherever its epilogue
 * applies, 3 = automatic with the ping-pong persistent engine (k_gemm_8p: dense A, plain /
 * fp32-residual epilogues, K >= 128) where the persistent engine would run, 4 = ping-pong engine
 * wherever it applies.  All modes give bit-identical results for the same split-K choice;
 * split-K (i2pc_gemm_ws with a workspace, knob "gemm_splitk") runs in modes 0 and 3 only and adds
 * the fp32 partial sums in another order, so a few-tile K >= 4096 call may differ in the last
 * bits between modes 0/3 and 1/2/4, and between i2pc_gemm (never splits) and i2pc_gemm_ws. */
int i2pc_gemm_set_engine(int mode);

/* Kernel-selection knobs for A/B measurement (not part of the drop-in surface).  Like the engine
 * mode they are THREAD-LOCAL: each host thread starts from the defaults below and a change
 * affects only the calls that thread makes, so concurrent callers on other threads / streams keep
 * their kernels (the re-entrancy promise above).  Every setting but gemm_splitk computes the same
 * results bit for bit:
 *   "gemm_tail"   1 = split the last round of a persistent GEMM into 256 x 128 tiles where that
 *                 saves a round
 *   "gemm_bn128"  1 = the persistent engine with 256 x 128 tiles for N % 256 != 0, N % 128 == 0
 *   "gemm_splitk" 1 = split-K for few-tile long-K calls given a workspace (i2pc_gemm_ws); the one
 *                 knob that changes results: the fp32 partial sums are added in another order
 *                 (within the network parity tolerance, tests/test_gemm_engines_gpu.py)
 *   "gemm_split_tile" split-K slice tile: 0 = 256 x 256 x 64 (default), 1 = 128 x 128 x 32
 *   "gemm_tile192" 1 = 384 x 192 tiles for N % 192 == 0 calls that fit one round
 *   "gemm_lnp_p"  1 = LayerNorm-fold producers (ln_part) on the persistent engine (160 x 256 or
 *                 256 x 256 tiles, N % 256 == 0), 0 = on the tile kernel (default: measured faster)
 *   "gemm_lnp_stream" bf16-stream producers (bf16 res + res_shift, bf16 out) on the persistent engine
 *                 (full rounds of 256 x 256 tiles + a 160-row remainder round; N % 256 == 0):
 *                 0 = the tile kernel (default: measured faster, r06), 1 = where K <= 2048, 2 = every K;
 *                 bit-identical
 *   "conv_halo"   3x3 stride-1 pad-1 convs of 64-channel NHWC maps (N % 64 == 0) on the LDS-halo kernel
 *                 (one input halo per spatial output tile, the nine taps read from LDS): 1 = 16 x 16
 *                 pixels / 4 waves, 2 = 16 x 16 / 8 waves, 3 = 8 x 16 / 4 waves (default), 4 = 8 x 32 /
 *                 4 waves; 0 = the implicit GEMM.  Bit-identical (same K order)
 *   "gelu_tanh"   1 = act 1 (GELU) evaluated in the tanh form x * sigmoid(1.5958 (x + 0.044715 x^3))
 *                 (|difference to the erf form| <= 2.2e-4; default), 0 = the erf form
 *   "gemm_resq"   1 = the 8-wave 320 x 256 / 384 x 192 tile kernels stage a bf16 residual's rows in LDS
 *                 one epilogue pass ahead (LDS-DMA, one wait per pass); 2 = also the row shifts in LDS
 *                 and the bias in registers before the first pass, and each pass's wait counted past the
 *                 previous pass's stores (default); 0 = plain loads in the epilogue; bit-identical
 *   "gemm_simple_epi" 1 = tile / halo-conv kernel calls whose epilogue is bias (+ activation) (+ a bf16
 *                 residual) -> bf16 run an epilogue compiled without the generic one's other features
 *                 (default), 0 = the generic epilogue; bit-identical
 *   "gemm_tail160" 1 = a persistent GEMM's last partial round as 160 x 256 tiles where 256 x 128
 *                 tiles do not fit one round (DPT-Large FC1)
 *   "gemm_stagger" 1 = in the 8-wave GEMM kernels waves 4-7 issue the next K-stage's loads half-way
 *                 through each K-step (their SIMD partners' MFMAs cover the issue), 0 = every wave at
 *                 the top of the step
 *   "unp_rows"    1 = the row-sweep unprojection kernel
 *   "unp_nt"      1 = non-temporal point stores
 *   "unp_rpt"     point rows per thread of the row-sweep kernel, 1..8
 *   "sel_windows" 1 = the window-only p2 / p98 selection of i2pc_unproject (one sweep), 0 = the
 *                 histogram levels (the band path's)
 *   "sel_parts"   sub-batches of i2pc_unproject's selection chain, run on forked side streams so
 *                 their small launches overlap (joined before the unprojection launch; graph
 *                 capture follows the fork); 0 = automatic = 1 (2-4 measured slower, r03)
 *   "sel_rows"    output rows per selection-sweep workgroup, 1..64 (default 16)
 *   "sel_lband"   a single image's windows resolved by the band kernels with a local exchange
 *                 (fine histogram and target-bin compaction over 96 workgroups) instead of one
 *                 workgroup per window: -1 = automatic (from 2 M pixels; default), 0 = off, 1 = on
 *   "sel_scratch" 1 = every image of a window selection goes to the selection from scratch (the
 *                 fallback of a missed window; tests and measurement only), default 0
 *   "attn_lazy"   1 = skip the softmax rescale of a key tile that raised no row's running max
 *   "attn_scalar" 1 = unpacked exponent FMAs and a permlane row max
 *   "attn_rb"     i2pc_attention_q2 / _q2_fp8: 1 = each 32-key half's K (and V^T) fragment reads issued
 *                 together ahead of their MFMAs (counted waits), 0 = one read per MFMA; bit-identical,
 *                 default 1
 *   "ln_f2"       1 = the register-resident LayerNorm for dim 384 (k_layernorm2)
 *   "ln_apply_gs" DIAGNOSTIC reproducer of the r04 nondeterminism: 1 = i2pc_ln_apply as
 *                 the r04 grid-stride kernel (row statistics by vector loads), 2 / 3 / 4 / 5 = the same with an
 *                 agent-scope acquire first / agent-scope loads / a vector-L1 invalidate first / agent-scope
 *                 loads of the row statistics only; 0 = the product kernel (default)
 *   "resize_rows" 1 = bilinear resizes / 2x upsamples whose channel count is a power of two (8..2048)
 *                 run row-mapped (k_resize_rowmap: no per-output index divisions, lane-consecutive
 *                 taps; bit-identical), 0 = the flat-index kernels; default 1
 * Defaults: the I2PC_GEMM_TAIL / _GEMM_BN128 / _GEMM_SPLITK / _GEMM_SPLIT_TILE / _GEMM_TILE192 /
 * _GEMM_LNP_P / _GEMM_TAIL160 / _GEMM_STAGGER / _UNP_ROWS / _UNP_NT / _UNP_RPT / _SEL_WIN / _ATTN_LAZY /
 * _ATTN_SCALAR environment variables, else 1, 1, 1, 0, 1, 0, 1, 1, 1, 1, 8, 1, 1, 1; sel_parts 0, sel_rows 16, sel_lband -1, ln_f2 1.  A HIP graph keeps
 * the kernels it captured: re-capture after changing a knob.  An unknown name fails with I2PC_EINVAL
 * and an error message listing every knob. */
int i2pc_set_tuning(const char* name, int value);

/* LayerNorm over the last dim: x fp32 [rows][dim] (row stride ldx) -> y bf16 [rows][dim]
 * (row stride ldy); gamma/beta fp32 [dim]; two-pass mean/variance in fp32.
 * (nn.LayerNorm, modeling_dpt.py:233-234). dim % 64 == 0, dim <= 2048. */
int i2pc_layernorm(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps,
                   int rows, int dim, void* y, int64_t ldy, void* stream);
/* i2pc_layernorm that also stores each row's mean (fp32 [rows]; e.g. the first ln_shift of a
 * LayerNorm-folded encoder). */
int i2pc_layernorm_stats(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps,
                         int rows, int dim, void* y, int64_t ldy, float* row_mean, void* stream);

/* Fused multi-head self-attention (softmax(Q K^T * scale) V, no mask), head_dim 64.
 * qkv: bf16 [batch*tokens][3*heads*64] (Q | K | V column blocks, the fused QKV GEMM output);
 * out: bf16 [batch*tokens][heads*64]. (DPTSelfAttention, modeling_dpt.py:123-154) */
int i2pc_attention(const void* qkv, int batch, int tokens, int heads, float scale, void* out, void* stream);
/* i2pc_attention writing the MX fp8 operand of the next GEMM (DPT-Hybrid's attention-out on the fp8
 * engine) instead of bf16: out e4m3fn [batch*tokens][ldo = heads*64], out_scale E8M0 bytes, row r's
 * 32-column block j at byte r * ldo_scale * 4 + j (ldo_scale in dwords, >= heads*64/128).  The bytes
 * equal i2pc_quant_fp8 of i2pc_attention's bf16 output (quantised from the bf16-rounded values) under
 * the same "attn_scalar" / "attn_lazy" knobs; the diagnostic I2PC_ATTN_OCC / I2PC_ATTN_OLD variants of
 * i2pc_attention have no fp8 twin. */
int i2pc_attention_fp8(const void* qkv, int batch, int tokens, int heads, float scale, void* out, int64_t ldo,
                       void* out_scale, int64_t ldo_scale, void* stream);
/* i2pc_attention with Q already in the exp2 domain: the Q block of qkv holds q * scale * log2(e) (the
 * network folds that factor into the Q rows of its QKV weights and bias in fp32, before their bf16
 * rounding), and out = softmax_2(Q K^T) V = softmax(q K^T * scale) V.  Runs the threshold-rescale
 * kernel (k_attention_fast: no per-score scale FMA or tile max; the running max moves only when a
 * tile's probabilities could reach 2^8).  Same argument rules as i2pc_attention. */
int i2pc_attention_q2(const void* qkv, int batch, int tokens, int heads, void* out, void* stream);
/* i2pc_attention_q2 writing the MX fp8 operand (as i2pc_attention_fp8; the bytes equal i2pc_quant_fp8
 * of i2pc_attention_q2's bf16 output). */
int i2pc_attention_q2_fp8(const void* qkv, int batch, int tokens, int heads, void* out, int64_t ldo,
                          void* out_scale, int64_t ldo_scale, void* stream);

/* Bilinear 2x upsample, align_corners = True, NHWC bf16 (nn.functional.interpolate,
 * modeling_dpt.py:504-506, 698), optional + add (bf16, output shape). */
int i2pc_upsample2x(const void* x, int batch, int h, int w, int c, const void* add, void* y, void* stream);
/* The same upsample written as the MX fp8 operand of i2pc_gemm_fp8 (e4m3 [pixels][ldy] bytes + E8M0 scale
 * dwords [pixels][ldy_scale]): the bytes equal i2pc_quant_fp8 of i2pc_upsample2x's bf16 output, without
 * that bf16 map (DPT-Hybrid fp8: the last fusion stage's output feeds only the head's first conv).
 * c % 32 == 0, ldy % 16 == 0. */
int i2pc_upsample2x_fp8(const void* x, int batch, int h, int w, int c, const void* add, void* y, int64_t ldy,
                        void* y_scale, int64_t ldy_scale, void* stream);

/* General bilinear resize of an NHWC bf16 map to out_h x out_w with torch's
 * upsample_bilinear2d index rules (align_corners 1: the DPT/Depth-Anything fusion and
 * head resizes, modeling_depth_anything.py:169-174, 296-301; 0: the fusion residual
 * resize, :161-163), optional + add (bf16, output shape). c % 8 == 0. */
int i2pc_resize_bilinear(const void* x, int batch, int h, int w, int c, int out_h, int out_w,
                         int align_corners, const void* add, void* y, void* stream);

/* Elementwise helpers of the ViT stem / neck. */
/* rows [b*tokens + 0] of the fp32 residual stream = cls + pos[0] (modeling_dpt.py:226-231) */
int i2pc_cls_pos(const float* cls, const float* pos0, int batch, int tokens, int dim, float* x, void* stream);
/* fp32 -> bf16 copy of a [rows][dim] block */
int i2pc_f32_to_bf16(const float* x, int64_t n, void* y, void* stream);
/* depth[b][p] = relu( sum_c x[b][p][c] * w[c] + bias ), x bf16 NHWC with c <= 64
 * (last 1x1 conv + ReLU of DPTDepthEstimationHead, modeling_dpt.py:701-702) */
int i2pc_head_out(const void* x, int64_t pixels, int c, const float* w, float bias, float* depth, void* stream);
/* Fused head tail (DPTDepthEstimationHead head[1..5], modeling_dpt.py:679-716, and the
 * Depth-Anything head after conv1): depth[b][y][x] = relu(b4 + sum_co w4[co] *
 * bf16(relu(b2[co] + conv3x3(resize_ac(x), w2)[co]))) where resize_ac is the bilinear
 * align_corners=True resize of x (bf16 NHWC [batch, h, w, c], pitch c % 8 == 0, of which the
 * first cin channels are used, cin % 32 == 0: Depth-Anything-V2-Small pads its 32 head
 * channels to 64) to (out_h, out_w); w2: bf16 [32][9*c] packed (ky, kx, ci); b2, w4: fp32
 * [32]; depth fp32 [batch, out_h, out_w].  Replaces i2pc_resize_bilinear + a 3x3 conv +
 * i2pc_head_out without materialising the resized map.  The resize must not shrink by more
 * than a tile's LDS source window holds (the heads enlarge: 2x for DPT, 1.75x for DA). */
int i2pc_head_upconv(const void* x, int batch, int h, int w, int c, int cin, int out_h, int out_w, const void* w2,
                     const float* b2, const float* w4, float b4, float* depth, void* stream);

/* Area-averaging downscale, cv2.resize(image, (out_w, out_h), interpolation=INTER_AREA)
 * as process_image_pipeline applies it above 3072 px (backend/app.py:436-445); OpenCV's
 * published algorithm restated (parity against cv2 unpinned: not installed here).
 * src uint8 [batch, h, w, channels] -> dst uint8 [batch, out_h, out_w, channels];
 * out_h <= h and out_w <= w (EUNSUPPORTED otherwise). */
int i2pc_resize_area(const uint8_t* src, int batch, int h, int w, int channels, uint8_t* dst, int out_h, int out_w,
                     void* stream);

/* ------------------------------------------------------------------------
 * Network input (app.py:103 cvtColor BGR->RGB + app.py:109 DPTImageProcessorPil):
 * Pillow-exact bicubic resample, rescale 1/255, normalise, optional patchify.
 * A plan holds the per-size Pillow coefficient tables (computed on the host and
 * uploaded once: create/destroy are NOT stream-ordered; i2pc_preprocess is).
 * ------------------------------------------------------------------------ */
typedef struct i2pc_preprocess_plan i2pc_preprocess_plan;
int i2pc_preprocess_plan_create(int in_h, int in_w, int out_h, int out_w, const float* mean3, const float* std3,
                                int patch, i2pc_preprocess_plan** plan);
void i2pc_preprocess_plan_destroy(i2pc_preprocess_plan* plan);
/* bgr: uint8 [batch, in_h, in_w, 3]; layout 0 -> float32 [batch, 3, out_h, out_w] (pixel_values);
 * layout 1 -> bf16 [batch * (out_h/patch)*(out_w/patch)][pitch], pitch = 3*patch*patch rounded up
 * to a multiple of 64 (the GEMM K granule; 768 for patch 16, 640 for patch 14), column order
 * (c, py, px) (the im2col of the patch-embedding conv, modeling_dpt.py:60-69,
 * modeling_dinov2.py Dinov2PatchEmbeddings); the pad columns are never written (zero them once). */
int i2pc_preprocess(const i2pc_preprocess_plan* plan, const uint8_t* bgr, int batch, int layout, void* out, void* stream);

/* ------------------------------------------------------------------------
 * Network executor: the whole depth stage of process_with_depth_anything (backend/app.py:99-122:
 * BGR->RGB :103, the processor :109, the forward :111-116) for a batch, with no Python.  The model is
 * a prepared-network file (image_to_pointcloud_amd/model_file.py writes it from a loaded network:
 * Depth-Anything-V2, the reference's `load_model("depth-anything-v2")`, app.py:78-82) made for one
 * input size; i2pc_model_create uploads its weights and allocates every buffer once, so
 * i2pc_depth_forward is launch-only and stream-ordered (graph-capturable).  The depth equals the
 * Python pipeline's (PointCloudPipeline.infer_depth) bit for bit.
 * ------------------------------------------------------------------------ */
typedef struct i2pc_model i2pc_model;
/* Read a prepared-network file for `batch` images of in_h x in_w (must be the size the file was made
 * for).  EUNSUPPORTED for a family / configuration the executor does not run. */
int i2pc_model_create(const char* path, int batch, int in_h, int in_w, i2pc_model** model);
int i2pc_model_destroy(i2pc_model* model);
/* The batch, input size and model-resolution depth size (depth_h x depth_w) of a model. */
int i2pc_model_io(const i2pc_model* model, int* batch, int* in_h, int* in_w, int* depth_h, int* depth_w);
/* bgr: uint8 [batch][in_h][in_w][3] (cv2 order, app.py:99) on the device -> depth fp32
 * [batch][depth_h][depth_w] (predicted_depth, app.py:116), on `stream`. */
int i2pc_depth_forward(i2pc_model* model, const uint8_t* bgr, float* depth, void* stream);
/* Host-only check of a prepared-network file: its 32 header ints, 16 header floats and tensor
 * count (model_file.py I_* / F_* slots); no device work. */
int i2pc_model_file_info(const char* path, int32_t* ints32, float* floats16, int* ntensors);

/* ------------------------------------------------------------------------
 * Artefact writers (save_point_cloud, backend/app.py:310-389) from HOST buffers
 * (xyz float32 [n][3], rgb uint8 [n][3] or NULL for grey 128). Not stream-ordered.
 * ------------------------------------------------------------------------ */
/* XYZ ASCII "%.6f %.6f %.6f %d %d %d\n" (save_xyz, app.py:380-389); `threads` format in parallel. */
int i2pc_write_xyz(const char* path, const float* xyz, const uint8_t* rgb, int64_t n, int threads);
/* Binary little-endian PLY, double x/y/z + uchar red/green/blue (save_ply via Open3D, app.py:333-345). */
int i2pc_write_ply(const char* path, const float* xyz, const uint8_t* rgb, int64_t n);
/* LAS 1.2 point format 2, offsets = per-axis min, scale `scale` (0.01 in the reference),
 * RGB = c*256 (save_las via laspy, app.py:347-378). n must be > 0. */
int i2pc_write_las(const char* path, const float* xyz, const uint8_t* rgb, int64_t n, double scale);

#ifdef __cplusplus
}
#endif
#endif /* I2PC_H_ */

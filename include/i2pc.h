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
 *   - re-entrant; one call may run per stream concurrently.
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
  int32_t smooth_ksize;/* kernel size; only the default 5 is supported */
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

/* Gather every stride-th point (preview subsample, app.py:496-506):
 * out_xyz/out_rgb [count] with count = ceil(n / stride). */
int i2pc_gather_stride(const float* xyz, const uint8_t* rgb, int64_t n, int64_t stride,
                       float* out_xyz, float* out_rgb, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* I2PC_H_ */

/* A C caller of the native network executor (include/i2pc.h): the whole depth stage of
 * process_with_depth_anything (backend/app.py:99-122) with no Python.
 *
 *   depth_forward <network file> <batch> <in_h> <in_w> <images.u8> <depth.f32>
 *
 * images.u8: batch x in_h x in_w x 3 uint8 BGR (raw bytes); depth.f32 receives
 * batch x depth_h x depth_w float32 (raw).  The network file is written once by
 * image_to_pointcloud_amd.model_file.export_depth_anything. */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>

#include "i2pc.h"

static int fail(const char* what) {
  fprintf(stderr, "depth_forward: %s: %s\n", what, i2pc_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s <network file> <batch> <in_h> <in_w> <images.u8> <depth.f32>\n", argv[0]);
    return 2;
  }
  const int batch = atoi(argv[2]), in_h = atoi(argv[3]), in_w = atoi(argv[4]);
  i2pc_model* m = NULL;
  if (i2pc_model_create(argv[1], batch, in_h, in_w, &m)) return fail("i2pc_model_create");
  int b, ih, iw, dh, dw;
  if (i2pc_model_io(m, &b, &ih, &iw, &dh, &dw)) return fail("i2pc_model_io");
  const size_t nin = (size_t)b * ih * iw * 3, nout = (size_t)b * dh * dw;
  unsigned char* h_in = (unsigned char*)malloc(nin);
  float* h_out = (float*)malloc(nout * sizeof(float));
  FILE* f = fopen(argv[5], "rb");
  if (!f || fread(h_in, 1, nin, f) != nin) { fprintf(stderr, "depth_forward: cannot read %s\n", argv[5]); return 1; }
  fclose(f);
  void *d_in = NULL, *d_out = NULL;
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess || hipMalloc(&d_in, nin) != hipSuccess ||
      hipMalloc(&d_out, nout * sizeof(float)) != hipSuccess ||
      hipMemcpyAsync(d_in, h_in, nin, hipMemcpyHostToDevice, s) != hipSuccess) {
    fprintf(stderr, "depth_forward: HIP setup failed\n");
    return 1;
  }
  if (i2pc_depth_forward(m, (const uint8_t*)d_in, (float*)d_out, s)) return fail("i2pc_depth_forward");
  if (hipMemcpyAsync(h_out, d_out, nout * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    fprintf(stderr, "depth_forward: copy back failed\n");
    return 1;
  }
  f = fopen(argv[6], "wb");
  if (!f || fwrite(h_out, sizeof(float), nout, f) != nout) { fprintf(stderr, "depth_forward: cannot write %s\n", argv[6]); return 1; }
  fclose(f);
  printf("depth_forward: %d images %dx%d -> depth %dx%d\n", b, ih, iw, dh, dw);
  i2pc_model_destroy(m);
  hipFree(d_in);
  hipFree(d_out);
  hipStreamDestroy(s);
  free(h_in);
  free(h_out);
  return 0;
}

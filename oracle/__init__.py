"""CPU oracle for the image -> point-cloud hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package
(`image_to_pointcloud_amd/`) imports, links or executes anything from this
directory.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may use it, and only as the checker / the timed CPU
baseline -- never as the thing measured or shipped.

Contents
--------
unproject_ref.py   numpy / pure-Python restatement of
                   /root/reference/backend/app.py:174-250 (depth_to_point_cloud),
                   :391-417 (generate_gis_metadata), :496-506 (preview stride),
                   plus numpy-2 percentile / nanmedian semantics it relies on.
preprocess_ref.py  restatement of the DPT image processor (PIL bicubic resample,
                   rescale, normalize) that feeds the depth network
                   (app.py:103,109 -> transformers DPTImageProcessorPil).
sor_ref.py         restatement of refine_point_cloud (app.py:252-269): Open3D's
                   RemoveStatisticalOutliers (open3d>=0.17.0) over an exact scipy
                   cKDTree kNN, itself pinned to brute force.

Parity pinning
--------------
* unprojection / percentiles / bounds / preview: pinned bit-exact against
  golden fixtures produced by importing the reference itself
  (tests/golden/gen_golden.py, run in the build container only).
* cv2.resize(INTER_LINEAR) and cv2.GaussianBlur: OpenCV is absent from the
  container, so these restatements are "parity unpinned" against cv2; they are
  pinned against torch bilinear (align_corners=False) within fp32 rounding.
* PIL bicubic resample: pinned bit-exact against Pillow 12.2 (present here and
  on the GPU box).
* statistical outlier removal: Open3D is absent, so "parity unpinned" against
  Open3D itself; the restatement's kNN is pinned to exhaustive search
  (tests/test_sor.py).

The reference's own C/C++ sources are not on this path (it is Python), so there
is no oracle/_ref build.
"""

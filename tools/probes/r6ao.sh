set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P=$PWD/image_to_pointcloud_amd/libi2pc_prev.so
C=$PWD/image_to_pointcloud_amd/libi2pc.so
mkdir -p gpurun_out
for lib in $C $P $C $P; do
  echo "== $(basename $lib)"
  I2PC_LIB=$lib timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu \
     tests/test_depth_anything_gpu.py tests/test_determinism_gpu.py tests/test_multirank_gpu.py > gpurun_out/r6ao.log 2>&1
  rc=$?; grep -E "passed|failed|^E .*runs differ|^E .*AssertionError" gpurun_out/r6ao.log | head -5
  [ $rc -le 1 ] || exit $rc
done

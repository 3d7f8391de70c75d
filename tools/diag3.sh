set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so
O=gpurun_out/diag3.txt; rm -f $O
for v in 0 1 3 5; do
  echo "== 8192^2 x 1024 persistent, diag bits $v (1 drop stores, 2 same tile, 4 no loads)" >> $O
  I2PC_GEMM_DROP_STORES=$v I2PC_GEMM_P=2 timeout -k 10 120 python -u tools/stamps_p.py 8192 8192 1024 >> $O 2>&1 || exit 1
done
grep -v amdgpu.ids $O

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/diag17.txt; rm -f $O
timeout -k 10 600 python -u -m pytest tests/test_ln_fold_gpu.py tests/test_gemm_engines_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t17.log 2>&1 || { tail -30 gpurun_out/t17.log; exit 1; }
tail -1 gpurun_out/t17.log >> $O
for lib in sold snew sold snew; do
  echo "== $lib" >> $O
  for a in "18464 1024 1024 320 256 bf16" "18464 1024 1024 320 256 lnpbf" "18464 1024 4096 320 256 lnpbf" "43840 384 1536 384 192 lnpbf"; do
    I2PC_LIB=image_to_pointcloud_amd/libi2pc_$lib.so timeout -k 10 120 python -u tools/stamps_tile.py $a >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O | sed 's/start.*first/first/; s/end.*//'

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/diag4.txt; rm -f $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_engines_gpu.py tests/test_ln_fold_gpu.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/eng.log 2>&1 || { tail -20 gpurun_out/eng.log; exit 1; }
tail -2 gpurun_out/eng.log >> $O
for v in 0 1; do
  echo "== stagger $v" >> $O
  I2PC_GEMM_STAGGER=$v I2PC_GEMM_P=2 I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so timeout -k 10 120 python -u tools/stamps_p.py 8192 8192 1024 >> $O 2>&1 || exit 1
  I2PC_GEMM_STAGGER=$v I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so timeout -k 10 120 python -u tools/stamps_p.py 18464 4096 1024 gelu >> $O 2>&1 || exit 1
done
timeout -k 10 600 python -u tools/ab_pipeline.py --variant base: --variant nostagger:gemm_stagger=0 >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O

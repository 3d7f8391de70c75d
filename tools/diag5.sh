set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/diag5.txt; rm -f $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_engines_gpu.py tests/test_ln_fold_gpu.py tests/test_padding_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/eng.log 2>&1 || { tail -20 gpurun_out/eng.log; exit 1; }
tail -1 gpurun_out/eng.log >> $O
for v in 0 1; do
  echo "== stagger $v" >> $O
  for a in "18464 1024 1024 320 256 lnp" "18464 1024 4096 320 256 lnp"; do
  I2PC_GEMM_STAGGER=$v I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so timeout -k 10 120 python -u tools/stamps_tile.py $a >> $O 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u tools/ab_pipeline.py --variant base: --variant nostagger:gemm_stagger=0 >> $O 2>&1 || exit 1
timeout -k 10 600 python -u tools/ab_pipeline.py --model depth-anything-v2 --variant base: --variant nostagger:gemm_stagger=0 >> $O 2>&1 || exit 1
timeout -k 10 600 python -u tools/ab_pipeline.py --model dpt-hybrid --batch 64 --variant base: --variant nostagger:gemm_stagger=0 >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O

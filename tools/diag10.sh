set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/diag10.txt; rm -f $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_engines_gpu.py tests/test_ln_fold_gpu.py tests/test_padding_gpu.py tests/test_kernels_gpu.py tests/test_depth_anything_gpu.py tests/test_dpt_gpu.py -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/t10.log 2>&1 || { tail -30 gpurun_out/t10.log; exit 1; }
grep -h '^parity' gpurun_out/t10.log >> $O; tail -1 gpurun_out/t10.log >> $O
for lib in stamps_old stamps stamps_old stamps; do
  echo "== $lib" >> $O
  for a in "18464 1024 1024 320 256 bf16" "18464 1024 1024 320 256 lnp" "294912 256 2304 320 256 bf16"; do
    I2PC_LIB=image_to_pointcloud_amd/libi2pc_$lib.so timeout -k 10 120 python -u tools/stamps_tile.py $a >> $O 2>&1 || exit 1
  done
done
echo "== new lnpbf" >> $O
I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so timeout -k 10 120 python -u tools/stamps_tile.py 18464 1024 1024 320 256 lnpbf >> $O 2>&1 || exit 1
for v in 1 0 1 0; do
  I2PC_BF16_STREAM=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b10_$v.json 2>/dev/null || exit 1
  echo "stream=$v $(python -c "import json;d=json.loads(open('gpurun_out/b10_$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['rooflines']['dpt_blocks']['frac'])")" >> $O
done
for v in 1 0; do
  I2PC_BF16_STREAM=$v timeout -k 10 300 python -u bench.py --model depth-anything-v2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b10da_$v.json 2>/dev/null || exit 1
  echo "DA stream=$v $(python -c "import json;d=json.loads(open('gpurun_out/b10da_$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['rooflines']['dpt_blocks']['frac'])")" >> $O
done
grep -v amdgpu.ids $O

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/diag8.txt; rm -f $O
for a in "18464 1024 1024 320 256 bf16" "18464 1024 1024 320 256 lnp" "18464 1024 1024 320 256 lnpbf" "18464 1024 4096 320 256 lnp" "18464 1024 4096 320 256 lnpbf"; do
  I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so timeout -k 10 120 python -u tools/stamps_tile.py $a >> $O 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/epi_cost.py >> $O 2>&1 || exit 1
D=gpurun_out/tr8; rm -rf $D; mkdir -p $D
I2PC_BF16_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/s1 -o t --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/b1.json 2>&1 || exit 1
I2PC_BF16_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/s0 -o t --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/b0.json 2>&1 || exit 1
grep -v amdgpu.ids $O

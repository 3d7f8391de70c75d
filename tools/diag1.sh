set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so
for a in "18464 1024 1024 320 256 bf16" "18464 1024 1024 320 256 lnp" "18464 1024 4096 320 256 bf16" "18464 1024 4096 320 256 lnp"; do
  timeout -k 10 120 python -u tools/stamps_tile.py $a >> gpurun_out/stamps_tile.txt 2>&1 || exit 1
done
for a in "18464 3072 1024" "18464 4096 1024 gelu"; do
  timeout -k 10 120 python -u tools/stamps_p.py $a >> gpurun_out/stamps_p.txt 2>&1 || exit 1
done
unset I2PC_LIB
D=gpurun_out/epi_trace; rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o t --output-format csv -- python -u tools/epi_cost.py > gpurun_out/epi.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamps_tile.txt gpurun_out/stamps_p.txt gpurun_out/epi.log

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/diag12.txt; rm -f $O
for lib in s0 s1 s2 s0 s1 s2; do
  echo "== $lib" >> $O
  for a in "18464 1024 1024 320 256 bf16" "18464 1024 1024 320 256 lnpbf" "18464 1024 4096 320 256 lnpbf" "43840 384 1536 384 192 lnpbf"; do
    I2PC_LIB=image_to_pointcloud_amd/libi2pc_$lib.so timeout -k 10 120 python -u tools/stamps_tile.py $a >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O | grep -v "^blocks" 
grep -v amdgpu.ids $O | grep "^blocks" | sed 's/start.*first/first/; s/end.*//' 

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so
O=gpurun_out/diag2.txt; rm -f $O
echo "== QKV stores dropped" >> $O
I2PC_GEMM_DROP_STORES=1 timeout -k 10 120 python -u tools/stamps_p.py 18464 3072 1024 >> $O 2>&1 || exit 1
echo "== QKV tail split off (4 full rounds)" >> $O
I2PC_GEMM_TAIL=0 timeout -k 10 120 python -u tools/stamps_p.py 18464 3072 1024 >> $O 2>&1 || exit 1
echo "== O-proj shape on the persistent engine (292 tiles)" >> $O
I2PC_GEMM_P=2 timeout -k 10 120 python -u tools/stamps_p.py 18464 1024 1024 >> $O 2>&1 || exit 1
echo "== 4096^2 x 1024: one full round" >> $O
I2PC_GEMM_P=2 timeout -k 10 120 python -u tools/stamps_p.py 4096 4096 1024 >> $O 2>&1 || exit 1
echo "== 8192^2 x 1024: four rounds" >> $O
I2PC_GEMM_P=2 timeout -k 10 120 python -u tools/stamps_p.py 8192 8192 1024 >> $O 2>&1 || exit 1
echo "== 8192^2 x 1024: four rounds, stores dropped" >> $O
I2PC_GEMM_DROP_STORES=1 I2PC_GEMM_P=2 timeout -k 10 120 python -u tools/stamps_p.py 8192 8192 1024 >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O

set -o pipefail
cd $GRAFT_REPO_ROOT
export I2PC_LIB=$GRAFT_REPO_ROOT/image_to_pointcloud_amd/libi2pc_stamps.so
timeout -k 10 120 python tools/stamps_p.py 18464 3072 1024 > gpurun_out/stamps_p.txt 2>&1 || exit 1
timeout -k 10 120 python tools/stamps_p.py 18464 4096 1024 gelu >> gpurun_out/stamps_p.txt 2>&1 || exit 1
timeout -k 10 120 python tools/stamps_p.py 18464 1024 4096 >> gpurun_out/stamps_p.txt 2>&1 || exit 1
echo all_ok

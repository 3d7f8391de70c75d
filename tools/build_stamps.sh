# Diagnostic build: libi2pc_stamps.so = libi2pc.so with s_memtime stamps in the GEMM kernels.
set -e
cd "$(dirname "$0")/.."
python -m image_to_pointcloud_amd.build > /dev/null
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -I include \
  -DI2PC_STAMPS -c image_to_pointcloud_amd/csrc/gemm.hip -o build/i2pc/gemm_stamps.o
objs=$(ls build/i2pc/*.o | grep -v -e gemm.o -e gemm_stamps.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o image_to_pointcloud_amd/libi2pc_stamps.so $objs build/i2pc/gemm_stamps.o -lrccl
echo built stamps lib

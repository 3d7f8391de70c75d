# Diagnostic: libi2pc_<tag>.so = libi2pc.so with gemm.hip built with extra flags (e.g. -DI2PC_EPI_PRE=1 -DI2PC_STAMPS)
# usage: bash tools/build_variant.sh <tag> <flags...>
set -e
cd "$(dirname "$0")/.."
tag=$1; shift
python -m image_to_pointcloud_amd.build > /dev/null
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -I include \
  "$@" -c image_to_pointcloud_amd/csrc/gemm.hip -o build/i2pc/gemm_$tag.o
objs=$(ls build/i2pc/*.o | grep -v -e 'gemm.o' -e 'gemm_')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o image_to_pointcloud_amd/libi2pc_$tag.so $objs build/i2pc/gemm_$tag.o -lrccl
echo built libi2pc_$tag.so

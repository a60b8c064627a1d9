#!/bin/bash
# Variant libslam355.so for A/B and counter runs on the GPU box:
#   scripts/build_variant.sh NAME FILE.hip [extra hipcc flags...]
# recompiles one source file of the current tree with the extra flags and links
# it with the default objects of slam-1_amd/build/ into slam-1_amd/prof/libslam355_NAME.so
# (run `make -C slam-1_amd` first).
set -e
NAME=$1
SRC=$2
shift 2
cd "$(dirname "$0")/../slam-1_amd"
mkdir -p prof/build_$NAME
base=$(basename "$SRC" .hip)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics \
  -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-mfma-vgpr-form "$@" \
  -c "csrc/$base.hip" -o "prof/build_$NAME/$base.o"
objs=$(ls build/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "prof/libslam355_$NAME.so" $objs "prof/build_$NAME/$base.o"
echo "prof/libslam355_$NAME.so"

#!/bin/bash
# Like build_variant.sh, but the source file comes from another directory (e.g. a
# previous revision: git show REV:slam-1_amd/csrc/ba.hip > DIR/ba.hip, plus the
# headers it includes):  scripts/build_variant_src.sh NAME DIR/FILE.hip [flags...]
set -e
NAME=$1
SRC=$(readlink -f "$2")
shift 2
cd "$(dirname "$0")/../slam-1_amd"
mkdir -p prof/build_$NAME
base=$(basename "$SRC" .hip)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics \
  -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-mfma-vgpr-form -I csrc -I ../include "$@" \
  -c "$SRC" -o "prof/build_$NAME/$base.o"
objs=$(ls build/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "prof/libslam355_$NAME.so" $objs "prof/build_$NAME/$base.o"
echo "prof/libslam355_$NAME.so"

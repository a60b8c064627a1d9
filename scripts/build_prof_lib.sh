#!/bin/bash
# Instrumented libslam355.so variant: build_prof_lib.sh NAME -DFLAG [...] ->
# slam-1_amd/prof/libslam355_NAME.so (profiling scripts select it with SLAM355_LIB).
set -e
NAME="$1"
shift
cd "$(dirname "$0")/../slam-1_amd"
mkdir -p "prof/build_$NAME"
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics \
    -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-mfma-vgpr-form "$@" -c $f -o "prof/build_$NAME/$(basename $f .hip).o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "prof/libslam355_$NAME.so" prof/build_$NAME/*.o

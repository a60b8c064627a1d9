#!/bin/bash
# Instrumented libslam355.so (-DSLAM_ORB_PROFILE: per-phase cycle counters of
# k_orb_tile) for scripts/orb_prof.py, built in slam-1_amd/prof/.
set -e
cd "$(dirname "$0")/../slam-1_amd"
mkdir -p prof/build_orb
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics \
    -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-mfma-vgpr-form -DSLAM_ORB_PROFILE -c $f -o prof/build_orb/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o prof/libslam355_orbprof.so prof/build_orb/*.o

#!/bin/bash
# Instrumented libslam355.so (-DSLAM_LINM_PROFILE: per-workgroup phase stamps of
# k_lin_mfma) for scripts/linm_prof.py, built in slam-1_amd/prof/.
set -e
cd "$(dirname "$0")/../slam-1_amd"
mkdir -p prof/build_linm
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics \
    -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-mfma-vgpr-form -DSLAM_LINM_PROFILE -c $f -o prof/build_linm/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o prof/libslam355_linm.so prof/build_linm/*.o

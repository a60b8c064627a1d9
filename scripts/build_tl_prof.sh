#!/bin/bash
# Instrumented variant of libslam355.so (-DSLAM_TL_PROFILE) for scripts/tl_prof.py,
# built next to the product library (slam-1_amd/prof/), product library rebuilt after.
set -e
cd "$(dirname "$0")/../slam-1_amd"
make -s clean && make -s -j8 HIPFLAGS_EXTRA=-DSLAM_TL_PROFILE
mkdir -p prof && mv slam355/libslam355.so prof/libslam355_tlprof.so
make -s clean && make -s -j8

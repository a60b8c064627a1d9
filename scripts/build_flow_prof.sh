#!/bin/bash
# Instrumented variant of libslam355.so (-DSLAM_FLOW_PROFILE) for scripts/flow_prof.py,
# built into slam-1_amd/prof/, product library rebuilt after.
set -e
cd "$(dirname "$0")/../slam-1_amd"
make -s clean && make -s -j8 HIPFLAGS_EXTRA=-DSLAM_FLOW_PROFILE
mkdir -p prof && mv slam355/libslam355.so prof/libslam355_flowprof.so
make -s clean && make -s -j8

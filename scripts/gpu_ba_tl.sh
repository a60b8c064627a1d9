#!/bin/bash
# Tiled-solver checks: BA/dist parity tests, panel phase timing, C4/C5 bench.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
TAG="${1:-tl}"
bash scripts/gpu_tests.sh "$TAG" tests/test_ba.py tests/test_dist.py && \
SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_tlprof.so timeout -k 10 200 python scripts/tl_prof.py && \
timeout -k 10 300 python bench.py --workload ba --c4 --steps 20 > gpurun_out/bench_c4_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py --workload ba --c5 --steps 5 --warmup 2 > gpurun_out/bench_c5_$TAG.log 2>&1
rc=$?
tail -c 300 gpurun_out/bench_c4_$TAG.log; tail -c 300 gpurun_out/bench_c5_$TAG.log
exit $rc

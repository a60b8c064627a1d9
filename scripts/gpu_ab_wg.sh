#!/bin/bash
# Workgroup-size A/B of the 1024-lane kernels that wait for whole free CUs
# beside ORB (k_assemble, compact_kernel): BA / matcher GPU tests on each
# variant, then the tracking bench alternating.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/r4s2g; mkdir -p $OUT
for v in asm256 cwg256; do
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -k 10 400 python -u -m pytest tests/test_ba.py tests/test_matcher.py tests/test_pipeline.py -x -q -m gpu -k "batched or c3 or window or compact or tracker or knn" --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
done
bash scripts/gpu_ab_tracking.sh r4s2g_tr 3 def asm256 asm512 cwg256 asmcwg || exit 1
for v in def asm256; do
  if [ $v = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
  timeout -k 10 120 python3 bench.py --workload ba --ba-batch 16 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/b16_$v.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/b16_$v.json'));print('b16 $v', round(d['value']), round(d['ms_per_step']*1e3,1))"
done
echo ok

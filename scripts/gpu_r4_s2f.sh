#!/bin/bash
# ORB A/B (NMS candidates of the small levels in LDS vs HEAD): ORB / pipeline /
# BoW GPU parity tests, ORB alone alternating, tracking bench alternating.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/r4s2f; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_orb.py tests/test_pipeline.py tests/test_bow.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_orb.log 2>&1 || { tail -30 $OUT/pytest_orb.log; exit 1; }
tail -1 $OUT/pytest_orb.log
for i in 1 2 3; do
  echo "def $(timeout -k 10 120 python3 scripts/orb_time.py 2>/dev/null | tail -1)" || exit 1
  echo "orbbase $(SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_orbbase.so timeout -k 10 120 python3 scripts/orb_time.py 2>/dev/null | tail -1)" || exit 1
done | tee $OUT/orb_alone.txt
bash scripts/gpu_r4_abn.sh r4s2f_tr 3 def orbbase || exit 1
echo ok

#!/bin/bash
# ORB restructure check: the ORB GPU parity tests, ORB alone (new default vs
# an old build, alternating), the per-level phase profile, then the tracking
# bench A/B.  scripts/gpu_r4_orb.sh TAG OLD_SO [N_AB]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; OLD=$2; N=${3:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_orb.py tests/test_pipeline.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_orb.log 2>&1 || { tail -30 $OUT/pytest_orb.log; exit 1; }
tail -1 $OUT/pytest_orb.log
for i in 1 2 3; do
  timeout -k 10 120 python3 scripts/orb_time.py 2>/dev/null | tail -1 || exit 1
  SLAM355_LIB=$ROOT/$OLD timeout -k 10 120 python3 scripts/orb_time.py 2>/dev/null | tail -1 || exit 1
done
timeout -k 10 120 python3 scripts/orb_prof.py > $OUT/orb_prof.txt 2>/dev/null || exit 1
cat $OUT/orb_prof.txt
bash scripts/gpu_r4_ab_lib.sh $TAG/ab $N $OLD || exit 1

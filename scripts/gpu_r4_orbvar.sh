#!/bin/bash
# ORB variants: parity tests on the default build, ORB alone for the default and
# each variant library (alternating), then the tracking bench A/B of the
# default against each variant.  scripts/gpu_r4_orbvar.sh TAG N_AB VAR_SO...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_orb.py tests/test_pipeline.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_orb.log 2>&1 || { tail -30 $OUT/pytest_orb.log; exit 1; }
tail -1 $OUT/pytest_orb.log
for i in 1 2; do
  timeout -k 10 120 python3 scripts/orb_time.py 2>/dev/null | tail -1 || exit 1
  for v in "$@"; do SLAM355_LIB=$ROOT/$v timeout -k 10 120 python3 scripts/orb_time.py 2>/dev/null | tail -1 || exit 1; done
done
k=0
for v in "$@"; do k=$((k+1)); bash scripts/gpu_r4_ab_lib.sh $TAG/ab$k $N $v || exit 1; done

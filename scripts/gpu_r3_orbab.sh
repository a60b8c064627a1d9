#!/bin/bash
# ORB change check: bit-exact ORB GPU tests with the in-tree library, SQ
# counters of k_orb_tile for each named variant (prof/libslam355_<v>.so), and
# alternating A/B timing of base vs the variants (scripts/orb_time.py).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
shift
OUT="$ROOT/gpurun_out/orbab_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_orb.py tests/test_bow.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
for v in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY \
    -d "$OUT/sq_$v" -o p --output-format csv -- python3 "$ROOT/scripts/orb_run.py" > "$OUT/sq_$v.log" 2>&1) || exit 1
  python scripts/pmc_counters.py "$OUT/sq_$v.json" "$OUT/sq_$v" > /dev/null || exit 1
done
find "$OUT" -name "*.csv" -delete
for rep in 1 2 3; do
  for v in "$@"; do
    SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -k 10 120 python scripts/orb_time.py >> "$OUT/orb_time.log" 2>&1 || exit 1
  done
done
grep ms/launch "$OUT/orb_time.log"
echo done

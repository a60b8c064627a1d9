#!/bin/bash
# ORB LDS study (round 3): per-phase split of LDS instructions / bank
# conflicts from SQ counter passes over the phase-cut builds
# (prof/libslam355_cut{1,2,3,6,7,8}.so, -DSLAM_ORB_CUT), the cycle split
# (-DSLAM_ORB_PROFILE), A/B timing of base vs the named variants, and the ORB
# GPU tests with the in-tree library.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
shift
OUT="$ROOT/gpurun_out/orbcut_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_orb.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_orbprof.so timeout -k 10 200 python scripts/orb_prof.py > "$OUT/orb_prof.log" 2>&1 || exit 1
for v in base cut1 cut2 cut3 cut6 cut7 cut8 "$@"; do
  (cd /tmp && export TMPDIR=/tmp && SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS \
    -d "$OUT/sq_$v" -o p --output-format csv -- python3 "$ROOT/scripts/orb_run.py" > "$OUT/sq_$v.log" 2>&1) || exit 1
  python scripts/pmc_counters.py "$OUT/sq_$v.json" "$OUT/sq_$v" > /dev/null || exit 1
done
find "$OUT" -name "*.csv" -delete
for rep in 1 2; do
  for v in base "$@"; do
    SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -k 10 120 python scripts/orb_time.py >> "$OUT/orb_time.log" 2>&1 || exit 1
  done
done
echo done

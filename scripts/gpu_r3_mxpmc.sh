#!/bin/bash
# SQ counters of the matcher micro-bench (batch 512) for each named variant.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
shift
OUT="$ROOT/gpurun_out/mxpmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    -d "$OUT/sq_$v" -o p --output-format csv -- python3 "$ROOT/bench.py" --workload matcher --batch 512 --steps 3 --warmup 1 > "$OUT/sq_$v.log" 2>&1 || exit 1
  python3 "$ROOT/scripts/pmc_counters.py" "$OUT/sq_$v.json" "$OUT/sq_$v" > /dev/null || exit 1
done
find "$OUT" -name "*.csv" -delete
echo done

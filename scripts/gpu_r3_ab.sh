#!/bin/bash
# A/B timing of ORB builds (alternating processes), then the N=2 bench
# rehearsal (gloo, one GPU) through bench.py's own rank launcher.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
shift
OUT="$ROOT/gpurun_out/ab_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2; do
  for lib in "$@"; do
    SLAM355_LIB=$ROOT/$lib timeout -k 10 120 python scripts/orb_time.py >> "$OUT/orb_time.log" 2>&1 || exit 1
  done
done
grep ms/launch "$OUT/orb_time.log"
echo done

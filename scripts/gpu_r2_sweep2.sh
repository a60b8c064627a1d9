#!/bin/bash
# Tracking bench: disjoint CU partitions for local BA, and BA-after-ORB overlap.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/sweep_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
B="python bench.py --no-cpu-baseline --no-ba-scale --steps 20 --warmup 3"
for c in 16 32 48 64; do
  timeout -k 10 120 $B --ba-cus $c > "$OUT/trk_bacus$c.log" 2>&1 || exit 1
done
timeout -k 10 120 $B --ba-overlap after-orb > "$OUT/trk_afterorb.log" 2>&1 || exit 1
timeout -k 10 120 $B > "$OUT/trk_default.log" 2>&1 || exit 1
echo done

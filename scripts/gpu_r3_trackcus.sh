#!/bin/bash
# Tracking-tail CU mask sweep: the tail's stream limited to the first N CUs
# (ORB on the first 216), local BA unrestricted, alternating with the default.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/trackcus_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for n in 0 216 232 0 200 240 216; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --track-cus $n --steps 16 --warmup 4 > "$OUT/t$n.json" 2> "$OUT/t$n.err" || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/t$n.json')); d['track_cus']=$n; print(json.dumps(d))" >> "$OUT/all.jsonl" || exit 1
done
echo done

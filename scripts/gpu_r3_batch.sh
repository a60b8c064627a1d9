#!/bin/bash
# Frame pairs per step (--batch) sweep of the default tracking bench (windows
# per step follow: one C3 window per 8 frames), each in its own process.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/batch_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for b in 32 64 48 96 32; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --batch $b --steps 12 --warmup 3 > "$OUT/b$b.json" 2> "$OUT/b$b.err" || exit 1
  cat "$OUT/b$b.json" >> "$OUT/all.jsonl"
done
echo done

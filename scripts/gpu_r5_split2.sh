#!/bin/bash
# Round 5: chunks per workgroup of the linearisation for small landmark shards
# (per-rank share of the sharded C4 / C5 iteration, alone on the GPU, HIP wall
# per iteration).   scripts/gpu_r5_split2.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
for cfg in "C4 1 0 2" "C4 1 0 3" "C4 1 0 4" "C4 2 0 1" "C4 2 0 2" "C4 2 0 3" "C4 4 0 1" "C4 4 0 2" "C4 4 0 3" "C4 8 0 1" "C4 8 0 2" "C4 8 0 3" "C5 8 0 1" "C5 8 0 2" "C5 8 0 3" "C5 1 0 2" "C5 1 0 4"; do
  set -- $cfg
  timeout -k 10 120 python3 scripts/shard_split.py $1 $2 $3 30 $4 >> $OUT/split.jsonl 2>> $OUT/split.err || { tail -20 $OUT/split.err; exit 1; }
  tail -1 $OUT/split.jsonl
done

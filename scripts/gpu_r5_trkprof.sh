#!/bin/bash
# Round 5: cProfile of the bench with the tracked leg (host build breakdown).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python3 -m cProfile -o $OUT/b.prof bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline --no-ba-scale --no-pcie-leg --no-tracked-ba > $OUT/b.json 2> $OUT/b.err || { tail -30 $OUT/b.err; exit 1; }
python3 - <<PY > $OUT/prof.txt
import pstats
s = pstats.Stats("$OUT/b.prof")
s.sort_stats("cumulative").print_callees("tracked_ba")
s.sort_stats("cumulative").print_callees("problems")
s.sort_stats("cumulative").print_callees(r"\bbuild\b")
s.sort_stats("tottime").print_stats(25)
PY
head -150 $OUT/prof.txt

#!/bin/bash
# Alternating knob re-check at the final default (6 query blocks, 16-window BA, ORB on 224 CUs):
# linearisation chunks per workgroup 4 / 5 (default) / 6 and 80 frame pairs per step.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/final_knobs"
mkdir -p "$OUT"
cd "$ROOT"
for r in 0 1 2; do
  for v in "def:" "cpw4:--chunks-per-wg 4" "cpw6:--chunks-per-wg 6" "b80:--batch 80"; do
    tag="${v%%:*}"; args="${v#*:}"
    timeout -k 10 150 python bench.py --no-cpu-baseline $args > "$OUT/${tag}_$r.json" 2> "$OUT/${tag}_$r.err" || exit $?
    echo "$tag $r $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value'])" "$OUT/${tag}_$r.json")" | tee -a "$OUT/summary.txt"
  done
done

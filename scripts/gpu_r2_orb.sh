#!/bin/bash
# ORB change check: bit-exact ORB / pipeline tests, phase profile, tracking bench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/orb_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_orb.py tests/test_pipeline.py tests/test_bow.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
timeout -k 10 200 python scripts/orb_prof.py > "$OUT/orb_prof.log" 2>&1 || exit 1
B="python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 30 --warmup 3"
for c in 216 192 176; do
  timeout -k 10 120 $B --orb-cus $c > "$OUT/trk_c$c.log" 2>&1 || exit 1
done
timeout -k 10 120 $B --no-orb-pipeline --ba-serial > "$OUT/trk_serial.log" 2>&1 || exit 1
echo done

#!/bin/bash
# PnP hypothesis-kernel A/B: geometry + pipeline GPU tests on the tree's
# library, then pnp_time.py under rocprofv3 kernel stats for the old / new
# variants (slam-1_amd/prof/libslam355_{jacold,jacnew}.so), then a bench line.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/pnp_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_geometry.py tests/test_pipeline.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
n=0
for v in jacold jacnew jacold jacnew; do
  n=$((n + 1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}_$n" -o run \
    -- python3 "$ROOT/scripts/pnp_time.py" $v > "$OUT/${v}_$n.log" 2>&1) || exit 1
done
find "$OUT" -name "*kernel_trace.csv" -delete
timeout -k 10 150 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
echo done

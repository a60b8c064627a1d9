#!/bin/bash
# k_pnp_hyp register cap A/B (prof/libslam355_wpe2.so: amdgpu_waves_per_eu(2),
# spills to scratch): geometry GPU tests on the variant, PnP alone under kernel
# stats, and the tracking bench alternating default / variant.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/wpe_$TAG"
V="$ROOT/slam-1_amd/prof/libslam355_wpe2.so"
mkdir -p "$OUT"
cd "$ROOT"
SLAM355_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_geometry.py -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_wpe2" -o run \
  -- python3 "$ROOT/scripts/pnp_time.py" wpe2 > "$OUT/pnp_wpe2.log" 2>&1) || exit 1
find "$OUT" -name "*kernel_trace.csv" -delete
for i in 1 2; do
  for v in def wpe2; do
    lib=""; [ "$v" = wpe2 ] && lib=$V
    SLAM355_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 16 --warmup 4 > "$OUT/${v}_$i.json" 2> "$OUT/${v}_$i.err" || exit 1
  done
done
echo done

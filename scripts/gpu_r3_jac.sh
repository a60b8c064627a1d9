#!/bin/bash
# LDS-resident Jacobi A/B: geometry / pipeline GPU tests (tree), PnP alone under
# kernel stats (tree vs prof/libslam355_jacold.so), tracking bench alternating.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/jac_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_geometry.py tests/test_pipeline.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
for v in tree jacold; do
  lib=""; [ "$v" != tree ] && lib="$ROOT/slam-1_amd/prof/libslam355_$v.so"
  (cd /tmp && export TMPDIR=/tmp && SLAM355_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/st_$v" -o run \
    -- python3 "$ROOT/scripts/pnp_time.py" > "$OUT/pnp_$v.log" 2>&1) || exit 1
done
find "$OUT" -name "*kernel_trace.csv" -delete
bash scripts/gpu_r3_ab.sh "jac_$TAG" jacold 3 || exit 1
echo done

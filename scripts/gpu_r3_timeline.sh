#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace, slam355 kernels only via
# scripts/trace_extract.py): the default tracking bench and the batched
# local-BA windows alone.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/tl_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trk" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 8 --warmup 2 > "$OUT/trk.log" 2>&1 || exit 1
python3 "$ROOT/scripts/trace_extract.py" "$OUT/trk" "$OUT/trk.csv" || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ba" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --ba-batch 8 --chunks-per-wg 8 --steps 20 --warmup 3 > "$OUT/ba.log" 2>&1 || exit 1
python3 "$ROOT/scripts/trace_extract.py" "$OUT/ba" "$OUT/ba.csv" || exit 1
find "$OUT" -name "*kernel_trace.csv" -delete
echo done

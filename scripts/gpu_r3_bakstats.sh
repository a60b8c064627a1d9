#!/bin/bash
# Kernel stats of the batched 8-window BA (cpw 8) for the tree's library and a
# variant (prof/libslam355_<v>.so), alternating: gpu_r3_bakstats.sh TAG VARIANT
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
VAR="$2"
OUT="$ROOT/gpurun_out/bakstats_$TAG"
mkdir -p "$OUT"
for i in 1 2; do
  for v in tree $VAR; do
    lib=""; [ "$v" != tree ] && lib="$ROOT/slam-1_amd/prof/libslam355_$v.so"
    (cd /tmp && export TMPDIR=/tmp && SLAM355_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}_$i" -o run \
      -- python3 "$ROOT/bench.py" --workload ba --ba-batch 8 --chunks-per-wg 8 --steps 30 --warmup 3 > "$OUT/${v}_$i.json" 2> "$OUT/${v}_$i.err") || exit 1
  done
done
find "$OUT" -name "*kernel_trace.csv" -delete
echo done

#!/bin/bash
# Round-2 experiment sweep: local BA alone (batched windows), tracking bench
# variants (serial BA, CU masks).  Every GPU step has its own time limit.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/sweep_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
B="python bench.py --no-cpu-baseline --no-ba-scale --steps 20 --warmup 3"
timeout -k 10 120 python bench.py --workload ba --ba-batch 4 --steps 50 --warmup 5 > "$OUT/ba_b4.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload ba --ba-batch 1 --steps 50 --warmup 5 > "$OUT/ba_b1.log" 2>&1 || exit 1
timeout -k 10 120 $B --ba-serial > "$OUT/trk_serial.log" 2>&1 || exit 1
for c in 240 224 208; do
  timeout -k 10 120 $B --track-cus $c > "$OUT/trk_cus$c.log" 2>&1 || exit 1
done
timeout -k 10 120 $B --priority equal > "$OUT/trk_prio_equal.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_b4" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --ba-batch 4 --steps 30 --warmup 3 > "$OUT/prof_b4.log" 2>&1 || exit 1
find "$OUT" -name "*kernel_trace.csv" -delete
echo done

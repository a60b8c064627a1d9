#!/bin/bash
# Round-2 profile of the default bench (tracking + batched local BA):
#   kernel-trace stats, HBM traffic (FETCH_SIZE / WRITE_SIZE passes), and SQ
#   counter passes (MFMA / VALU / LDS) -- each pass its own rocprofv3 run.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r2}"
shift || true
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --no-cpu-baseline --no-ba-scale $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
  -- python3 $B --steps 20 --warmup 5 > "$OUT/stats.log" 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$c" -o run \
    -- python3 $B --steps 3 --warmup 1 > "$OUT/$c.log" 2>&1 || exit 1
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" "$OUT/pmc_traffic.json" > /dev/null || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --output-format csv -d "$OUT/sq1" -o run -- python3 $B --steps 3 --warmup 1 > "$OUT/sq1.log" 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  --output-format csv -d "$OUT/sq2" -o run -- python3 $B --steps 3 --warmup 1 > "$OUT/sq2.log" 2>&1 || exit 1
python3 "$ROOT/scripts/pmc_counters.py" "$OUT/pmc_sq.json" "$OUT/sq1" "$OUT/sq2" > /dev/null || exit 1
# keep the summaries only (gpurun copies back <= 64 MiB)
find "$OUT" -name "*kernel_trace.csv" -delete
find "$OUT" -name "*counter_collection.csv" -delete
echo done

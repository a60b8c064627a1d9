#!/bin/bash
# k_lin_mfma change check: BA parity tests, batched-window timing, phase split, LDS counters
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lin_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_ba.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload ba --ba-batch 4 --steps 50 --warmup 5 > "$OUT/ba_b4.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload ba --ba-batch 1 --steps 50 --warmup 5 > "$OUT/ba_b1.log" 2>&1 || exit 1
timeout -k 10 120 python scripts/linm_prof.py 4 1 > "$OUT/linm.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d "$OUT/sq" -o run -- python3 "$ROOT/bench.py" --workload ba --ba-batch 4 --steps 10 --warmup 2 > "$OUT/sq.log" 2>&1 || exit 1
python3 "$ROOT/scripts/pmc_counters.py" "$OUT/pmc_sq.json" "$OUT/sq" > /dev/null || exit 1
find "$OUT" -name "*counter_collection.csv" -delete
find "$OUT" -name "*kernel_trace.csv" -delete
echo done

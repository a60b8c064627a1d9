#!/bin/bash
# ORB change check (round 3): bit-exact ORB GPU tests, per-phase cycle split,
# SQ counters of k_orb_tile (LDS instructions / bank conflicts / waits), and a
# tracking bench line.  Libraries are built beforehand on the CPU side.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/orb_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_orb.py tests/test_pipeline.py tests/test_bow.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
timeout -k 10 200 python scripts/orb_prof.py > "$OUT/orb_prof.log" 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d "$OUT/sq1" -o p1 --output-format csv -- python3 "$ROOT/scripts/orb_run.py" > "$OUT/sq1.log" 2>&1) || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH \
  -d "$OUT/sq2" -o p2 --output-format csv -- python3 "$ROOT/scripts/orb_run.py" > "$OUT/sq2.log" 2>&1) || exit 1
python scripts/pmc_counters.py "$OUT/orb_sq.json" "$OUT/sq1" "$OUT/sq2" > /dev/null || exit 1
find "$OUT" -name "*.csv" -delete
timeout -k 10 150 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 30 --warmup 3 > "$OUT/bench.log" 2>&1 || exit 1
echo done

#!/bin/bash
# PMC counter passes on the BA LM kernels (one pass per counter group).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_${1:-ba}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/scripts/ba_iter_only.py" > "$OUT/p1.log" 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_FLAT --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/scripts/ba_iter_only.py" > "$OUT/p2.log" 2>&1
echo "exit=$?"

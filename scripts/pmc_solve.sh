#!/bin/bash
# PMC counter passes on the BA LM kernels (one pass per counter group).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_${1:-solve}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/scripts/ba_iter_only.py" > "$OUT/p1.log" 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_IFETCH_LEVEL --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/scripts/ba_iter_only.py" > "$OUT/p2.log" 2>&1
echo "exit=$?"

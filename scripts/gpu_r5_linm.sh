#!/bin/bash
# Round 5: k_lin_mfma phase split (profiling build) for the bench's 16-window
# C3 launch set at 16 / 8 chunks per workgroup and for 1 chunk per workgroup.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
for cfg in "16 16" "16 8" "1 1"; do
  set -- $cfg
  timeout -k 10 120 python3 scripts/linm_prof.py $1 $2 > $OUT/linm_$1_$2.txt 2>&1 || { tail $OUT/linm_$1_$2.txt; exit 1; }
  echo "== $1 windows, $2 chunks/WG"; grep -v amdgpu.ids $OUT/linm_$1_$2.txt | tail -12
done

#!/bin/bash
# Session-2 fourth pass: the whole GPU suite + smoke at the current library, then a
# 3-way tracking A/B of the matcher (current: register nibbles + XCD order;
# lutxcd: LDS tables + XCD order; mxbase: the round-4 HEAD matcher).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/r4s2d; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash scripts/gpu_r4_abn.sh r4s2d_tr 4 def lutxcd mxbase || exit 1
echo ok

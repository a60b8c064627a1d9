#!/bin/bash
# Rehearsal of the driver's N>1 bench path with 2 ranks on one GPU (gloo stands in
# for RCCL, which refuses two ranks per device), plus smoke().
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/multirank_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
SLAM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench2.log" 2>&1 || exit 1
echo done

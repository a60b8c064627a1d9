#!/bin/bash
# Rehearsal of the driver's multi-rank command on the one-GPU box: 2 ranks
# over gloo sharing the GPU (a functional check of the N > 1 path: frame-pair
# shards, the pose-chain all-gather, the sharded C4 leg; not a scaling datum).
#   scripts/gpu_r6_g2.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
export SLAM_DIST_BACKEND=gloo
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 6 --warmup 2 > $OUT/g2.json 2> $OUT/g2.err || { tail -30 $OUT/g2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/g2.json').read().strip().splitlines()[-1]);print(round(d['value']), d['n_gpus'], d['config'].get('parallelism'), 'sharded', d.get('local_ba_sharded', {}).get('iters_per_s'), d.get('local_ba_sharded', {}).get('ranks'))"

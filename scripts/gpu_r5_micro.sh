#!/bin/bash
# Round 5: f64 / DPP instruction costs (micro), then the whole GPU suite and the
# driver's bench command at the current tree.   scripts/gpu_r5_micro.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r5_micro}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 60 ./scripts/micro/f64_dpp > $OUT/f64_dpp.txt 2>&1 || { cat $OUT/f64_dpp.txt; exit 1; }
cat $OUT/f64_dpp.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print('bench', round(d['value']), round(d['ms_per_step'],3), round(d['local_ba_sharded']['iters_per_s']), d['stage_ms_per_step'])"

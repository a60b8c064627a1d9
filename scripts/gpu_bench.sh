#!/bin/bash
# Round-4 bench pass: the driver's exact command (--steps 20 --warmup 5) N times,
# plus optional extra argument sets, each under its own time limit, chained with &&.
#   scripts/gpu_bench.sh TAG N [extra bench args...]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$1"
mkdir -p "$OUT"
cd "$ROOT"
N="${2:-2}"
shift 2 || true
for i in $(seq 1 "$N"); do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit $?
  echo "bench $i: $(python3 -c "import json,sys;d=json.load(open('$OUT/bench_$i.json'));print(round(d['value']),round(d['ms_per_step'],3),round(d['host_issue_ms_per_step'],3))")"
done

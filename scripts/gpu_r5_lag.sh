#!/bin/bash
# Round 5: tracked-leg lag A/B (alternating runs of the driver's bench command).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2; do
  for lag in 2 3; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ba-scale --no-pcie-leg --tracked-lag $lag > $OUT/b_${lag}_$i.json 2> $OUT/b_${lag}_$i.err || { tail -30 $OUT/b_${lag}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${lag}_$i.json'));t=d['tracked_source'];print('lag', $lag, round(d['value']), round(t['frames_per_s']), round(t['host_build_ms_per_step'],2), t['local_ba_ms_per_step'])"
  done
done

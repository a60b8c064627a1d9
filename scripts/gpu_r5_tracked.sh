#!/bin/bash
# Round 5: the tracked-source leg of the tracking bench (WindowMapper + lag-1
# host build) -- a short run, then the driver's command.  scripts/gpu_r5_tracked.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 6 --warmup 2 --no-cpu-baseline --no-ba-scale --no-pcie-leg --no-tracked-ba > $OUT/short.json 2> $OUT/short.err || { tail -30 $OUT/short.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/short.json'));print(round(d['value']), json.dumps(d.get('tracked_source'))[:1500])"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));t=d['tracked_source'];print(round(d['value']), round(t['frames_per_s']), 'build/step', round(t['host_build_ms_per_step'],3), 'per window', round(t['host_build_ms_per_window'],4), 'wait', round(t['host_wait_ms_per_step'],3), t['window_cams_pts_obs_mean'], t['lin_modes'], t['local_ba_ms_per_step'])"

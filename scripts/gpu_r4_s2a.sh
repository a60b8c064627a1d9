#!/bin/bash
# Round-4 session-2 first pass: matcher A/B (in-register nibbles + XCD order vs
# HEAD), then scripts/gpu_r4_s2b.sh against the 2x2-pivot factor alone, and a
# C4 line of the round-4 HEAD library.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
bash scripts/gpu_r4_mx.sh r4s2_mx 2 slam-1_amd/prof/libslam355_mxbase.so || exit 1
bash scripts/gpu_r4_s2b.sh r4s2_ba slam-1_amd/prof/libslam355_bafac.so || exit 1
for i in 1 2; do
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_babase.so timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > gpurun_out/r4s2_ba/c4_base_$i.json || exit 1
  python3 -c "import json;a=json.load(open('gpurun_out/r4s2_ba/c4_base_$i.json'));print('base', $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1))"
done
echo ok

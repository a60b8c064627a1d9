#!/bin/bash
# Round-2 end-of-session evidence at HEAD: all GPU tests, the default-bench
# profile (kernel stats, PMC traffic, SQ counters), ORB phase split, dataflow
# solve phases, C4 / C5 bench lines + kernel stats.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r2}"
OUT="$ROOT/gpurun_out/final_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
bash scripts/gpu_tests.sh "$TAG" || exit 1
timeout -k 10 200 python scripts/orb_prof.py > "$OUT/orb_prof.log" 2>&1 || exit 1
SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_flowprof.so timeout -k 10 200 python scripts/flow_prof.py > "$OUT/flow_prof.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload ba --c4 --steps 50 --warmup 5 > "$OUT/ba_c4.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload ba --c5 --steps 20 --warmup 3 > "$OUT/ba_c5.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload ba --ba-batch 8 --steps 200 --warmup 20 > "$OUT/ba_b8.log" 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --c4 --steps 20 --warmup 3 > "$OUT/ba_c4_prof.log" 2>&1) || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --c5 --steps 5 --warmup 2 > "$OUT/ba_c5_prof.log" 2>&1) || exit 1
find "$OUT" -name "*kernel_trace.csv" -delete
bash scripts/gpu_profile_r2.sh "$TAG" || exit 1
echo done

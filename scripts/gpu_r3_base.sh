#!/bin/bash
# Round-3 evidence at HEAD: every GPU test (one pytest process), smoke, the
# default bench line (driver command form), the profile passes of the default
# bench (kernel stats, FETCH/WRITE PMC, SQ counters), and kernel stats of the
# C4 / C5 LM iterations on one GPU (the Amdahl table of DESIGN.md §7).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
cd "$ROOT"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh "$TAG" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 || exit 1
timeout -k 10 400 python bench.py > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err" || exit 1
bash scripts/gpu_profile.sh "$TAG" || exit 1
for c in c4 c5; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG/$c" -o run \
    -- python3 "$ROOT/bench.py" --workload ba --$c --steps 20 --warmup 3 > "$ROOT/gpurun_out/prof_$TAG/$c.json" 2> "$ROOT/gpurun_out/prof_$TAG/$c.err") || exit 1
done
find "$ROOT/gpurun_out/prof_$TAG" -name "*kernel_trace.csv" -delete
echo done

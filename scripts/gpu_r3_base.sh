#!/bin/bash
# Round-3 evidence at HEAD: every GPU test (one pytest process), smoke, the
# default bench line (driver command form), then the profile passes of the
# default bench (kernel stats, FETCH/WRITE PMC, SQ counters).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
cd "$ROOT"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh "$TAG" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 || exit 1
timeout -k 10 400 python bench.py > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err" || exit 1
bash scripts/gpu_profile_r2.sh "$TAG" || exit 1
echo done

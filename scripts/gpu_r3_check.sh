#!/bin/bash
# Round-3 change check: every GPU test (one pytest process), smoke, then the
# ORB evidence script.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
cd "$ROOT"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh "$TAG" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 || exit 1
bash scripts/gpu_r3_orb.sh "$TAG" || exit 1
echo done

#!/bin/bash
# GPU parity tests only (one pytest process), with a time limit.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOT/gpurun_out"
cd "$ROOT"
TAG="${1:-r1}"
shift || true
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread "$@" \
  > "gpurun_out/pytest_gpu_$TAG.log" 2>&1
rc=$?
tail -5 "gpurun_out/pytest_gpu_$TAG.log"
exit $rc

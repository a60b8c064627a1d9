#!/bin/bash
# Tracking-stream CU budget sweep (bench tracking workload).
set -e
cd "$GRAFT_REPO_ROOT"
for c in "$@"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-ba-scale --track-cus $c > gpurun_out/sweep_$c.log 2>&1
done

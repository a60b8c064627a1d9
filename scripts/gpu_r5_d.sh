#!/bin/bash
# Round 5 pass D: BA / dist GPU tests at HEAD (single-instance tile factor),
# flow timeline, C4 / C5 vs round-4 ba.hip with final costs, ORB phase split
# (batched group vs per-level).   scripts/gpu_r5_d.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
bash scripts/gpu_r5_c.sh $TAG || exit 1
for v in bat nobat; do
  if [ $v = nobat ]; then export SLAM_ORB_NOBATCH=1; else unset SLAM_ORB_NOBATCH; fi
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_orbprof.so timeout -k 10 120 python3 scripts/orb_prof.py > $OUT/orb_phases_$v.txt 2>&1 || { tail $OUT/orb_phases_$v.txt; exit 1; }
  echo $v; cat $OUT/orb_phases_$v.txt
done
unset SLAM_ORB_NOBATCH

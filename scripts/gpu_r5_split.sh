#!/bin/bash
# Round 5: measured per-rank kernel split of the sharded C4 / C5 LM iteration
# (scripts/shard_split.py under rocprofv3 --stats, one run per world size /
# rank).   scripts/gpu_r5_split.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for cfg in "C4 1 0" "C4 2 0" "C4 2 1" "C4 4 0" "C4 4 3" "C4 8 0" "C4 8 7" "C5 1 0" "C5 8 0" "C5 8 7"; do
  set -- $cfg
  d=$OUT/${1}_w${2}_r${3}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 $ROOT/scripts/shard_split.py $1 $2 $3 20 > $d.json 2> $d.err || { tail -20 $d.err; exit 1; }
  find $d -name "*kernel_trace.csv" -delete
  tail -1 $d.json
done

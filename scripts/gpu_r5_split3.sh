#!/bin/bash
# Round 5: per-rank split at HEAD (shard chunk rule, empty-block assembly exit,
# flow changes) under rocprofv3, C4 / C5 at W = 1 / 8.   scripts/gpu_r5_split3.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu -k "tiled or flow or c4 or c5 or distributed or capi or folded or shard" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
for cfg in "C4 1 0" "C4 2 0" "C4 4 0" "C4 8 0" "C4 8 7" "C5 1 0" "C5 8 0" "C5 8 7"; do
  set -- $cfg
  d=$OUT/${1}_w${2}_r${3}
  cpw=""
  if [ $2 -gt 1 ]; then cpw=$(python3 -c "import sys;sys.path[:0]=['$ROOT/slam-1_amd'];from slam355.dist import shard_chunks_per_wg as f;n=(300000 if '$1'=='C4' else 1200000)//$2;v=f(n);print(v if v else 0)"); fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 $ROOT/scripts/shard_split.py $1 $2 $3 20 $cpw > $d.json 2> $d.err || { tail -20 $d.err; exit 1; }
  find $d -name "*kernel_trace.csv" -delete
  tail -1 $d.json
done

#!/bin/bash
# Round 6: the per-rank split of the sharded LM iteration (DESIGN §7's Amdahl
# table) -- C4 at W = 1 / 2 / 4 / 8 (rank 0, and rank 7 at W = 8), C5 at W = 1
# / 8 (ranks 0 and 7) -- each shard alone on this GPU under rocprofv3 kernel
# stats, then the dataflow solve's per-column timeline (-DSLAM_FLOW_PROFILE
# build, scripts/flow_prof.py).   scripts/gpu_r6_split.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT/split"
cd /tmp && export TMPDIR=/tmp
for cfg in "C4 1 0" "C4 2 0" "C4 4 0" "C4 8 0" "C4 8 7" "C5 1 0" "C5 8 0" "C5 8 7"; do
  set -- $cfg
  d=$OUT/split/${1}_w${2}_r${3}
  cpw=""
  if [ $2 -gt 1 ]; then cpw=$(python3 -c "import sys;sys.path[:0]=['$ROOT/slam-1_amd'];from slam355.dist import shard_chunks_per_wg as f;n=(300000 if '$1'=='C4' else 1200000)//$2;v=f(n);print(v if v else 0)"); fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 $ROOT/scripts/shard_split.py $1 $2 $3 20 $cpw > $d.json 2> $d.err || { tail -20 $d.err; exit 1; }
  find $d -name "*kernel_trace.csv" -delete
done
python3 $ROOT/scripts/split_summary.py $OUT/split > $OUT/split/summary.json || exit 1
python3 -c "
import json;d=json.load(open('$OUT/split/summary.json'))
for k,v in d.items(): print(k, 'div', v['divided'], 'rep', v['replicated'], 'wall', v.get('wall_us_per_iter'))"
cd "$ROOT"
if [ -f slam-1_amd/prof/libslam355_fp.so ]; then
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_fp.so timeout -k 10 200 python3 scripts/flow_prof.py $OUT/flow > $OUT/flow_phases.log 2>&1 || exit 1
  grep "^C4\|^C5" $OUT/flow_phases.log
fi

#!/bin/bash
# Round 5 pass A: pose-graph TRF (register-resident) + the 16x16 factor with
# L's columns in LDS.  Tests (pose graph, folded batch, tiled / flow BA), the
# pose-graph A/B vs the round-4 kernel, per-column flow timelines (HEAD and
# round-4 ba.hip), C4 / C5 A/B (HEAD, round-4 ba.hip, HEAD without the LDS columns).   scripts/gpu_r5_a.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_posegraph.py tests/test_ba.py -x -v -m gpu -k "trf or posegraph or objective or folded or tiled or flow or c4 or c5" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for k in reg lds reg lds; do
  if [ $k = lds ]; then export SLAM_CHAIN_TRF=lds; else unset SLAM_CHAIN_TRF; fi
  timeout -k 10 120 python3 scripts/pg_time.py 500 5 >> "$OUT/pg_time.jsonl" 2>> "$OUT/pg_time.err" || { tail -20 "$OUT/pg_time.err"; exit 1; }
done
unset SLAM_CHAIN_TRF
cat "$OUT/pg_time.jsonl"
for v in flowprof1 flowprofr4; do
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -k 10 200 python3 scripts/flow_prof.py > $OUT/flow_$v.log 2>&1 || { tail $OUT/flow_$v.log; exit 1; }
  echo $v; grep -E "^C|factor of" $OUT/flow_$v.log
done
for i in 1 2; do
  for v in def r4 faccol0; do
    if [ $v = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_${v}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_${v}_$i.json || exit 1
    python3 -c "import json;a=json.load(open('$OUT/c4_${v}_$i.json'));b=json.load(open('$OUT/c5_${v}_$i.json'));print('$v', $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1), '| C5', round(b['value']), round(b['ms_per_step']*1e3,1), 'pg', round(b['pose_graph']['ms_per_solve'],2))"
  done
done

#!/bin/bash
# Round 5 pass B: whole GPU suite + smoke, the driver's bench command, and
# rocprofv3 kernel stats of the 2-rank gloo C4 rehearsal on one GPU (per-rank
# kernel split of the sharded LM iteration).   scripts/gpu_r5_b.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']),round(d['ms_per_step'],3),d['roofline']['stage'],round(d['roofline']['frac'],4),d['stage_ms_per_step'])"
export SLAM_DIST_BACKEND=gloo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4_g2 -o run -- python3 $ROOT/bench.py --gpus 2 --workload ba --c4 --steps 20 --warmup 3 > $OUT/c4_g2.json 2> $OUT/c4_g2.err || { tail -20 $OUT/c4_g2.err; exit 1; }
find $OUT -name "*kernel_trace.csv" -delete
ls -R $OUT/prof_c4_g2 | head -20
cat $OUT/c4_g2.json | tail -1

#!/bin/bash
# Evidence set of a round: GPU tests + smoke, the driver's bench command x3,
# C4 / C5 / batched-BA / matcher lines, then the profile passes of the default
# bench (kernel stats, FETCH_SIZE / WRITE_SIZE, two SQ passes).  Each GPU step
# has its own time limit; the steps are chained with && (a failure ends the call).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r5_final}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 1
  python3 -c "import json;d=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1]);print('bench', $i, round(d['value']), round(d['ms_per_step'],3), round(d['host_issue_ms_per_step'],3), round(d['pcie_inclusive']['frames_per_s']), round(d['local_ba_sharded']['iters_per_s']))"
done
timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/ba_c4.json || exit 1
timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/ba_c5.json || exit 1
timeout -k 10 120 python3 bench.py --workload ba --ba-batch 16 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/ba_b16.json || exit 1
timeout -k 10 120 python3 bench.py --workload ba --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/ba_c3.json || exit 1
timeout -k 10 120 python3 bench.py --workload matcher --steps 20 --warmup 3 2>/dev/null | tail -1 > $OUT/matcher_b32.json || exit 1
python3 -c "
import json
for f in ('ba_c4','ba_c5','ba_b16','ba_c3','matcher_b32'):
    d=json.load(open('$OUT/'+f+'.json')); print(f, round(d['value'],1), d['unit'], round(d['ms_per_step']*1e3,1))
"
bash scripts/gpu_profile.sh $TAG --no-pcie-leg --no-tracked-ba --no-tracked-leg || exit 1
echo done

#!/bin/bash
# Round 5: linearisation chunks per workgroup of the bench's C3 windows
# (partial-row traffic vs parallelism): batched C3 alone and the driver's bench,
# alternating, then FETCH/WRITE of the batched C3 launch set at each setting.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2; do
  for c in 8 16 32; do
    timeout -k 10 120 python3 bench.py --workload ba --ba-batch 16 --chunks-per-wg $c --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/b16_${c}_$i.json || exit 1
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ba-scale --no-tracked-ba --no-pcie-leg --no-tracked-leg --chunks-per-wg $c > $OUT/bench_${c}_$i.json 2> $OUT/bench_${c}_$i.err || { tail -20 $OUT/bench_${c}_$i.err; exit 1; }
    python3 -c "import json;a=json.load(open('$OUT/b16_${c}_$i.json'));d=json.load(open('$OUT/bench_${c}_$i.json'));print('cpw', $c, $i, 'B16', round(a['value']), round(a['ms_per_step']*1e3,1), '| bench', round(d['value']), round(d['ms_per_step'],3), round(d['roofline_stages']['local_ba']['ms_per_iter'],4), round(d['stage_ms_per_step']['local_ba'],3))"
  done
done
cd /tmp && export TMPDIR=/tmp
for c in 8 16 32; do
  for k in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $k --output-format csv -d $OUT/pmc_$c/$k -o run -- python3 $ROOT/bench.py --workload ba --ba-batch 16 --chunks-per-wg $c --steps 3 --warmup 1 > /dev/null 2>&1 || exit 1
  done
  python3 $ROOT/scripts/pmc_summary.py $OUT/pmc_$c $OUT/pmc_$c.json | grep -E "lin_mfma|k_assemble|solve_blk|back_trial" || true
done
find $OUT -name "*counter_collection.csv" -size +20M -delete
echo done

#!/bin/bash
# Round 5: PnP change vs the HEAD geometry.hip (prof/libslam355_geohead.so):
# geometry / pipeline GPU tests, PnP alone under kernel stats (both builds),
# the bench alternating, SQ counters of the hypothesis LM.   scripts/gpu_r5_pnp.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
VAR=$ROOT/slam-1_amd/prof/libslam355_geohead.so
timeout -k 10 500 python -u -m pytest tests/test_geometry.py tests/test_pipeline.py -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
for v in new head; do
  if [ $v = head ]; then export SLAM355_LIB=$VAR; else unset SLAM355_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pnp_$v -o run -- python3 $ROOT/scripts/pnp_time.py > $OUT/pnp_$v.txt 2>&1 || { tail $OUT/pnp_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/pnp_$v.txt)"; grep -h "k_pnp" $OUT/pnp_$v/run_kernel_stats.csv | cut -d, -f1-4
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/sq_$v -o run -- python3 $ROOT/scripts/pnp_time.py > /dev/null 2>&1 || exit 1
done
unset SLAM355_LIB
find $OUT -name "*kernel_trace.csv" -delete
cd $ROOT
python3 - <<PY
import csv, collections
for v in ("new", "head"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open("$OUT/sq_%s/run_counter_collection.csv" % v)):
        if "k_pnp_hyp_lm" in r["Kernel_Name"]:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    m = {c: sum(x.values()) / len(x) for c, x in acc.items()}
    print(v, "k_pnp_hyp_lm conflict/LDS %.2f" % (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]), {c: round(x) for c, x in m.items()})
PY
find $OUT -name "*counter_collection.csv" -delete
for i in 1 2; do
  for v in new head; do
    if [ $v = head ]; then export SLAM355_LIB=$VAR; else unset SLAM355_LIB; fi
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ba-scale --no-tracked-ba --no-pcie-leg --no-tracked-leg > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { tail -20 $OUT/bench_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_${v}_$i.json'));print('$v', $i, round(d['value']),round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['stage_ms_per_step'].items()})"
  done
done
unset SLAM355_LIB

#!/bin/bash
# Matcher A/B: the default library (A) vs a variant (B, SLAM355_LIB):
# matcher GPU tests on A, the C2 micro-bench and the tracking bench alternating,
# then per library one kernel-trace stats pass and one FETCH_SIZE pass of the
# tracking bench (knn2_mx_kernel's in-pipeline duration and HBM bytes).
#   scripts/gpu_ab_matcher.sh TAG N VARIANT_SO ['pytest -k expr']
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; VAR=$3; K=${4:-"knn or match or hamming or tracker or pipeline"}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
sel() { if [ $1 = B ]; then export SLAM355_LIB=$ROOT/$VAR; else unset SLAM355_LIB; fi; }
for i in $(seq 1 $N); do
  for v in A B; do
    sel $v
    timeout -k 10 120 python3 bench.py --workload matcher --steps 20 --warmup 3 2>/dev/null | tail -1 > $OUT/mx_${v}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tracked-ba --no-ba-scale --no-pcie-leg 2>/dev/null | tail -1 > $OUT/tr_${v}_$i.json || exit 1
    python3 -c "
import json
m=json.load(open('$OUT/mx_${v}_$i.json')); d=json.load(open('$OUT/tr_${v}_$i.json')); s=d['stage_ms_per_step']
print('$v', $i, 'micro', round(m['value'],1), m['unit'], '| tracking', round(d['value']), round(d['ms_per_step'],3), 'stereo', round(s.get('stereo_knn2', -1),3), 'mx launch', round(d['roofline_stages']['matcher']['ms_per_launch'],3))"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  sel $v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$v -o run \
    -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tracked-ba --no-ba-scale --no-pcie-leg > $OUT/stats_$v.log 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$v -o run \
    -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-tracked-ba --no-ba-scale --no-pcie-leg > $OUT/fetch_$v.log 2>&1 || exit 1
  python3 - "$OUT" "$v" <<'EOF'
import csv, glob, sys
out, v = sys.argv[1], sys.argv[2]
st = glob.glob(f"{out}/stats_{v}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(st)):
    if "knn2" in r["Name"] or "orb_tile" in r["Name"] or "pnp_hyp" in r["Name"]:
        print(v, r["Name"][:40], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
cc = glob.glob(f"{out}/fetch_{v}/**/*counter_collection.csv", recursive=True)[0]
acc = {}
for r in csv.DictReader(open(cc)):
    if "knn2" in r["Kernel_Name"]:
        acc.setdefault(r["Dispatch_Id"], 0.0)
        acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
vals = list(acc.values())
print(v, "knn2 FETCH_SIZE per dispatch (KB, mean)", round(sum(vals) / max(len(vals), 1), 1), "n", len(vals))
EOF
done
find $OUT -name "*kernel_trace.csv" -delete
find $OUT -name "*counter_collection.csv" -delete -o -name "*agent_info.csv" -delete
echo done

#!/bin/bash
# Kernel-trace + stats of the default tracking bench (the driver's step counts).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r4_prof}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tracked-ba --no-ba-scale --no-pcie-leg > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:22]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} {float(r['TotalDurationNs'])/tot*100:6.1f}%")
PY

#!/bin/bash
# PnP change check: the geometry / pipeline GPU parity tests, then the tracking
# bench A/B against an older build.  scripts/gpu_r4_pnp.sh TAG OLD_SO [N_AB]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; OLD=$2; N=${3:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_geometry.py tests/test_pipeline.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_pnp.log 2>&1 || { tail -30 $OUT/pytest_pnp.log; exit 1; }
tail -1 $OUT/pytest_pnp.log
bash scripts/gpu_r4_ab_lib.sh $TAG/ab $N $OLD || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/stats" -o run \
  -- python3 $ROOT/bench.py --no-cpu-baseline --no-ba-scale --no-pcie-leg --no-tracked-ba --steps 20 --warmup 5 > "$ROOT/$OUT/stats.log" 2>&1 || exit 1
python3 - "$ROOT/$OUT/stats/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("k_pnp", "k_orb_tile", "knn2_mx", "k_fm_hyp", "k_lin_mfma")):
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
find "$ROOT/$OUT" -name "*kernel_trace.csv" -delete

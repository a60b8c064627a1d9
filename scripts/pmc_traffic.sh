#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters (MI355X_MICROARCH.md,
# HBM / rocprofv3 sections): FETCH_SIZE and WRITE_SIZE in separate passes
# (they do not fit one TCC pass), kernel trace only, then a per-kernel summary
# (FETCH_SIZE doubled for gfx950, kB -> bytes) in gpurun_out/pmc_traffic_<tag>.json
# (commit it as profiles/pmc_traffic.json: bench.py reports it as roofline.traffic).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r1}"
shift || true
OUT="$ROOT/gpurun_out/pmc_traffic_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$c" -o run \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$OUT/$c.log" 2>&1 || exit $?
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" "$ROOT/gpurun_out/pmc_traffic_${TAG}.json"

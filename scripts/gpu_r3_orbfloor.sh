#!/bin/bash
# ORB LDS floor sweep (one ORB workgroup per CU, room for a local-BA
# linearisation workgroup beside it) x ORB CU mask, tracking bench.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/orbfloor_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for cfg in "0 216" "82432 256" "82432 216" "0 216" "82432 256" "82432 240"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --orb-lds-floor $1 --orb-cus $2 --steps 20 --warmup 4 > "$OUT/f$1_c$2.json" 2> "$OUT/f$1_c$2.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/f$1_c$2.json')); d['floor']=$1; d['cus']=$2; print(json.dumps(d))" >> "$OUT/all.jsonl" || exit 1
done
echo done

#!/bin/bash
# VALU / SALU / LDS instructions of k_orb_tile by phase: one SQ pass per
# SLAM_ORB_CUT build (every level stops after phase k) and one of the default.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r4_orbcut"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in orbcut1 orbcut2 orbcut3 orbcut6 orbcut7 orbcut8 default; do
  if [ $v = default ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD \
    --output-format csv -d "$OUT/$v" -o run -- python3 $ROOT/scripts/orb_time.py > "$OUT/$v.log" 2>&1 || exit 1
  tail -1 "$OUT/$v.log"
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in ["orbcut1", "orbcut2", "orbcut3", "orbcut6", "orbcut7", "orbcut8", "default"]:
    f = glob.glob(os.path.join(out, v, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(float); n = collections.Counter()
    for fn in f:
        for r in csv.DictReader(open(fn)):
            if "k_orb_tile" not in r["Kernel_Name"]: continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    disp = max(1, n["SQ_INSTS_VALU"] // max(1, len(set()))) if False else None
    print(v, {k: round(acc[k] / 1e6, 1) for k in sorted(acc)}, "rows", dict(n))
PY
find "$OUT" -name "*counter_collection.csv" -size +5M -delete

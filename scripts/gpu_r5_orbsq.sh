#!/bin/bash
# Round 5: ORB LDS bank conflicts per phase -- SQ counters of the per-level
# ORB (SLAM_ORB_NOBATCH=1) cut after each phase (prof/libslam355_orbcut{k}.so,
# -DSLAM_ORB_CUT=k), plus the full kernel per-level and batched; one
# rocprofv3 --pmc pass per build (scripts/orb_time.py, 33 launches).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
C="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
run() {  # name lib nobatch
  if [ "$3" = 1 ]; then export SLAM_ORB_NOBATCH=1; else unset SLAM_ORB_NOBATCH; fi
  SLAM355_LIB=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/$1 -o run -- python3 $ROOT/scripts/orb_time.py > $OUT/$1.log 2>&1 || return 1
}
for k in 1 2 3 6 7 8; do run cut$k $ROOT/slam-1_amd/prof/libslam355_orbcut$k.so 1 || exit 1; done
run full_nobat $ROOT/slam-1_amd/slam355/libslam355.so 1 || exit 1
run full_bat $ROOT/slam-1_amd/slam355/libslam355.so 0 || exit 1
unset SLAM_ORB_NOBATCH
python3 - <<PY > $OUT/summary.txt
import csv, collections
names = ["cut1", "cut2", "cut3", "cut6", "cut7", "cut8", "full_nobat", "full_bat"]
for n in names:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    with open("$OUT/%s/run_counter_collection.csv" % n) as f:
        for r in csv.DictReader(f):
            if "k_orb_tile" not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    m = {c: sum(v.values()) / len(v) for c, v in acc.items()}
    print(n, {c: round(v) for c, v in sorted(m.items())},
          "conflict/LDS %.3f" % (m["SQ_LDS_BANK_CONFLICT"] / max(1, m["SQ_INSTS_LDS"])),
          "wait/wave %.3f" % (m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]))
PY
cat $OUT/summary.txt
find $OUT -name "*counter_collection.csv" -delete
find $OUT -name "*kernel_trace.csv" -delete

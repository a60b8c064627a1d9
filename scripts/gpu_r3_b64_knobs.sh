#!/bin/bash
# Batch-64 default bench against one-knob variants (ORB CU mask, linearisation
# chunks per workgroup), alternating in separate processes:
#   gpu_r3_b64_knobs.sh TAG [ROUNDS] [SET]
# SET "mask" (default): ORB CU mask 200 / 232 / all and 5 chunks per WG;
# SET "cpw": 3 / 4 / 5 / 6 chunks per linearisation WG against the default;
# SET "misc": stream priority, BA windows over two streams, ORB mask 208;
# SET "trk": tracking-tail CU mask 240 / 248 (the last CUs left to local BA);
# SET "mb16": chunks per WG 6 / 8 and ORB mask 208 / 224 with 16-window launches;
# SET "orbmask": ORB mask 224 / 232 / 240 with 16-window launches;
# SET "valu": the integer-VALU kNN-2 kernel in the pipeline;
# SET "prio": stream priorities equal / tracking-high at the final default.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
N="${2:-2}"
SET="${3:-mask}"
if [ "$SET" = prio ]; then
  KNOBS=("default::" "prio_equal::--priority equal" "cpw4::--chunks-per-wg 4")
elif [ "$SET" = valu ]; then
  KNOBS=("default::" "valu::--valu")
elif [ "$SET" = orbmask ]; then
  KNOBS=("default::" "orb224::--orb-cus 224" "orb232::--orb-cus 232" "orb240::--orb-cus 240")
elif [ "$SET" = mb16 ]; then
  KNOBS=("default::" "cpw6::--chunks-per-wg 6" "cpw8::--chunks-per-wg 8" "orb208::--orb-cus 208" "orb224::--orb-cus 224")
elif [ "$SET" = trk ]; then
  KNOBS=("default::" "trk248::--track-cus 248" "trk240::--track-cus 240")
elif [ "$SET" = misc ]; then
  KNOBS=("default::" "prio_equal::--priority equal" "prio_track::--priority track" "bastreams2::--ba-streams 2" "orb208::--orb-cus 208")
elif [ "$SET" = cpw ]; then
  KNOBS=("default::" "cpw3::--chunks-per-wg 3" "cpw4::--chunks-per-wg 4" "cpw5::--chunks-per-wg 5" "cpw6::--chunks-per-wg 6")
else
  KNOBS=("default::" "orb200::--orb-cus 200" "orb232::--orb-cus 232" "orball::--orb-cus 0" "cpw5::--chunks-per-wg 5")
fi
OUT="$ROOT/gpurun_out/b64knobs_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=("${KNOBS[@]}")
for i in $(seq 1 $N); do
  for v in "${V[@]}"; do
    name="${v%%::*}"; flags="${v#*::}"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba $flags > "$OUT/${name}_$i.json" 2> "$OUT/${name}_$i.err" || exit 1
  done
done
echo done

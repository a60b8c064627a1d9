#!/bin/bash
# Round 6: which stream gets the high HIP stream priority in the driver's bench
# (bench.py --priority ba | track | equal), two alternating rounds.
set -o pipefail
mkdir -p gpurun_out/prio
for i in 1 2; do
  for pr in ba track equal; do
    timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie-leg --no-tracked-leg --priority $pr > gpurun_out/prio/${pr}_$i.json 2> gpurun_out/prio/${pr}_$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/prio/${pr}_$i.json').read().strip().splitlines()[-1]);print('$pr', $i, round(d['value']), round(d['ms_per_step'],3), {k:round(v,2) for k,v in d['stage_ms_per_step'].items()})"
  done
done

#!/bin/bash
# bench.py --ba-source tracked beside the default line (round 5)
set -e
OUT=gpurun_out/r5_basrc; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/default.json 2> $OUT/default.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --ba-source tracked > $OUT/tracked.json 2> $OUT/tracked.err
tail -n1 $OUT/default.json; tail -n1 $OUT/tracked.json

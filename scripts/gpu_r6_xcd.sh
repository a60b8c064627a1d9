#!/bin/bash
# Round 6: XCD-aware placement of the batched local-BA launches -- A/B of the
# default library against slam-1_amd/prof/libslam355_x0.so (-DSLAM_BA_XCD=0):
# the driver's bench, the 16-window BA line, and the FETCH_SIZE / WRITE_SIZE
# passes of the 16-window BA workload.   scripts/gpu_r6_xcd.sh TAG [ROUNDS] [trk]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd "$ROOT"
for i in $(seq 1 ${2:-2}); do
  for v in x0 def; do
    if [ $v = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
    timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit 1
    timeout -k 10 120 python3 bench.py --workload ba --ba-batch 16 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/b16_${v}_$i.json || exit 1
    python3 -c "import json;a=json.loads(open('$OUT/bench_${v}_$i.json').read().strip().splitlines()[-1]);b=json.load(open('$OUT/b16_${v}_$i.json'));print('$v', $i, 'bench', round(a['value']), round(a['stage_ms_per_step']['local_ba'],3), '| b16', round(b['value']), round(b['ms_per_step']*1e3,1))"
  done
done
# PMC workload: the 16-window BA line, or (third argument "trk") the driver's
# tracking bench as scripts/gpu_profile.sh runs it
if [ "$3" = trk ]; then
  PMC_ARGS="--no-cpu-baseline --no-ba-scale --no-pcie-leg --no-tracked-ba --no-tracked-leg --steps 3 --warmup 1"
else
  PMC_ARGS="--workload ba --ba-batch 16 --steps 5 --warmup 1"
fi
cd /tmp && export TMPDIR=/tmp
for v in x0 def; do
  if [ $v = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
  mkdir -p $OUT/pmc_$v
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/pmc_$v/$c -o run \
      -- python3 $ROOT/bench.py $PMC_ARGS > $OUT/pmc_$v/$c.log 2>&1 || exit 1
  done
  python3 $ROOT/scripts/pmc_summary.py $OUT/pmc_$v $OUT/pmc_$v.json > /dev/null || exit 1
  find $OUT/pmc_$v -name "*counter_collection.csv" -delete
  find $OUT/pmc_$v -name "*kernel_trace.csv" -delete
  python3 -c "
import json;d=json.load(open('$OUT/pmc_$v.json'))['kernels']
tot=0
for k in ('k_lin_mfma','k_assemble','k_solve_blk','k_back_trial'):
    v=sum(e['hbm_bytes'] for kk,e in d.items() if kk.split('<')[0]==k); tot+=v; print('$v', k, round(v/1e6,2), 'MB')
print('$v total', round(tot/1e6,2), 'MB')"
done

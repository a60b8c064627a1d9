#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/r4_fold
timeout -k 10 700 python -u -m pytest tests/test_ba.py tests/test_pipeline.py tests/test_dist.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_fold/pytest.log 2>&1 || { tail -40 gpurun_out/r4_fold/pytest.log; exit 1; }
tail -2 gpurun_out/r4_fold/pytest.log
bash scripts/gpu_r4_ab.sh r4_fold_ab 3 "" "--no-fold" || exit 1
for f in "" "--no-fold"; do
  timeout -k 10 120 python3 bench.py --workload ba --ba-batch 16 --steps 40 --warmup 5 $f 2>/dev/null | tail -1 > gpurun_out/r4_fold/b16$f.json || exit 1
  timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 $f 2>/dev/null | tail -1 > gpurun_out/r4_fold/c4$f.json || exit 1
  python3 -c "import json;a=json.load(open('gpurun_out/r4_fold/b16$f.json'));b=json.load(open('gpurun_out/r4_fold/c4$f.json'));print('fold' if '$f'=='' else 'nofold', 'b16', round(a['value']), round(a['ms_per_step']*1e3,1), 'c4', round(b['value']), round(b['ms_per_step']*1e3,1))"
done

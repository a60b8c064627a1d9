#!/bin/bash
# Round-4: the residency-free flow solve (BA + dist GPU tests), then the
# shard rehearsal script.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/r4_flow
timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_flow/pytest.log 2>&1 || { tail -40 gpurun_out/r4_flow/pytest.log; exit 1; }
tail -2 gpurun_out/r4_flow/pytest.log
timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 30 --warmup 5 > gpurun_out/r4_flow/c4.json 2>&1 || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r4_flow/c4.json'));print('c4', round(d['value']), d['ms_per_step'])"
bash scripts/gpu_r4_shards.sh

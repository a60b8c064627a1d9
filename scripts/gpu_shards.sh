set -o pipefail
# tracking shards of one sequence: GPU tests + the 1-rank and 2-rank (gloo, one GPU) rehearsals
mkdir -p gpurun_out/r4_q3
timeout -k 10 400 python -u -m pytest tests/test_dist.py -x -v -m gpu -k "shards_gather or gather_pose or capi_comm" --timeout 300 --timeout-method thread > gpurun_out/r4_q3/pytest.log 2>&1 || { tail -30 gpurun_out/r4_q3/pytest.log; exit 1; }
tail -2 gpurun_out/r4_q3/pytest.log
timeout -k 10 300 python3 bench.py --gpus 1 --batch 64 --steps 8 --warmup 2 --no-cpu-baseline --no-ba-scale --no-tracked-ba --no-pcie-leg > gpurun_out/r4_q3/g1.json 2> gpurun_out/r4_q3/g1.err || { tail gpurun_out/r4_q3/g1.err; exit 1; }
SLAM_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --batch 32 --steps 8 --warmup 2 --no-cpu-baseline --no-ba-scale --no-tracked-ba --no-pcie-leg > gpurun_out/r4_q3/g2.json 2> gpurun_out/r4_q3/g2.err || { tail gpurun_out/r4_q3/g2.err; exit 1; }
python3 -c "
import json
for f in ('g1','g2'):
  d=json.load(open(f'gpurun_out/r4_q3/{f}.json')); t=d['tracking']; print(f, d['n_gpus'], round(d['value']), t['trajectory_sha1'], t['frames_chained'], t['trajectory_t_err_m_max_from_frame0'])
"

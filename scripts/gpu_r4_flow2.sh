set -o pipefail
mkdir -p gpurun_out/r4_flow2
timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu -k "tiled or flow or c4 or c5 or distributed or capi" --timeout 300 --timeout-method thread > gpurun_out/r4_flow2/pytest.log 2>&1 || { tail -40 gpurun_out/r4_flow2/pytest.log; exit 1; }
tail -2 gpurun_out/r4_flow2/pytest.log
bash scripts/gpu_r4_ab_c4.sh r4_ab_c4_v2 slam-1_amd/prof/libslam355_oldflow.so

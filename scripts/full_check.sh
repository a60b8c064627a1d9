set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/pmc_traffic.sh r1p > gpurun_out/pmc_r1p.log 2>&1 && \
mkdir -p profiles && cp gpurun_out/pmc_traffic_r1p.json profiles/pmc_traffic.json && \
bash scripts/gpu_check.sh r1p

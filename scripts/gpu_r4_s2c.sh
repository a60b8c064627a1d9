#!/bin/bash
# Session-2 third pass: BA tests + C4 / C5 lines of the current library vs the
# round-4 HEAD library, flow-solve timeline; then a 4-way tracking A/B (current,
# HEAD matcher, matcher without the XCD order, PnP kernels at wave priority 3).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
bash scripts/gpu_r4_s2b.sh r4s2c_ba slam-1_amd/prof/libslam355_babase.so || exit 1
bash scripts/gpu_r4_abn.sh r4s2c_tr 3 def mxbase mxnoxcd pnpprio || exit 1
echo ok

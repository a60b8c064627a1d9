#!/bin/bash
# SQ instruction / stall counters for k_orb_tile (one pass per counter set).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/orbpmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d gpurun_out/orbpmc/p1 -o p1 --output-format csv -- python3 scripts/orb_run.py > gpurun_out/orbpmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH \
  -d gpurun_out/orbpmc/p2 -o p2 --output-format csv -- python3 scripts/orb_run.py > gpurun_out/orbpmc/p2.log 2>&1

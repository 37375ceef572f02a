#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02y
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export OVS_SKIP_BUILD=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
  -d gpurun_out/r02y/sq -o run -- python3 tools/diag/chord_shard_speed.py 2000000 > gpurun_out/r02y/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH -d gpurun_out/r02y/fetch -o run -- python3 tools/diag/chord_shard_speed.py 2000000 > gpurun_out/r02y/fetch.log 2>&1 || exit 2
echo done

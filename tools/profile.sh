#!/bin/bash
# Profile one bench workload on the GPU box: kernel trace + stats, then separate PMC passes
# (SQ stall breakdown; FETCH_SIZE; WRITE_SIZE), per MI355X_MICROARCH.md §rocprofv3.
# usage: tools/profile.sh <workload> <outdir> [extra bench args...]
set -e
W=$1; OUT=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
ARGS="--workload $W --steps 3 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d "$OUT/sq" -o run -- python3 bench.py $ARGS > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
echo profile-done

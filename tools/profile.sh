#!/bin/bash
# Profile one bench workload on the GPU box: kernel trace + stats, then separate PMC passes
# (SQ stall breakdown; FETCH_SIZE; WRITE_SIZE), per MI355X_MICROARCH.md §rocprofv3, and the
# summary (tools/prof_summary.py) + traffic JSON (tools/pmc_json.py) of the dominant kernel.
# usage: tools/profile.sh <workload> <outdir> <kernel substring> [extra bench args...]
set -e
W=$1; OUT=$2; K=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
ARGS="--workload $W --steps 5 --warmup 2 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1
echo "kt done $W"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d "$OUT/sq" -o run -- python3 bench.py $ARGS > "$OUT/sq.log" 2>&1
echo "sq done $W"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
python3 tools/prof_summary.py "$OUT" "$K" > "$OUT/summary.txt"
python3 tools/pmc_json.py "$OUT/summary.txt" "$K" "$W" "$OUT" > /dev/null
grep '^{' "$OUT/kt.log" | tail -1 > "$OUT/bench_under_kt.json" || true
# the raw rocprofv3 databases are large: keep only the summaries and logs
rm -rf "$OUT/kt" "$OUT/sq" "$OUT/fetch" "$OUT/write"
echo "profile done $W"

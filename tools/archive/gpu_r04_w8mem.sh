# round-4: FETCH / WRITE bytes of the W = 8 emulation of config C (K1 shard step, compaction)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc/fetch -o run -- python3 tools/diag/shard_w8_model.py --workload C > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc/write -o run -- python3 tools/diag/shard_w8_model.py --workload C > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 1; }
python tools/prof_summary.py $O/pmc k_chord_lanes > $O/pmc_mem.txt
python tools/prof_summary.py $O/pmc k_compact > $O/pmc_mem_compact.txt && rm -rf $O/pmc
grep -E "FETCH|WRITE" $O/pmc_mem.txt $O/pmc_mem_compact.txt | head -12

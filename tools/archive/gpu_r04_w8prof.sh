# round-4: kernel trace of the W = 8 emulation of config C (per-dispatch K1 shard-step times)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/ktW8C/kt -o run -- python3 tools/diag/shard_w8_model.py --workload C > $O/ktW8C.log 2>&1 || { tail -5 $O/ktW8C.log; exit 1; }
python tools/prof_summary.py $O/ktW8C k_chord_lanes > $O/ktW8C.txt && rm -rf $O/ktW8C
head -12 $O/ktW8C.txt
grep -A3 "dispatches" $O/ktW8C.txt | head -8

# round-4: where the W = 8 shard step loses time -- the same 2^23-node ring routed by the single
# route kernel, by the shard step at W = 1 (no hand-offs) and (the cost model) on eight arcs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29631
timeout -k 10 300 python -u bench.py --workload C --nodes 8388608 --no-cpu-baseline > $O/bench_C23_single.json 2> $O/bench_C23_single.err || { tail -20 $O/bench_C23_single.err; exit 1; }
OVS_BENCH_SHARD=1 timeout -k 10 300 python -u bench.py --workload C --nodes 8388608 --no-cpu-baseline > $O/bench_C23_shard.json 2> $O/bench_C23_shard.err || { tail -20 $O/bench_C23_shard.err; exit 1; }
for t in single shard; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], 'kernel %.3f ms' % d['roofline']['kernel_ms'], d['config'].get('mean_hops'), d['config'].get('hop_rounds'))" $O/bench_C23_$t.json $t; done
OVS_BENCH_SHARD=1 timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt23/kt -o run -- python3 bench.py --workload C --nodes 8388608 --no-cpu-baseline --steps 3 --warmup 1 > $O/kt23.log 2>&1 || { tail -5 $O/kt23.log; exit 1; }
python tools/prof_summary.py $O/kt23 k_chord_lanes > $O/kt23.txt && rm -rf $O/kt23
head -6 $O/kt23.txt; grep dispatches $O/kt23.txt
# lane census of the K1 launches (diagnostic build -DOVS_CHORD_STATS: wave iterations, lanes consuming a line)
OVS_LIB=$PWD/oversim_amd/libovs_kbr_k1stats.so timeout -k 10 300 python -u tools/diag/shard_w8_model.py --workload C > $O/w8_C_stats.jsonl 2> $O/w8_C_stats.err || { tail -20 $O/w8_C_stats.err; exit 1; }
OVS_LIB=$PWD/oversim_amd/libovs_kbr_k1stats.so timeout -k 10 300 python -u bench.py --workload C --no-cpu-baseline --steps 1 --warmup 0 > $O/bench_C_stats.json 2> $O/bench_C_stats.err || { tail -20 $O/bench_C_stats.err; exit 1; }
grep k1stats $O/w8_C_stats.err | head -12; grep k1stats $O/bench_C_stats.err | tail -1

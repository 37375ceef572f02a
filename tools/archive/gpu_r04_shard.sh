# sharded paths at W = 1 (OVS_BENCH_SHARD=1: the multi-GPU host path, collectives over RCCL at world 1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29631
for w in C E; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_${w}_single.json 2> $O/bench_${w}_single.err || { tail -20 $O/bench_${w}_single.err; exit 1; }
  OVS_BENCH_SHARD=1 timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_${w}_shard.json 2> $O/bench_${w}_shard.err || { tail -20 $O/bench_${w}_shard.err; exit 1; }
  for t in single shard; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], 'kernel %.3f ms' % d['roofline']['kernel_ms'], d['config'].get('hop_rounds'))" $O/bench_${w}_$t.json $w $t; done
done
OVS_BENCH_SHARD=1 timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/ktC/kt -o run -- python3 bench.py --workload C --no-cpu-baseline --steps 3 --warmup 1 > $O/ktC.log 2>&1 || { tail -5 $O/ktC.log; exit 1; }
python3 tools/prof_summary.py $O/ktC k_chord_lanes > $O/ktC.txt; rm -rf $O/ktC; head -30 $O/ktC.txt
OVS_BENCH_SHARD=1 timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/ktE/kt -o run -- python3 bench.py --workload E --no-cpu-baseline --steps 3 --warmup 1 > $O/ktE.log 2>&1 || { tail -5 $O/ktE.log; exit 1; }
python3 tools/prof_summary.py $O/ktE k_kad_route > $O/ktE.txt; rm -rf $O/ktE; head -30 $O/ktE.txt

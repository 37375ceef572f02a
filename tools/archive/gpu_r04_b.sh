# round-4: shard suites + KademliaLarge on arcs, refresh suites, bench R / E / B, W = 1 sharded bench, W = 8 model (E)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_shard.py tests/test_gpu_kad_large.py tests/test_gpu_kad_refresh.py tests/test_gpu_kad_maint.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for w in R E B; do timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], 'kernel %.3f' % d['roofline']['kernel_ms'])" $O/bench_$w.json $w; done
bash tools/gpu_r04_shard.sh $1 > $O/shard_w1.txt 2>&1 || { tail -20 $O/shard_w1.txt; exit 1; }
grep -E "^C |^E " $O/shard_w1.txt
timeout -k 10 600 python -u tools/diag/shard_w8_model.py --workload E > $O/w8_E.jsonl 2> $O/w8_E.err || { tail -20 $O/w8_E.err; exit 1; }
tail -2 $O/w8_E.jsonl

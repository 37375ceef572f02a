set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_b_alpha; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_kad.py tests/test_gpu_kad_refresh.py tests/test_gpu_lookupcall.py tests/test_shard.py -m gpu -x -v --timeout 300 --timeout-method thread -k "kad or Kad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for w in B E; do timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }; cat $O/bench_$w.json; done

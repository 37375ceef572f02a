# Kademlia GPU check: the Kademlia parity files, then bench lines for B and E.
# usage: bash tools/gpu_kad.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kad.py tests/test_gpu_kad_tables.py tests/test_gpu_lookupcall.py tests/test_gpu_timed.py tests/test_shard.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for w in B E; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done

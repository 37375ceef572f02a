# Round 5: GPU parity suite (optionally a -k filter), then bench lines WITH the CPU baseline and the
# bench's own parity check for the named workloads.
# usage: bash tools/gpu_r05_check.sh <outdir> "<pytest -k expr or ''>" [workloads...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
K="$1"; shift
export OVS_SKIP_BUILD=1
if [ "$K" != "none" ]; then
  if [ -n "$K" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  else
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  fi
  tail -2 $O/gpu_tests.log
fi
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done

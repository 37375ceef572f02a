# GPU parity tests for a subset (pytest -k / file args), then optional bench lines.
# usage: bash tools/gpu_tests.sh <outdir> "<pytest selectors>" [workloads...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; T=$2; shift 2; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done

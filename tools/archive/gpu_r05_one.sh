# Round 5: a pytest -k selection on the GPU, then an optional command (e.g. a model run).
# usage: bash tools/gpu_r05_one.sh <outdir> "<-k expr>" [cmd...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
K="$1"; shift
export OVS_SKIP_BUILD=1
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
if [ $# -gt 0 ]; then
  timeout -k 10 600 "$@" > $O/cmd.out 2> $O/cmd.err || { tail -30 $O/cmd.err; tail -5 $O/cmd.out; exit 1; }
  tail -8 $O/cmd.out
fi

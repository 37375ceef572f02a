# round 6: a pytest -k selection on the GPU, then optionally the N > 1 rehearsal of some workloads.
# usage: bash tools/gpu_r06_tests.sh <outdir> "<-k expr>" [rehearsal workloads...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=$1; O=gpurun_out/$1; shift; mkdir -p $O
K="$1"; shift
export OVS_SKIP_BUILD=1
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
if [ $# -gt 0 ]; then
  bash tools/gpu_r06_rehearse.sh $D/rehearse "$@" || exit 1
fi

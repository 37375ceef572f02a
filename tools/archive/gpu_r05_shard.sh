# Round 5: the sharded-path tests (native round loop, replicated top levels, C consumers, ADVICE
# fixes), then the W = 8 cost model of config C with the default replicated levels.
# usage: bash tools/gpu_r05_shard.sh <outdir> [model-args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread \
  -k "native or c_consumer or emulated or failed_rebuild or capacity_change or cohorts or two_processes" \
  > $O/shard_tests.log 2>&1 || { tail -40 $O/shard_tests.log; exit 1; }
tail -3 $O/shard_tests.log
timeout -k 10 600 python -u tools/diag/shard_w8_model.py --workload C "$@" > $O/w8_C.jsonl 2> $O/w8_C.err || { tail -20 $O/w8_C.err; exit 1; }
tail -4 $O/w8_C.jsonl

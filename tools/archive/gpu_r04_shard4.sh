# round-4: shard suites (incl. KademliaLarge on arcs), W = 1 bench of the sharded paths, W = 8 cost model (E)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_shard.py tests/test_gpu_kad_large.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/shard_tests.log 2>&1 || { tail -40 $O/shard_tests.log; exit 1; }
tail -3 $O/shard_tests.log
bash tools/gpu_r04_shard.sh $1 || exit 1
timeout -k 10 600 python -u tools/diag/shard_w8_model.py --workload E > $O/w8_E.jsonl 2> $O/w8_E.err || { tail -20 $O/w8_E.err; exit 1; }
tail -3 $O/w8_E.jsonl

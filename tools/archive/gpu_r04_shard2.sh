# round-4: sharded Kademlia without the round-1 state records, the step at 3 waves; shard suites + W = 1 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_shard.py tests/test_gpu_shard_full.py tests/test_gpu_kad_large.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/shard_tests.log 2>&1 || { tail -40 $O/shard_tests.log; exit 1; }
tail -3 $O/shard_tests.log
bash tools/gpu_r04_shard.sh $1

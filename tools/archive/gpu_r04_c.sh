# round-4: Chord shard suites with the key-started first round, W = 1 bench of the sharded paths
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_shard.py tests/test_gpu_chord.py tests/test_gpu_lookupcall.py tests/test_gpu_shard_full.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/gpu_r04_shard.sh $1 > $O/shard_w1.txt 2>&1 || { tail -20 $O/shard_w1.txt; exit 1; }
grep -E "^C |^E " $O/shard_w1.txt

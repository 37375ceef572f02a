# round-4: single-entry findNode blocks by insertion (A/B against the sort + merge build), Kademlia
# GPU suites, then the W = 8 cost model of config C
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
bash tools/gpu_ab.sh $1 "R E B" noins || exit 1
bash tools/gpu_ab.sh $1/rep "R E B" noins || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_kad.py tests/test_gpu_kad_refresh.py tests/test_gpu_kad_large.py tests/test_gpu_timed.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python -u tools/diag/shard_w8_model.py --workload C > $O/w8_C.jsonl 2> $O/w8_C.err || { tail -20 $O/w8_C.err; tail -5 $O/w8_C.jsonl; exit 1; }
tail -2 $O/w8_C.jsonl

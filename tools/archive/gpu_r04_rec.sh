# round-4: R/Kademlia (recursive routes and LookupCalls) parity, K2g, the K2 regression set
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_kad_recursive.py tests/test_gpu_kad_general.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/rec.log 2>&1 || { tail -60 $O/rec.log; exit 1; }
tail -3 $O/rec.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_kad.py tests/test_gpu_kad_tables.py tests/test_gpu_lookupcall.py tests/test_gpu_chord.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log

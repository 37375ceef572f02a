# round-4: preloaded sources at refill (K1: no PH_FETCH iteration; K2: no dependent source load in
# the refill iteration) -- Chord and Kademlia suites, A/B against builds without (nopre: neither,
# kadnopre: K1 preload only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_chord.py tests/test_gpu_lookupcall.py tests/test_gpu_timed.py tests/test_shard.py tests/test_gpu_c_consumer.py tests/test_gpu_kad.py tests/test_gpu_kad_large.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh $1 "C E B" nopre kadnopre || exit 1
bash tools/gpu_ab.sh $1/rep "C E B" nopre kadnopre || exit 1

# round-4: preloaded sources in K3 (Koorde) and K2x (refresh) -- suites, A/B against builds without
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_koorde.py tests/test_gpu_kad_refresh.py tests/test_gpu_kad_maint.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh $1 "K R" k3nopre kxnopre || exit 1
bash tools/gpu_ab.sh $1/rep "K R" k3nopre kxnopre || exit 1

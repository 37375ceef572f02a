# round-4: K2x keeps an unrequested responder list's first 32 entries in LDS -- suites, A/B, WRITE_SIZE
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_kad_refresh.py tests/test_gpu_kad_maint.py tests/test_gpu_kad.py tests/test_gpu_kad_large.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh $1 "R" kxnolvis || exit 1
bash tools/gpu_ab.sh $1/rep "R" kxnolvis || exit 1
timeout -k 10 600 bash tools/profile.sh R $O/R k_kad_refresh || exit 1
grep -E "FETCH|WRITE|mean of the last" $O/R/summary.txt | cut -c90-

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench_C.json 2> $O/bench_C.err && \
bash tools/profile.sh C $O/profC && python tools/prof_summary.py $O/profC k_chord_route > $O/profC.txt

# round-4: K3 reads a responder's successor codes (line 1) only when its walk needs them
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_koorde.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload K --no-cpu-baseline > $O/bench_K_$rep.json 2> $O/bench_K_$rep.err || { tail -20 $O/bench_K_$rep.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('K', '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'])" $O/bench_K_$rep.json
done
timeout -k 10 600 bash tools/profile.sh K $O/K k_koorde_route || exit 1
grep -E "FETCH|WRITE|mean of the last|# resources" -A0 $O/K/summary.txt | cut -c100-

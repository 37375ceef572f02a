# round-4: K2x internal visited lists in the context's cached buffer (no per-call hipMalloc / hipFree)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_kad_refresh.py tests/test_gpu_kad_maint.py tests/test_gpu_koorde.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline > $O/bench_R_$rep.json 2> $O/bench_R_$rep.err || { tail -20 $O/bench_R_$rep.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('R', '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], 'kernel %.3f ms' % d['roofline']['kernel_ms'])" $O/bench_R_$rep.json
done

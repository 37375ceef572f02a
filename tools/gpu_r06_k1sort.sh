# round 6: K1 key order A/B -- bench C with the in-step counting sort off / 12 / 14
# bits, then the key-order parity test.  usage: bash tools/gpu_r06_k1sort.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
for v in off 12 14 off2; do
  case $v in off|off2) export OVS_K1_SORT=0 ;; *) export OVS_K1_SORT=1 OVS_K1_SORT_BITS=$v ;; esac
  timeout -k 10 300 python3 -u bench.py --workload C --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.4g' % d['value'], '%.4f ms' % d['ms_per_step'], 'kernel %.4f' % d['roofline']['kernel_ms'])" $O/bench_$v.json $v
done
unset OVS_K1_SORT OVS_K1_SORT_BITS
timeout -k 10 300 python -u -m pytest tests/test_gpu_chord.py -m gpu -x -v --timeout 170 --timeout-method thread -k key_order > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log

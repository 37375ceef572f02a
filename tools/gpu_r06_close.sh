# round 6 closing check on the final tree.  usage: bash tools/gpu_r06_close.sh <outdir> tests|bench [workloads...]
#   tests: the whole GPU suite (as the driver runs it) and __graft_entry__.smoke()
#   bench: one bench line per workload (each with its CPU baseline and parity check), then the
#          profiles (kernel trace + SQ + FETCH/WRITE passes) of C and E (tools/profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; MODE=$2; shift 2; mkdir -p $O
export OVS_SKIP_BUILD=1
if [ $MODE = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  tail -3 $O/smoke.log
else
  for w in ${*:-C A B D E K R}; do
    timeout -k 10 600 python3 -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d.get('parity') or {}
print(sys.argv[2], '%.4g' % d['value'], d['unit'], '%.3f ms' % d['ms_per_step'], 'frac', d['roofline']['frac'], 'parity', p.get('checked'), p.get('mismatches'))" $O/bench_$w.json $w
  done
  if [ "${PROF:-1}" = 1 ]; then
    timeout -k 10 600 bash tools/profile.sh C $O/prof_C k_chord_lanes || exit 1
    timeout -k 10 600 bash tools/profile.sh E $O/prof_E k_kad_route || exit 1
  fi
fi

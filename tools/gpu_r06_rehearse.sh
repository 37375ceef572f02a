# round 6: the bench's N > 1 path end to end on one GPU -- 2 and 4 ranks as separate processes sharing
# cuda:0, exchanges over gloo (RCCL cannot put two ranks on one device).  Each line must carry the
# sharded parity check (every rank checks the done records it holds of a sample against the oracle):
# parity.mismatches == 0 and checked == expected.  Not a scaling measurement.
# usage: bash tools/gpu_r06_rehearse.sh <outdir> [workloads (default C D E)]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
WLS="${*:-C D E}"
export OVS_SKIP_BUILD=1 OVS_BENCH_BACKEND=gloo
# a heartbeat file while the runs go (each run has its own time limit and bench.py its stage watchdog)
( while sleep 30; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for n in 2 4; do
  for w in $WLS; do
    extra=""
    [ $w = D ] && extra="--lookups 2000000"
    timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2963$n bench.py --gpus $n --workload $w --no-cpu-baseline --steps 3 --warmup 1 $extra > $O/bench_${w}_n$n.json 2> $O/bench_${w}_n$n.err || { tail -30 $O/bench_${w}_n$n.err; exit 1; }
    python -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['parity'] or {}
print(sys.argv[2], sys.argv[3], '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], d['config'].get('hop_rounds'), 'parity', p.get('checked'), '/', p.get('expected'), 'mismatches', p.get('mismatches'))
sys.exit(0 if p and p['mismatches'] == 0 and p['checked'] == p['expected'] else 1)" $O/bench_${w}_n$n.json $w $n || exit 1
  done
done

# round-5: the bench's N > 1 path end to end on one GPU -- 2 and 4 ranks as separate processes
# sharing cuda:0, exchanges over gloo (RCCL cannot put two ranks on one device): the JSON line,
# per-rank step times and the sharded results' completeness check, not a scaling measurement
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1 OVS_BENCH_BACKEND=gloo
for n in 2 4; do
  for w in C E; do
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2963$n bench.py --gpus $n --workload $w --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_${w}_n$n.json 2> $O/bench_${w}_n$n.err || { tail -30 $O/bench_${w}_n$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], d['n_gpus'], d['config'].get('parallelism'), d['config'].get('hop_rounds'))" $O/bench_${w}_n$n.json $w $n
  done
done

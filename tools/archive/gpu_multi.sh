# N-rank rehearsal of bench.py on ONE GPU (gloo exchange through host memory; correctness of the
# N > 1 path, not a performance number).  usage: bash tools/gpu_multi.sh <outdir> <nranks> [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; N=$2; shift 2; mkdir -p $O
export OVS_SKIP_BUILD=1 OVS_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $N "$@" > $O/multi_$N.json 2> $O/multi_$N.err || { tail -30 $O/multi_$N.err; exit 1; }
grep metric $O/multi_$N.json

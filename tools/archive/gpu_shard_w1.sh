# The sharded host path under RCCL at world size 1 (torch.distributed.run, backend nccl): the
# count all-gather, the exchange bookkeeping and the cohort streams run as on N GPUs.
# usage: bash tools/gpu_shard_w1.sh <outdir> [workloads...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1 OVS_BENCH_SHARD=1
for w in ${@:-C E}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --workload $w --no-cpu-baseline > $O/bench_shard_$w.json 2> $O/bench_shard_$w.err \
      || { tail -30 $O/bench_shard_$w.err; exit 1; }
  cat $O/bench_shard_$w.json
done

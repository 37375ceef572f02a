# A/B of the sharded host path at world size 1 (RCCL) across engine builds.
# usage: bash tools/gpu_shard_ab.sh <outdir> <workload> [tags...]   (main = in-tree library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; W=$2; shift 2; mkdir -p $O
export OVS_SKIP_BUILD=1 OVS_BENCH_SHARD=1
for tag in main "$@"; do
  if [ $tag = main ]; then unset OVS_LIB; else export OVS_LIB=$PWD/oversim_amd/libovs_kbr_$tag.so; fi
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29513 bench.py --workload $W --no-cpu-baseline > $O/shard_${W}_$tag.json 2> $O/shard_${W}_$tag.err \
      || { tail -20 $O/shard_${W}_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], 'kernel %.3f' % d['roofline']['kernel_ms'])" $O/shard_${W}_$tag.json $tag
done

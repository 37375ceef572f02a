# round-4: sharded Kademlia step cost experiments at W = 1 (config E): main vs alternative libraries
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29633
for tag in main "$@"; do
  if [ $tag = main ]; then export OVS_LIB=$PWD/oversim_amd/libovs_kbr.so; else export OVS_LIB=$PWD/oversim_amd/libovs_kbr_$tag.so; fi
  OVS_BENCH_SHARD=1 timeout -k 10 300 python -u bench.py --workload E --no-cpu-baseline > $O/E_$tag.json 2> $O/E_$tag.err || { tail -20 $O/E_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], 'kernel %.3f' % d['roofline']['kernel_ms'])" $O/E_$tag.json $tag
done

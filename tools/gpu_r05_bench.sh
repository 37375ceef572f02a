# Round 5: the driver's default bench line (C, with the oracle parity check and CPU baseline), then
# the RCCL > 1 GB probe.  usage: bash tools/gpu_r05_bench.sh <outdir> [workloads...] [rccl]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1
for w in "$@"; do
  if [ $w = rccl ]; then
    timeout -k 10 300 python3 -u tools/diag/rccl_big.py ${RCCL_ARGS:-} > $O/rccl.out 2> $O/rccl.err || { tail -20 $O/rccl.err; exit 1; }
    cat $O/rccl.out
  else
    timeout -k 10 600 python3 -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
    cut -c1-1500 $O/bench_$w.json
  fi
done
# k1stats: bench C on the OVS_CHORD_STATS library -- K1's lines by kind (the per-launch line census)
if [ "${K1STATS:-0}" = 1 ]; then
  OVS_LIB=$PWD/oversim_amd/libovs_kbr_k1stats.so timeout -k 10 300 python3 -u bench.py --workload C --steps 1 --warmup 0 --no-cpu-baseline > $O/k1stats_C.json 2> $O/k1stats_C.err || { tail -5 $O/k1stats_C.err; exit 1; }
  grep k1stats $O/k1stats_C.err | tail -2
fi

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
# k1stats: bench C on the OVS_CHORD_STATS library -- K1's lines by kind (the per-launch line census;
# built by tools/build_alt_src.sh k1stats chord.hip -DOVS_CHORD_STATS)
if [ "${K1STATS:-0}" = 1 ]; then
  OVS_LIB=$PWD/oversim_amd/libovs_kbr_k1stats.so timeout -k 10 300 python3 -u bench.py --workload C --steps 1 --warmup 0 --no-cpu-baseline > $O/k1stats_C.json 2> $O/k1stats_C.err || { tail -5 $O/k1stats_C.err; exit 1; }
  grep k1stats $O/k1stats_C.err | tail -2
fi
# kxstats: bench R on the OVS_KX_STATS library -- K2x's reads and writes by kind per launch
# (tools/build_alt_src.sh kxstats kad_refresh.hip -DOVS_KX_STATS)
if [ "${KXSTATS:-0}" = 1 ]; then
  OVS_LIB=$PWD/oversim_amd/libovs_kbr_kxstats.so timeout -k 10 300 python3 -u bench.py --workload R --steps 1 --warmup 0 --no-cpu-baseline > $O/kxstats_R.json 2> $O/kxstats_R.err || { tail -5 $O/kxstats_R.err; exit 1; }
  grep kxstats $O/kxstats_R.err | tail -2
fi
# ab: bench lines of each workload in ABW on the in-tree library and on each libovs_kbr_<tag>.so in AB
for tag in ${AB:-}; do
  for w in ${ABW:-R}; do
    if [ $tag = main ]; then L=$PWD/oversim_amd/libovs_kbr.so; else L=$PWD/oversim_amd/libovs_kbr_$tag.so; fi
    OVS_LIB=$L timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline > $O/ab_${tag}_$w.json 2> $O/ab_${tag}_$w.err || { tail -5 $O/ab_${tag}_$w.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" $O/ab_${tag}_$w.json $tag $w
  done
done

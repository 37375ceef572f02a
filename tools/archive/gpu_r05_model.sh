# Round 5: rocprof of the Kademlia table build at 2^24, then the W = 8 cost models (C; E with migration).
# usage: bash tools/gpu_r05_model.sh <outdir> [C] [E] [profC] [profE] [build]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1
for w in "$@"; do
  case $w in
    build)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/build -o b -- python3 -u tools/diag/kad_build_time.py --reps 2 > $O/build.out 2>&1 || { tail -20 $O/build.out; exit 1; }
      tail -4 $O/build.out ;;
    profC|profE)
      w2=${w#prof}; extra=""; [ $w2 = E ] && extra="--mig"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/$w -o k -- python3 -u tools/diag/shard_w8_model.py --workload $w2 $extra > $O/$w.out 2>&1 || { tail -20 $O/$w.out; exit 1; }
      grep summary $O/$w.out | cut -c1-400 ;;
    C|E)
      extra=""; [ $w = E ] && extra="--mig"
      timeout -k 10 600 python3 -u tools/diag/shard_w8_model.py --workload $w $extra > $O/w8$w.out 2> $O/w8$w.err || { tail -20 $O/w8$w.err; exit 1; }
      tail -6 $O/w8$w.out ;;
  esac
done
# k1stats: the W = 8 and W = 1 C models on the OVS_CHORD_STATS library (lines by kind per K1 launch)
if [ "${K1STATS:-0}" = 1 ]; then
  for W in 8 1; do
    OVS_LIB=$PWD/oversim_amd/libovs_kbr_k1stats.so timeout -k 10 600 python3 -u tools/diag/shard_w8_model.py --workload C --world $W > $O/k1s_w$W.out 2> $O/k1s_w$W.err || { tail -20 $O/k1s_w$W.err; exit 1; }
    grep -c k1stats $O/k1s_w$W.err
  done
fi
# ab: the C model on the in-tree library and on each oversim_amd/libovs_kbr_<tag>.so named in AB
for tag in ${AB:-}; do
  OVS_LIB=$PWD/oversim_amd/libovs_kbr_$tag.so timeout -k 10 600 python3 -u tools/diag/shard_w8_model.py --workload C > $O/ab_$tag.out 2> $O/ab_$tag.err || { tail -20 $O/ab_$tag.err; exit 1; }
  echo "$tag: $(grep summary $O/ab_$tag.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(max(d["step_ms_per_rank"]), d["rounds"])')"
done
# buildab: the 2^24 Kademlia build on each oversim_amd/libovs_kbr_<tag>.so named in BUILDAB (kernel trace)
for tag in ${BUILDAB:-}; do
  if [ $tag = main ]; then L=$PWD/oversim_amd/libovs_kbr.so; else L=$PWD/oversim_amd/libovs_kbr_$tag.so; fi
  OVS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/build_$tag -o b -- python3 -u tools/diag/kad_build_time.py --reps 2 > $O/build_$tag.out 2>&1 || { tail -20 $O/build_$tag.out; exit 1; }
  grep tables_sha $O/build_$tag.out
done
# buildpmc: kernel trace + SQ / FETCH / WRITE passes of the 2^24 Kademlia build (summary.txt)
if [ "${BUILDPMC:-0}" = 1 ]; then
  P=$O/buildpmc; mkdir -p $P
  A="tools/diag/kad_build_time.py --reps 1 --check-nodes 4096"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/kt -o run -- python3 -u $A > $P/kt.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $P/sq -o run -- python3 -u $A > $P/sq.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- python3 -u $A > $P/fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run -- python3 -u $A > $P/write.log 2>&1
  python3 tools/prof_summary.py $P k_kad > $P/summary.txt
  rm -rf $P/kt $P/sq $P/fetch $P/write
  grep -E "bucket_rows|sib_rows|k_kad_siblings" $P/summary.txt | cut -c1-200
fi
# toplev: the C model at each replicated-level count in TOPLEV
for L in ${TOPLEV:-}; do
  timeout -k 10 600 python3 -u tools/diag/shard_w8_model.py --workload C --top-levels $L > $O/c_top$L.out 2> $O/c_top$L.err || { tail -20 $O/c_top$L.err; exit 1; }
  echo "top $L: $(grep summary $O/c_top$L.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(max(d["step_ms_per_rank"]), d["rounds"])')"
done
# cpmc: SQ counters of the C model's kernels (the shard step K1 against the single-context check route)
if [ "${CPMC:-0}" = 1 ]; then
  P=$O/cpmc; mkdir -p $P
  timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $P/sq -o run -- python3 -u tools/diag/shard_w8_model.py --workload C > $P/sq.log 2>&1
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- python3 -u tools/diag/shard_w8_model.py --workload C > $P/fetch.log 2>&1
  python3 tools/prof_summary.py $P k_chord_lanes > $P/summary.txt
  rm -rf $P/sq $P/fetch
  grep -E "k_chord_lanes" $P/summary.txt | cut -c1-220
fi

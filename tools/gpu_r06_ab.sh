# round 6: bench A/B -- each workload in ABW on the in-tree library and on each libovs_kbr_<tag>.so
# named, interleaved, REPS times.  usage: ABW="B E" bash tools/gpu_r06_ab.sh <outdir> <tag>...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1
for rep in $(seq ${REPS:-2}); do
  for tag in main "$@"; do
    for w in ${ABW:-B E}; do
      if [ $tag = main ]; then L=$PWD/oversim_amd/libovs_kbr.so; else L=$PWD/oversim_amd/libovs_kbr_$tag.so; fi
      OVS_LIB=$L timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline ${ABARGS:-} > $O/ab_${tag}_${w}_$rep.json 2> $O/ab_${tag}_${w}_$rep.err || { tail -5 $O/ab_${tag}_${w}_$rep.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); p=d.get('parity') or {}; print(sys.argv[2], sys.argv[3], sys.argv[4], '%.4g' % d['value'], '%.4f' % d['ms_per_step'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'parity', p.get('checked'), p.get('mismatches'))" $O/ab_${tag}_${w}_$rep.json $tag $w $rep
    done
  done
done

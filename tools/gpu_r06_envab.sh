# round 6: bench A/B of the in-tree library under two environments (e.g. the dynamic tail on and
# OVS_NO_DYN=1), interleaved, REPS times.  usage: ABW="C D" bash tools/gpu_r06_envab.sh <outdir> "<env A>" "<env B>"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1
for rep in $(seq ${REPS:-2}); do
  i=0
  for envs in "$@"; do
    i=$((i + 1))
    for w in ${ABW:-C D}; do
      env $envs OVS_AB_TAG=$i timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline ${ABARGS:-} > $O/ab_${i}_${w}_$rep.json 2> $O/ab_${i}_${w}_$rep.err || { tail -5 $O/ab_${i}_${w}_$rep.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); p=d.get('parity') or {}; print(sys.argv[2], sys.argv[3], sys.argv[4], '%.4g' % d['value'], '%.4f' % d['ms_per_step'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'parity', p.get('checked'), p.get('mismatches'))" $O/ab_${i}_${w}_$rep.json "[$envs]" $w $rep
    done
  done
done

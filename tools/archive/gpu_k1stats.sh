# K1 line accounting (diagnostic build oversim_amd/libovs_kbr_k1stats.so, -DOVS_CHORD_STATS): the
# lines each K1 launch consumes by kind, for workloads C and D.  usage: bash tools/gpu_k1stats.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
for w in C D; do
  OVS_LIB=$PWD/oversim_amd/libovs_kbr_k1stats.so timeout -k 10 300 python -u bench.py --workload $w --steps 1 --warmup 0 \
      --no-cpu-baseline > $O/k1stats_$w.json 2> $O/k1stats_$w.err || { tail -5 $O/k1stats_$w.err; exit 1; }
  grep k1stats $O/k1stats_$w.err | tail -1
  python -c "import json; d=json.load(open('$O/k1stats_$w.json')); print('$w hops/launch', d['config']['mean_hops']*d['config']['lookups_per_gpu'])"
done

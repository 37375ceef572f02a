# A/B bench of alternative engine builds (tools/build_alt.sh) against the in-tree one.
# usage: bash tools/gpu_ab.sh <outdir> "<workloads>" [tags...]   ("" tag = in-tree library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; W=$2; shift 2; mkdir -p $O
export OVS_SKIP_BUILD=1
for tag in main "$@"; do
  for w in $W; do
    if [ $tag = main ]; then export OVS_LIB=$PWD/oversim_amd/libovs_kbr.so; else export OVS_LIB=$PWD/oversim_amd/libovs_kbr_$tag.so; fi
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_${w}_$tag.json 2> $O/bench_${w}_$tag.err || { tail -20 $O/bench_${w}_$tag.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], '%.4g' % d['value'], d['unit'], '%.3f ms' % d['ms_per_step'])" $O/bench_${w}_$tag.json $w $tag
  done
done

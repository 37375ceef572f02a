# Bench each build/var/<name> variant on the given workloads (value + kernel time only).
# usage: bash tools/gpu_variants.sh <outdir> "<variants>" [workloads...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; V=$2; shift 2; mkdir -p $O
export OVS_SKIP_BUILD=1
for w in "$@"; do
  for v in $V; do
    L=build/var/$v/libovs_kbr.so; [ "$v" = main ] && L=oversim_amd/libovs_kbr.so
    OVS_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/$v.$w.json 2> $O/$v.$w.err || { tail -5 $O/$v.$w.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$v.$w.json')); print('$v','$w', '%.4g'%d['value'], 'kernel_ms %.3f'%d['roofline']['kernel_ms'])"
  done
done

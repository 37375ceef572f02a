# Repeated bench lines for the named workloads (noise check): bash tools/gpu_rep.sh <reps> <workloads...>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; export OVS_SKIP_BUILD=1
R=$1; shift
for w in "$@"; do
  for i in $(seq 1 $R); do
    timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])" || exit 1
  done
done

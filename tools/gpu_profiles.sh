# Profiles (kernel trace + SQ + FETCH/WRITE passes) of the named workloads at HEAD, one directory
# per workload under gpurun_out/<outdir>.  usage: bash tools/gpu_profiles.sh <outdir> <workload:kernel>...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$1; shift
export OVS_SKIP_BUILD=1
for wk in "$@"; do
  w=${wk%%:*}; k=${wk#*:}
  timeout -k 10 600 bash tools/profile.sh $w gpurun_out/$O/$w $k || exit 1
  cat gpurun_out/$O/$w/bench_under_kt.json
done

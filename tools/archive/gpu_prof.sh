# Profile bench workloads: kernel trace + SQ/FETCH/WRITE PMC passes (tools/profile.sh), summarised.
# usage: bash tools/gpu_prof.sh <outdir> <kernel-substring> [workloads...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; K=$2; shift 2; mkdir -p $O
export OVS_SKIP_BUILD=1
for w in "$@"; do
  bash tools/profile.sh $w $O/prof$w && python tools/prof_summary.py $O/prof$w $K > $O/prof$w.txt || exit 1
  for p in kt sq fetch write; do tail -3 $O/prof$w/$p.log > $O/prof$w.$p.log; done
  rm -rf $O/prof$w
done
echo prof-done

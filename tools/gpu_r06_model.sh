# round 6: the W = 8 cost models (tools/diag/shard_w8_model.py, eight arcs emulated on one GPU, every
# lookup checked against the single-context route): C (2^23 ring), D (2^25: eight emulated arcs of the
# 2^26 ring do not fit one GPU's 288 GB), E (2^24, migrating lookups).
# usage: bash tools/gpu_r06_model.sh <outdir> [C] [D] [E]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1
for w in "$@"; do
  extra=""
  [ $w = E ] && extra="--mig"
  [ $w = D ] && extra="--nodes 33554432"
  timeout -k 10 900 python3 -u tools/diag/shard_w8_model.py --workload $w $extra > $O/w8$w.out 2> $O/w8$w.err || { tail -20 $O/w8$w.err; exit 1; }
  tail -3 $O/w8$w.out | cut -c1-600
done

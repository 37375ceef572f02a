# round-4: oversubscribed grids for K2 / K2x (2x, 4x waves per resident slot, shorter slices) A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
bash tools/gpu_ab.sh $1 "B E R" os2 os4 || exit 1
bash tools/gpu_ab.sh $1/rep "B E R" os2 os4 || exit 1

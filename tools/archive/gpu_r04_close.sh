# round-4 closing run: full GPU suite, smoke, bench lines with CPU baselines, then the kernel trace +
# SQ + FETCH/WRITE profiles of C and R (the kernels changed since r04_prof)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh $1 || exit 1
bash tools/gpu_profiles.sh $1_prof C:k_chord_lanes R:k_kad_refresh || exit 1

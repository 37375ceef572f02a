# Run GPU steps in order; a step that fails its assertions (pytest exit 1) does not stop the
# rest, anything else (a crash, an abort, a time limit) ends the call there.
# usage: bash tools/gpu_steps.sh '<step 1>' '<step 2>' ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export OVS_SKIP_BUILD=1
for step in "$@"; do
  echo "== $step"
  bash -c "$step"
  rc=$?
  echo "== rc $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

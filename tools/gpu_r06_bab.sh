# round 6: Kademlia snapshot build A/B at 2^24 -- kernel trace of tools/diag/kad_build_time.py for the
# in-tree library (packed bucket rows, one-pass node summary, two streams), the same with one stream
# (OVS_KB_SERIAL=1) and an alternative library (the round-5 kernels); the tables checksum must agree.
# usage: bash tools/gpu_r06_bab.sh <outdir> [alt library ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export OVS_SKIP_BUILD=1
CMD="python3 tools/diag/kad_build_time.py --reps 3"
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$tag -o run -- $CMD > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  grep '^{' $O/$tag.log
  python3 tools/prof_summary.py $O/kt_$tag > /dev/null 2>&1
  python3 - $O/kt_$tag/run_results.db $tag <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
big = [r for r in rows if 'k_kad_' in r[0] or 'onesweep' in r[0] or 'scan' in r[0].lower()]
# the builds of the 2^24 network: group dispatches between consecutive k_kad_tops launches
starts = [i for i, r in enumerate(rows) if 'k_kad_tops' in r[0]]
for j, s in enumerate(starts[:-1]):
    grp = rows[s:starts[j + 1]]
    span = (max(r[2] for r in grp) - grp[0][1]) * 1e-6
    ks = {}
    for n, a, b in grp:
        if 'k_kad_' in n:
            k = n.split('(')[0].split('::')[-1]
            ks[k] = ks.get(k, 0) + (b - a) * 1e-6
    print(sys.argv[2], 'build', j, 'span_ms %.2f' % span, 'kernels_ms %.2f' % sum(ks.values()),
          ' '.join('%s=%.2f' % (k, v) for k, v in sorted(ks.items(), key=lambda x: -x[1])))
PY
  rm -rf $O/kt_$tag
}
run main

for L in "$@"; do run $(basename $L .so) OVS_LIB=$PWD/$L; done

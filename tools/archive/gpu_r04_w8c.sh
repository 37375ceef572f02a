# round-4: W = 8 cost model of config C (Chord, 2^23 nodes on eight emulated arcs, 10M lookups per arc)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 900 python -u tools/diag/shard_w8_model.py --workload C > $O/w8_C.jsonl 2> $O/w8_C.err || { tail -20 $O/w8_C.err; tail -5 $O/w8_C.jsonl; exit 1; }
tail -2 $O/w8_C.jsonl
